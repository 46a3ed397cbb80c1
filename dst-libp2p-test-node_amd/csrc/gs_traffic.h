// gs_traffic.h — per-peer traffic of a finished batch (gs_set_traffic).
// Included by gs_relax.hip only (inside namespace gs::{anon}), after
// gs_relax_kernel.h.
//
// Every send of the batch is a function of the final keys:
//  * publish: the publisher's flood (or mesh) sends, fragment after fragment
//    through its uplink (k_traffic_pub, mirrors k_seed);
//  * forward: the first receipt of (m, f) at u sends one copy to each of
//    mesh(u) \ {src, publisher} minus the IDONTWANT skips, through u's uplink
//    FIFO (k_traffic_fwd, mirrors relax_lane; the FIFO start of a fragment is
//    re-folded over the group's final keys);
//  * lazy gossip: every holder of (m, f) sends an IHAVE to each gossip target
//    at its history_gossip heartbeats; a target that had not received (m, f)
//    by the IHAVE's arrival (its final key is later) answers with an IWANT and
//    gets the fragment (k_traffic_gossip, mirrors k_gossip).
// A send adds to the sender's tx columns; unless it is lost (churn: receiver
// offline at the arrival, or the message's lifetime over) it adds to the
// receiver's rx columns and the receiver returns ceil(packets / 2) pure ACKs
// (the ctrl columns). These passes only read the keys; the counters take
// atomics (diagnostic mode, off by default).

struct TrafficArgs {
  uint64_t* traffic;        // [N][GS_TRAFFIC_COLS]
  uint64_t W, pk, hdr;      // one fragment send: wire bytes, packets, header bytes
  uint64_t ihw, ihpk, ihhd; // one IHAVE RPC
  uint64_t iww, iwpk, iwhd; // one IWANT RPC
  uint64_t ack;             // header bytes of one ACK packet
  uint32_t Fe, flood, collide;
};

// Counters of one peer accumulated in registers, flushed with one atomic per
// non-zero column.
struct PeerTraffic {
  uint64_t txb = 0, txp = 0, txh = 0, rxb = 0, rxp = 0, rxh = 0, txc = 0, rxc = 0;
  __device__ void send(uint64_t n, uint64_t b, uint64_t p, uint64_t h) { txb += n * b; txp += n * p; txh += n * h; }
  // n arrivals of a p-packet send: rx, and the ACKs this peer returns
  __device__ void recv(uint64_t n, uint64_t b, uint64_t p, uint64_t h) {
    rxb += n * b; rxp += n * p; rxh += n * h; txc += n * ((p + 1) / 2);
  }
  __device__ void acked(uint64_t n, uint64_t p) { rxc += n * ((p + 1) / 2); }  // ACKs for n delivered sends
  __device__ void flush(const TrafficArgs& t, uint32_t x) const {
    unsigned long long* r = (unsigned long long*)(t.traffic + (size_t)x * GS_TRAFFIC_COLS);
    const uint64_t v[GS_TRAFFIC_COLS] = {txb, rxb, txp, rxp, txh, rxh, 0, 0, txc, rxc, txc * t.ack, rxc * t.ack};
#pragma unroll
    for (int k = 0; k < GS_TRAFFIC_COLS; k++)
      if (v[k]) atomicAdd(&r[k], (unsigned long long)v[k]);
  }
};

// One p-packet send s -> x arrived: x's rx and its ACKs (s's share is
// accumulated by the caller with PeerTraffic::acked).
__device__ __forceinline__ void tr_arrive(const TrafficArgs& t, uint32_t x, uint64_t b, uint64_t p, uint64_t h) {
  PeerTraffic q;
  q.recv(1, b, p, h);
  q.flush(t, x);
}
__device__ __forceinline__ void tr_count(const TrafficArgs& t, uint32_t x, int col) {
  atomicAdd((unsigned long long*)&t.traffic[(size_t)x * GS_TRAFFIC_COLS + col], 1ull);
}

// Publishes (publish_new_message, main.rs:101-143): one block per message.
__global__ __launch_bounds__(TB) void k_traffic_pub(RelaxArgs a, TrafficArgs t) {
  __shared__ uint32_t live[MAX_DEG];
  __shared__ uint32_t wcnt[TB / 64];
  const uint32_t m = blockIdx.x, p = a.pub[m], sp = a.stage[p], S = a.S;
  const uint64_t ser = a.tables[S * S + sp];
  if (a.churn && ep_off(a, a.q0[m], p)) return;  // offline publisher: nothing published
  if (threadIdx.x == 0) tr_count(t, p, GS_TR_PUBLISHED);
  uint32_t deg;
  const uint32_t* tg;
  bool packed;
  if (t.flood) { deg = (uint32_t)(a.row[p + 1] - a.row[p]); tg = a.col + a.row[p]; packed = false; }
  else {
    tg = a.churn ? ep_mesh(a, a.q0[m], p) : a.mesh + (size_t)p * MESH_W;
    deg = 0;
    while (deg < MESH_W && tg[deg] != EMPTY) deg++;
    packed = true;
  }
  if (a.churn && t.flood) {  // the connections online at t_pub, in id order (as k_seed)
    const uint32_t j = threadIdx.x;
    const bool on = j < deg && !ep_off(a, a.q0[m], tg[j]);
    const uint64_t bm = __ballot(on);
    if ((threadIdx.x & 63) == 0) wcnt[threadIdx.x >> 6] = (uint32_t)__popcll(bm);
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t q = 0; q < (threadIdx.x >> 6); q++) base += wcnt[q];
    if (on) live[base + (uint32_t)__popcll(bm & ((1ull << (threadIdx.x & 63)) - 1))] = tg[j];
    uint32_t tot = 0;
    for (uint32_t q = 0; q < TB / 64; q++) tot += wcnt[q];
    __syncthreads();
    deg = tot;
    tg = live;
  }
  PeerTraffic pt;
  const uint32_t total = t.Fe * deg;
  for (uint32_t i = threadIdx.x; i < total; i += TB) {
    const uint32_t f = i / deg, j = i % deg;
    const uint32_t w = packed ? (tg[j] & 0xFFFFFFu) : tg[j];
    const uint32_t sw = a.stage[w];
    const uint64_t sd = a.tables[S * S + S + sw];
    const uint64_t arr = ((uint64_t)f * deg + j + 1) * ser + a.tables[sp * S + sw] + (sd > ser ? sd - ser : 0);
    pt.send(1, t.W, t.pk, t.hdr);
    if (a.churn && ev_lost(a, m, arr, w)) continue;
    tr_arrive(t, w, t.W, t.pk, t.hdr);
    pt.acked(1, t.pk);
  }
  pt.flush(t, p);
}

// Forwards and completions: one lane per key (u, m, f); a wave holds whole
// FP-lane groups, so the uplink FIFO fold runs as in relax_lane.
template <int FP>
__global__ __launch_bounds__(TB) void k_traffic_fwd(RelaxArgs a, TrafficArgs t) {
  const int lane = threadIdx.x & 63;
  const uint32_t S = a.S, LL = a.L;
  const uint64_t smask = (1ull << a.sb) - 1;
  const uint64_t step = (uint64_t)gridDim.x * TB;
  for (uint64_t base = (uint64_t)blockIdx.x * TB + (threadIdx.x & ~63u); base < a.total; base += step) {
    const uint64_t gid = base + lane;  // wave-uniform loop: every lane joins the shuffles below
    const bool valid = gid < a.total;
    const uint64_t key = valid ? a.keys[gid] : INF64;
    const uint32_t u = valid ? row_of(gid, LL) : 0;
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t m = slot / FP, fl = slot & (FP - 1);
    const uint32_t pm = valid ? a.pub[m] : EMPTY;
    const bool got = key != INF64 && u != pm;
    {  // completed messages (reassembly, main.rs:79-99): every fragment of the group received
      constexpr uint64_t gmask = (FP == 64) ? ~0ull : ((1ull << FP) - 1);
      const uint64_t ok = __ballot(valid && (fl >= t.Fe || got));
      const bool lead = fl == 0 && got && !t.collide && ((ok >> (lane & ~(FP - 1))) & gmask) == gmask;
      if (lead) tr_count(t, u, GS_TR_RECEIVED);
    }
    const uint64_t tt = key >> a.tshift;
    const uint32_t src = (uint32_t)(key & smask);
    const uint32_t su = valid ? a.stage[u] : 0;
    const uint32_t ser = a.tables[S * S + su];
    const uint32_t* mrp = a.mesh + (size_t)u * MESH_W;
    bool dead = false;  // churn: received past the message's lifetime -> not forwarded
    if (got && a.churn) {
      const uint64_t h = ev_epoch(a, m, tt);
      dead = h > a.q0[m] + a.horizon;
      mrp = ep_mesh(a, dead ? a.q0[m] : h, u);
    }
    uint32_t row[MESH_W];
    uint32_t skip = ~0u, n = 0;
    if (got && !dead) {
      load_mesh_row(mrp, 0, row);
      skip = 0;
#pragma unroll
      for (int j = 0; j < (int)MESH_W; j++) {
        const uint32_t e = row[j];
        if (e == EMPTY) { skip |= 1u << j; continue; }
        const uint32_t w = e & 0xFFFFFFu;
        bool sk = w == src || w == pm;
        if (!sk && a.idw) {  // IDONTWANT from w already here (main.go:165)
          const uint64_t kw = a.keys[(size_t)w * LL + slot];
          sk = kw != INF64 && (kw >> a.tshift) + a.tables[(e >> STAGE_SHIFT) * S + su] <= tt;
        }
        if (sk) skip |= 1u << j; else n++;
      }
    }
    const uint64_t start = uplink_start<FP>(nullptr, 0, got, key, n, ser, a.tshift);
    if (!n) continue;
    PeerTraffic pt;
    pt.send(n, t.W, t.pk, t.hdr);
    uint32_t pos = 0;
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++) {
      if (skip & (1u << j)) continue;
      pos++;
      const uint32_t e = row[j];
      const uint32_t w = e & 0xFFFFFFu, sw = e >> STAGE_SHIFT;
      const uint32_t sd = a.tables[S * S + S + sw];
      const uint64_t arr = start + (uint64_t)pos * ser + a.tables[su * S + sw] + (sd > ser ? sd - ser : 0);
      if (a.churn && ev_lost(a, m, arr, w)) continue;
      tr_arrive(t, w, t.W, t.pk, t.hdr);
      pt.acked(1, t.pk);
    }
    pt.flush(t, u);
  }
}

// Lazy gossip: every holder lane (the publisher's own
// fragments from t_pub, a receiver's from its first receipt) at each of its
// history_gossip heartbeats.
template <int FP>
__global__ __launch_bounds__(TB) void k_traffic_gossip(RelaxArgs a, TrafficArgs t) {
  const uint32_t S = a.S, LL = a.L;
  const uint64_t step = (uint64_t)gridDim.x * TB;
  for (uint64_t gid = (uint64_t)blockIdx.x * TB + threadIdx.x; gid < a.total; gid += step) {
    const uint64_t key = a.keys[gid];
    if (key == INF64) continue;
    const uint64_t tt = key >> a.tshift;
    const uint32_t u = row_of(gid, LL), slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t m = slot / FP, sv = a.stage[u];
    const uint64_t ser = a.tables[S * S + sv];
    const uint64_t r0 = a.rel0[m];
    const uint64_t j0 = first_hb(tt, r0, a.hb_ns);
    PeerTraffic pt;
    for (uint32_t k = 0; k < a.hist; k++) {
      const uint64_t T = r0 + (j0 + k) * a.hb_ns;
      const uint64_t hab = a.habs0[m] + j0 + k;
      if (a.churn && (hab > a.q0[m] + a.horizon || ep_off(a, hab, u))) continue;
      for_each_gossip_target(a, u, hab, [&](uint32_t e) {
        const uint32_t w = e & 0xFFFFFFu, sw = e >> STAGE_SHIFT;
        const uint64_t ti = T + a.tables[sv * S + sw];
        const uint64_t sd = a.tables[S * S + S + sw];
        const uint64_t A = ti + a.tables[sw * S + sv] + ser + a.tables[sv * S + sw] + (sd > ser ? sd - ser : 0);
        pt.send(1, t.ihw, t.ihpk, t.ihhd);  // IHAVE u -> w
        if (a.churn && ev_lost(a, m, ti, w)) return;
        tr_arrive(t, w, t.ihw, t.ihpk, t.ihhd);
        pt.acked(1, t.ihpk);
        const uint64_t kw = a.keys[(size_t)w * LL + slot];
        if (kw != INF64 && (kw >> a.tshift) <= ti) return;  // w has it: no IWANT
        PeerTraffic wt;  // IWANT w -> u, then u's answer
        wt.send(1, t.iww, t.iwpk, t.iwhd);
        pt.recv(1, t.iww, t.iwpk, t.iwhd);
        wt.acked(1, t.iwpk);
        pt.send(1, t.W, t.pk, t.hdr);
        if (!(a.churn && ev_lost(a, m, A, w))) {
          wt.recv(1, t.W, t.pk, t.hdr);
          pt.acked(1, t.pk);
        }
        wt.flush(t, w);
      });
    }
    pt.flush(t, u);
  }
}
