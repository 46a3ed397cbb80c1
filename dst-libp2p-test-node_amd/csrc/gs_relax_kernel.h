// gs_relax_kernel.h — the hot kernels: one Delta-bucket of eager forwarding.
// Included by gs_relax.hip only (inside namespace gs::{anon}).
//
// Two implementations of one bucket, selected by GS_RELAX_VARIANT (bit 8):
//
//  * fused  k_relax: a wave owns 64 consecutive key lanes ("a tile"); it
//    scans them and forwards its active lanes in place. With 64 messages per
//    batch and F = 1 a tile is one peer's row, so pushes into a target w hit
//    one 512-B row. Only ~1/5 of the lanes are active per bucket and every
//    tile is a dependent chain (key -> mesh row -> final bits -> atomics), so
//    the kernel is latency bound.
//  * split  k_scan + k_frontier (default): the scan streams the keys,
//    compacts the bucket's arrivals with a wave ballot + mbcnt prefix into a
//    per-wave frontier segment (no returning atomics), and stores the final
//    bitset; the frontier kernel then runs the forward chain with every lane
//    carrying a real arrival (items of one peer stay adjacent, so pushes stay
//    row-coalesced).
//
// Option bits (all exact):
//   1 FILTER  read the target key first, atomicMin only when smaller
//   2 SKIP    per-tile {min pending key, scan stamp, push stamp} (fused); split:
//             per-tile min pending key + touched flag (+ next IHAVE arrival,
//             non-final count and scan stamp with lazy gossip)
//   4 FB      final bitset, 1 bit per key (N*L/8 bytes, L2/MALL resident),
//             written by the scanner; a push to a final target is dropped (a
//             final key cannot improve: every push lands >= the bucket end)
//   8 SPLIT   scan + frontier instead of the fused kernel

struct TileMeta {
  uint64_t tmin;     // min pending key (>= that launch's bucket end) at last scan
  uint32_t scanned;  // stamp (launch + 1) of the last scan
  uint32_t pushed;   // stamp of the last atomic push into the tile
};

struct RelaxArgs {
  uint64_t* keys;
  uint64_t* busy;
  TileMeta* meta;
  uint64_t* fbits;
  uint32_t* fr_idx;   // frontier: group index (gid / FP), per-wave segments
  uint64_t* fr_key;   // frontier: key (FP == 1)
  uint32_t* fr_cnt;   // frontier: items per wave segment
  uint64_t* tmin;     // split SKIP: min pending key per tile at its last scan
  uint8_t* touched;   // split SKIP: tile received a push since its last scan
  uint64_t* tgmin;    // split SKIP + gossip: next IHAVE arrival time of the tile's lanes (INF none)
  uint32_t* tnf;      // split SKIP + gossip: non-final lanes of the tile at its last scan
  uint32_t* tstamp;   // split SKIP + gossip: launch + 1 of the tile's last scan (k_gossip's seen filter)
  // lazy gossip
  uint32_t* gl_idx;   // gossip list: lane gid with an IHAVE arrival in this bucket
  uint32_t* gl_cnt;   // per scan wave
  uint64_t* nonfinal; // [3] lanes not final after scan k (slot k % 3)
  const uint64_t* rel0;   // per message: first heartbeat >= t_pub, relative ns
  const uint64_t* habs0;  // per message: its absolute heartbeat index
  const uint64_t* row;    // CSR (gossip targets are non-mesh connections)
  const uint32_t* col;
  uint64_t hb_ns, seed;
  uint32_t gl_cap, gossip, hist, d_lazy, gf_milli;
  uint32_t u0;        // global id of the first peer whose keys this context holds
  // churn: mesh / offline set of the epoch an event falls in
  const uint32_t* ring_mesh;  // [R][N][MESH_W]
  const uint64_t* ring_off;   // [R][w64]
  const uint64_t* q0;         // [B] epoch of t_pub
  const uint64_t* r0;         // [B] t_pub - start of that epoch
  uint32_t churn, ring_R, w64, horizon;
  // churn + gossip: receiver-centric lazy gossip over the inverse IHAVE lists
  // of each epoch (k_gossip_out_range + k_gossip_in_gather): [R][N][GT_IN]
  // senders (stage<<24 | id), EMPTY after the last, GT_REDO: recompute
  const uint32_t* ring_in;
  uint64_t* gl_key;            // receiver-centric: the listed lane's key
  // churn + gossip: heartbeats k >= gs_switch of a message (k counted from its
  // first heartbeat) are decided sender-centric: after the eager wave only the
  // peers that received it within their history window gossip it, a few
  // hundred per message, while the undelivered lanes stay ~10 % of all
  // so the scan appends every final lane that can gossip at such a
  // heartbeat to a holder list when it finalises it, and k_gossip walks only
  // the entries whose history window can still reach the bucket
  uint32_t* hs_idx;            // per scan wave: holders found by the wave (scratch, gl segments)
  uint64_t* hs_key;
  uint64_t* hl_min;            // [3] per launch: earliest IHAVE arrival of any holder (k_gossip walks if < hi)
  uint32_t* hl_idx;            // holder list: lane gid
  uint64_t* hl_key;            // its (final) key
  unsigned long long* hl_cnt;  // entries appended
  uint64_t* hl_lo;             // per launch: the bucket's start
  uint64_t* hl_end;            // per launch: list length after its scan
  uint32_t gs_switch;
  uint8_t* hwin;               // per lane: first gossip heartbeat index of its final key (255: none yet)
  const uint8_t* malive;       // churn + gossip, per message: its publisher was online at t_pub (else nobody holds it)
  uint64_t g0;                 //   and no IHAVE of the batch lands before g0 = min rel0 + the smallest latency
  const uint32_t* mesh;
  const uint32_t* pub;
  const uint8_t* stage;
  const uint32_t* tables;  // lat[S*S] | ser_up[S] | ser_dn[S]
  uint64_t* ctrl;
  uint64_t* counters;
  uint64_t total;          // N * L lanes
  uint64_t delta;
  uint64_t tmax;
  uint32_t seg_cap;        // frontier groups per wave segment
  uint32_t N, B, F, L, S, sb, tshift, launch, idw;
};

// n / d for n, d < 2^53: the correctly rounded double quotient is off by at
// most one, fixed exactly in integers (a 64-bit integer division is a long
// software sequence on gfx950)
// row of lane index gid (32-bit division whenever the index fits)
__device__ __forceinline__ uint32_t row_of(uint64_t gid, uint32_t LL) {
  return gid < (1ull << 32) ? (uint32_t)gid / LL : (uint32_t)(gid / LL);
}
__device__ __forceinline__ uint64_t udiv53(uint64_t n, uint64_t d) {
  uint64_t q = (uint64_t)((double)n / (double)d);
  if (q * d > n) q--;
  else if ((q + 1) * d <= n) q++;
  return q;
}

// ---- churn helpers; m = message index within the batch ----
// Epochs stay below 2^20 + horizon (gs_run checks the schedule), so the ring
// index is a 32-bit remainder.
template <class A>
__device__ __forceinline__ uint64_t ev_epoch(const A& a, uint32_t m, uint64_t t) {  // t relative to t_pub
  return a.q0[m] + udiv53(a.r0[m] + t, a.hb_ns);
}
template <class A>
__device__ __forceinline__ bool ep_off(const A& a, uint64_t h, uint32_t w) {
  return (a.ring_off[(size_t)((uint32_t)h % a.ring_R) * a.w64 + (w >> 6)] >> (w & 63)) & 1;
}
template <class A>
__device__ __forceinline__ const uint32_t* ep_mesh(const A& a, uint64_t h, uint32_t u) {
  return a.ring_mesh + ((size_t)((uint32_t)h % a.ring_R) * a.N + u) * MESH_W;
}
// Epoch of a time x >= 0 after heartbeat hab (heartbeat h opens epoch h): no
// division when x is shorter than a heartbeat.
__device__ __forceinline__ uint64_t ep_plus(uint64_t hab, uint64_t x, uint64_t hb) {
  return hab + (x < hb ? 0 : udiv53(x, hb));
}
// a delivery to w at relative time t is lost: past the message's lifetime or w offline
template <class A>
__device__ __forceinline__ bool ev_lost(const A& a, uint32_t m, uint64_t t, uint32_t w) {
  const uint64_t h = ev_epoch(a, m, t);
  return h > a.q0[m] + a.horizon || ep_off(a, h, w);
}

__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t x = __shfl_xor(v, off);
    v = x < v ? x : v;
  }
  return v;
}
// Block-level flush of wave-reduced values: one device-scope atomic per block
// instead of one per wave (same-address atomics serialize at the memory side,
// and a grid-wide counter sees thousands of waves per launch). Every thread of
// the block calls it. Wave wv stages its values at lds[wv * stride + k] (a
// block-shared area the caller owns; with stride >= the values per wave each
// wave touches only its own slot range). Slot 0 holds the min, slots
// 1..NS the sums.
template <int NW, int NS>
__device__ __forceinline__ void block_flush(uint64_t wmin, const uint64_t (&ws)[NS], unsigned long long* pmin,
                                            unsigned long long* const (&ps)[NS], uint64_t* lds, uint32_t stride) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    lds[wv * stride] = wmin;
#pragma unroll
    for (int k = 0; k < NS; k++) lds[wv * stride + 1 + k] = ws[k];
  }
  __syncthreads();
  if (threadIdx.x == 0 && pmin) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int i = 0; i < NW; i++) m = lds[i * stride] < m ? lds[i * stride] : m;
    if (m != ~0ull) atomicMin(pmin, (unsigned long long)m);
  }
  if (threadIdx.x >= 64 && threadIdx.x < 64 + NS) {  // another wave does the sums
    const int k = (int)threadIdx.x - 64;
    uint64_t t = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) t += lds[i * stride + 1 + k];
    if (t && ps[k]) atomicAdd(ps[k], (unsigned long long)t);
  }
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void load_mesh_row(const uint32_t* mesh, uint32_t u, uint32_t (&row)[MESH_W]) {
  const uint4* rp = reinterpret_cast<const uint4*>(mesh + (size_t)u * MESH_W);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 x = rp[q];
    row[4 * q] = x.x; row[4 * q + 1] = x.y; row[4 * q + 2] = x.z; row[4 * q + 3] = x.w;
  }
}

// Shared per-bucket constants in LDS.
struct BucketLds {
  uint32_t lat[MAX_STAGES * MAX_STAGES];
  uint32_t su[MAX_STAGES], sd[MAX_STAGES];
  uint32_t lmin[MAX_STAGES], lmax[MAX_STAGES];  // min/max latency out of each stage
  uint32_t imin[MAX_STAGES], imax[MAX_STAGES];  // min/max latency into each stage
  uint32_t lmax_all;                             // largest latency
};

__device__ __forceinline__ void load_tables(BucketLds& L, const RelaxArgs& a) {
  const uint32_t S = a.S;
  for (uint32_t i = threadIdx.x; i < S * S; i += TB) L.lat[i] = a.tables[i];
  if (threadIdx.x < S) {
    L.su[threadIdx.x] = a.tables[S * S + threadIdx.x];
    L.sd[threadIdx.x] = a.tables[S * S + S + threadIdx.x];
    uint32_t mn = ~0u, mx = 0;
    for (uint32_t s = 0; s < S; s++) {
      const uint32_t l = a.tables[threadIdx.x * S + s];
      mn = l < mn ? l : mn;
      mx = l > mx ? l : mx;
    }
    L.lmin[threadIdx.x] = mn;
    L.lmax[threadIdx.x] = mx;
    mn = ~0u;
    mx = 0;
    for (uint32_t s = 0; s < S; s++) {
      const uint32_t l = a.tables[s * S + threadIdx.x];
      mn = l < mn ? l : mn;
      mx = l > mx ? l : mx;
    }
    L.imin[threadIdx.x] = mn;
    L.imax[threadIdx.x] = mx;
  }
  if (threadIdx.x == 0) {
    uint32_t mx = 0;
    for (uint32_t i = 0; i < S * S; i++) mx = a.tables[i] > mx ? a.tables[i] : mx;
    L.lmax_all = mx;
  }
}

// With gossip on, launch k+1 has nothing to do once scan k left no lane
// non-final: every later IHAVE finds its target served.
__device__ __forceinline__ bool gossip_done(const RelaxArgs& a) {
  return a.gossip && a.launch > 0 && a.nonfinal[(a.launch + 2) % 3] == 0;
}

// First gossip heartbeat index j0 (relative to the message's first heartbeat
// rel0) with T_j0 >= t: heartbeats at rel0 + j*hb.
__device__ __forceinline__ uint64_t first_hb(uint64_t t, uint64_t rel0, uint64_t hb) {
  return t <= rel0 ? 0 : udiv53(t - rel0 + hb - 1, hb);
}

// Uplink FIFO across one (u, m)'s fragments: the FP-aligned lane group folds
// max(t_f, busy) + n_f * ser in (key, fragment) order (gossip answers bypass
// the FIFO, so two fragments can carry equal keys; the index breaks the tie)
// and stores the new FIFO end in busy[bi]. Returns the lane's uplink start.
// Closed form of the fold instead of FP sequential selection rounds (FP^2
// compares): with P_f = the sends queued before fragment f in that order,
//   start_f = max(busy + P_f, max over g <= f of t_g + P_f - P_g),
//   end     = max(busy + P, max over g of t_g + P - P_g),  P = all sends
// (O(FP) per lane; scripts/fifo_check.cpp compares it with the fold).
// Every lane of the wave must call this.
template <int FP>
__device__ __forceinline__ uint64_t uplink_start(uint64_t* busy, size_t bi, bool active, uint64_t key,
                                                 uint32_t n, uint32_t ser, uint32_t tshift) {
  uint64_t start = key >> tshift;
  if constexpr (FP > 1) {
    const int lane = threadIdx.x & 63;
    const int gb = lane & ~(FP - 1), me = lane - gb;
    const uint64_t ka = active ? key : INF64;
    // the group's keys are re-read by shuffle in each loop (no per-fragment
    // arrays live across the function: k_pull<8> spilled 187 VGPRs with them)
    uint64_t P = 0, tot = 0;  // sends before mine, all sends
    int first = -1;
#pragma unroll 8
    for (int g = FP - 1; g >= 0; g--) {
      const uint64_t kg = __shfl(ka, gb + g);
      const bool v = kg != INF64;
      if (v) first = g;
      const uint64_t d = (uint64_t)(uint32_t)__shfl((int)n, gb + g) * ser;
      tot += v ? d : 0;
      P += (v && (kg < ka || (kg == ka && g < me))) ? d : 0;
    }
    uint64_t s = 0, e = 0;
#pragma unroll 8
    for (int g = 0; g < FP; g++) {
      const uint64_t kg = __shfl(ka, gb + g), pg = __shfl(P, gb + g);
      if (kg == INF64) continue;
      const uint64_t tg = kg >> tshift;
      if (kg < ka || (kg == ka && g <= me)) s = max(s, tg + P - pg);
      e = max(e, tg + tot - pg);
    }
    if (first >= 0) {  // group-uniform
      const uint64_t cb = busy ? busy[bi] : 0;  // no busy array: the FIFO starts empty (gs_traffic.h)
      if (active) start = max(s, cb + P);
      if (busy && me == first) busy[bi] = max(e, cb + tot);
    }
  }
  return start;
}

// Forward one lane's first arrival (key at lane gid = u*L + slot). `active`
// must be true only for lanes finalised in this bucket; every lane of the wave
// must call this (FP > 1 shuffles across the FP-aligned lane group).
template <int FP, bool FILTER, bool SKIP, bool FB, bool TOUCH = false>
__device__ __forceinline__ void relax_lane(const RelaxArgs& a, const BucketLds& L, bool active,
                                           uint64_t key, uint32_t u, uint32_t slot, uint32_t pm,
                                           uint64_t& nmin, uint64_t& fd, uint64_t& nr, uint64_t& np, uint32_t& err) {
  const uint32_t S = a.S, LL = a.L;
  const uint64_t t = key >> a.tshift;
  const uint64_t smask = (1ull << a.sb) - 1;
  const uint32_t src = (uint32_t)(key & smask);
  const uint32_t hp = (uint32_t)((key >> a.sb) & ((1u << HOP_BITS) - 1));
  const uint32_t su = a.stage[u];
  const uint32_t ser = L.su[su];
  uint32_t row[MESH_W];
  uint32_t skip = 0, n = 0;
  const uint32_t* mrp = a.mesh + (size_t)u * MESH_W;
  bool dead = false;  // churn: received past the message's lifetime -> not forwarded
  if (active && a.churn) {
    const uint64_t h = ev_epoch(a, slot / FP, t);
    dead = h > a.q0[slot / FP] + a.horizon;
    mrp = ep_mesh(a, dead ? a.q0[slot / FP] : h, u);
  }
  if (active) {
    const uint4* rp = reinterpret_cast<const uint4*>(mrp);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 x = rp[q];
      row[4 * q] = x.x; row[4 * q + 1] = x.y; row[4 * q + 2] = x.z; row[4 * q + 3] = x.w;
    }
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++) {
      const uint32_t e = row[j];
      if (e == EMPTY || dead) { skip |= 1u << j; continue; }  // rows are EMPTY-padded at the tail
      const uint32_t w = e & 0xFFFFFFu;
      bool sk = (w == src) || (w == pm);
      if (!sk && a.idw) {  // IDONTWANT from w already here
        const uint64_t kw = a.keys[(size_t)w * LL + slot];
        sk = kw != INF64 && (kw >> a.tshift) + L.lat[(e >> STAGE_SHIFT) * S + su] <= t;
      }
      if (sk) skip |= 1u << j; else n++;
    }
  }
  const uint64_t start = uplink_start<FP>(a.busy, (size_t)u * a.B + slot / FP, active, key, n, ser, a.tshift);
  if (!active) return;
  fd++;
  nr += n;
  if (n && hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
  const uint64_t hbits = ((uint64_t)(hp + 1) << a.sb) | u;
  uint32_t fin = 0;  // targets already final: they still take an uplink slot
  if constexpr (FB) {
    uint64_t fw[MESH_W];
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++)
      fw[j] = (skip & (1u << j)) ? 0 : a.fbits[((size_t)(row[j] & 0xFFFFFFu) * LL + slot) >> 6];
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++)
      if ((fw[j] >> ((((size_t)(row[j] & 0xFFFFFFu)) * LL + slot) & 63)) & 1) fin |= 1u << j;
  }
  uint64_t old[MESH_W];
  if constexpr (FILTER) {
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++)
      old[j] = ((skip | fin) & (1u << j)) ? 0 : a.keys[(size_t)(row[j] & 0xFFFFFFu) * LL + slot];
  }
  uint32_t pos = 0;
#pragma unroll
  for (int j = 0; j < (int)MESH_W; j++) {
    if (skip & (1u << j)) continue;
    pos++;
    if (fin & (1u << j)) continue;
    const uint32_t e = row[j];
    const uint32_t w = e & 0xFFFFFFu, sw = e >> STAGE_SHIFT;
    const uint32_t sd = L.sd[sw];
    const uint64_t arr = start + (uint64_t)pos * ser + L.lat[su * S + sw] + (sd > ser ? sd - ser : 0);
    if (arr > a.tmax) err |= ERR_TIME;
    if (a.churn && ev_lost(a, slot / FP, arr, w)) continue;  // the send still took its uplink slot
    const uint64_t nk = (arr << a.tshift) | hbits;
    if (FILTER && !(nk < old[j])) continue;
    const size_t dst = (size_t)w * LL + slot;
    atomicMin((unsigned long long*)&a.keys[dst], (unsigned long long)nk);
    np++;
    if constexpr (SKIP) a.meta[dst >> 6].pushed = a.launch + 1;
    if constexpr (TOUCH) a.touched[dst >> 6] = 1;
    nmin = nk < nmin ? nk : nmin;
  }
}

__device__ __forceinline__ void flush_wave(const RelaxArgs& a, uint64_t nmin, uint64_t fd, uint64_t nr,
                                           uint64_t np, uint32_t err) {
  nmin = wave_min(nmin);
  fd = wave_sum(fd);
  nr = wave_sum(nr);
  np = wave_sum(np);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if ((threadIdx.x & 63) == 0) {
    if (nmin != INF64) atomicMin((unsigned long long*)&a.ctrl[(a.launch + 1) % 3], (unsigned long long)nmin);
    if (fd) atomicAdd((unsigned long long*)&a.counters[C_FD], (unsigned long long)fd);
    if (nr) atomicAdd((unsigned long long*)&a.counters[C_R_FWD], (unsigned long long)nr);
    if (np) atomicAdd((unsigned long long*)&a.counters[C_PUSH], (unsigned long long)np);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
}

// ---------------------------------------------------------------- fused ----
template <int FP, bool FILTER, bool SKIP, bool FB>
__global__ __launch_bounds__(TB) void k_relax(RelaxArgs a) {
  __shared__ BucketLds L;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctrl[(a.launch + 2) % 3] = INF64;
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64) return;  // grid-uniform: no pending keys left
  load_tables(L, a);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t LL = a.L, stamp = a.launch + 1;
  const int lane = threadIdx.x & 63;
  uint64_t nmin = INF64, fd = 0, nr = 0, np = 0;
  uint32_t err = 0;
  const uint64_t ntiles = (a.total + 63) >> 6;
  const uint64_t nwaves = (uint64_t)gridDim.x * (TB / 64);
  for (uint64_t tile = uniform64((uint64_t)blockIdx.x * (TB / 64) + (threadIdx.x >> 6)); tile < ntiles;
       tile += nwaves) {
    if constexpr (SKIP) {
      const TileMeta tm = a.meta[tile];
      const uint64_t tmin = uniform64(tm.tmin);
      const uint32_t scanned = __builtin_amdgcn_readfirstlane(tm.scanned);
      const uint32_t pushed = __builtin_amdgcn_readfirstlane(tm.pushed);
      if (pushed < scanned && (tmin == INF64 || (tmin >> a.tshift) >= hi)) {
        nmin = tmin < nmin ? tmin : nmin;
        continue;
      }
    }
    const uint64_t gid = (tile << 6) + lane;
    const bool valid = gid < a.total;
    const uint64_t key = valid ? a.keys[gid] : INF64;
    const uint64_t t = key >> a.tshift;
    const uint32_t u = valid ? (uint32_t)(gid / LL) : 0;
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t pm = valid ? a.pub[slot / FP] : EMPTY;
    const bool pending = key != INF64;
    const bool active = pending && t >= lo && t < hi && u != pm;
    const uint64_t later = (pending && t >= hi) ? key : INF64;
    nmin = later < nmin ? later : nmin;
    if constexpr (FB) {
      const uint64_t fw = __ballot(pending && t < hi);
      if (lane == 0) a.fbits[tile] = fw;
    }
    relax_lane<FP, FILTER, SKIP, FB>(a, L, active, key, u, slot, pm, nmin, fd, nr, np, err);
    if constexpr (SKIP) {
      const uint64_t tm = wave_min(later);
      if (lane == 0) {
        a.meta[tile].tmin = tm;
        a.meta[tile].scanned = stamp;
      }
    }
  }
  flush_wave(a, nmin, fd, nr, np, err);
}

// ---------------------------------------------------------------- split ----
// Scan: stream the keys, compact the bucket's arrivals (FP-lane groups with
// any active lane) into this wave's frontier segment, store the final bitset,
// reduce the next pending key.
template <int FP, bool SKIP, bool GOSSIP>
__global__ __launch_bounds__(TB) void k_scan(RelaxArgs a) {
  __shared__ BucketLds L;
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.ctrl[(a.launch + 2) % 3] = INF64;
    if (GOSSIP) a.nonfinal[(a.launch + 1) % 3] = 0;
    if (GOSSIP && a.hl_min) a.hl_min[(a.launch + 2) % 3] = INF64;
  }
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64) return;  // the frontier kernel exits on the same word
  if (GOSSIP && gossip_done(a)) return;
  if constexpr (GOSSIP) {
    load_tables(L, a);
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t LL = a.L;
  const uint64_t ntiles = (a.total + 63) >> 6;
  const uint64_t nwaves = (uint64_t)gridDim.x * (TB / 64);
  const size_t seg = (size_t)wave * a.seg_cap;
  const size_t gseg = (size_t)wave * a.gl_cap;
  uint64_t nmin = INF64, nonfin = 0, nscan = 0, nscan_g = 0, hmin = INF64;
  uint32_t cnt = 0, gcnt = 0, scnt = 0, err = 0;
  const uint64_t hspan = GOSSIP ? (uint64_t)a.hist * a.hb_ns : 0;
  // Tiles are visited per wave in groups: with SKIP a group is 64 consecutive
  // tiles whose metadata every lane loads at once (one coalesced load each,
  // instead of a dependent scalar chain per tile), and only the tiles that
  // cannot be skipped are scanned; without SKIP a group is one tile.
  constexpr uint64_t GT = SKIP ? 64 : 1;
  const uint64_t ngroups = (ntiles + GT - 1) / GT;
  for (uint64_t grp = uniform64(wave); grp < ngroups; grp += nwaves) {
   uint64_t todo = 1;
   if constexpr (SKIP) {
    // untouched since its last scan and nothing due in this bucket: the
    // tile's keys are unchanged, its min pending key stands for it. With
    // gossip its final lanes' next IHAVE arrival must lie beyond the bucket
    // too, and its non-final count stands.
    const uint64_t mt = grp * GT + lane;
    bool skip = false, eskip = false;
    if (mt < ntiles) {
      const uint64_t tm = a.tmin[mt];
      skip = !a.touched[mt] && (tm == INF64 || (tm >> a.tshift) >= hi);
      eskip = skip;
      uint64_t gm = INF64;
      if constexpr (GOSSIP) {
        if (skip) gm = a.tgmin[mt];
        skip = skip && (gm == INF64 || gm >= hi);
      }
      if (skip) {
        nmin = tm < nmin ? tm : nmin;
        if constexpr (GOSSIP) {
          if (gm != INF64) {
            const uint64_t gk = gm << a.tshift;
            nmin = gk < nmin ? gk : nmin;
          }
          nonfin += a.tnf[mt];
        }
      }
    }
    todo = __ballot(mt < ntiles && !skip);
    if (GOSSIP) nscan_g += (uint64_t)__popcll(__ballot(mt < ntiles && eskip && !skip));
   }
   while (todo) {  // wave-uniform
    const uint64_t tile = grp * GT + (uint64_t)__builtin_ctzll(todo);
    todo &= todo - 1;
    nscan++;
    const uint64_t gid = (tile << 6) + lane;
    const bool valid = gid < a.total;
    const uint64_t key = valid ? a.keys[gid] : INF64;
    const uint64_t t = key >> a.tshift;
    const uint32_t u = valid ? row_of(gid, LL) : 0;
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t pm = valid ? a.pub[slot / FP] : EMPTY;
    const bool pending = key != INF64;
    const bool active = pending && t >= lo && t < hi && u + a.u0 != pm;
    const uint64_t later = (pending && t >= hi) ? key : INF64;
    nmin = later < nmin ? later : nmin;
    const uint64_t fw = __ballot(pending && t < hi);
    if (lane == 0) a.fbits[tile] = fw;
    if constexpr (SKIP) {
      const uint64_t tmn = wave_min(later);
      if (lane == 0) {
        a.tmin[tile] = tmn;
        a.touched[tile] = 0;
      }
    }
    if constexpr (GOSSIP) {
      // final lanes gossip at the history_gossip heartbeats T >= t; their
      // IHAVEs reach targets at T + lat(s_v, s): list the lane if one of
      // those can fall in [lo, hi), fold the next one >= hi into nmin
      const bool fin = pending && t < hi;
      nonfin += (valid && !fin && slot % FP < a.F) ? 1u : 0u;  // padded fragments never arrive
      bool gwork = false, swork = false;  // receiver-centric entry (churn), sender-centric entry
      uint64_t gnext = INF64;
      // the first gossip heartbeat T_j0 < max(t, rel0) + hb, so a lane with
      // max(t, rel0) + hist*hb + lmax < lo is past its last IHAVE: skip it
      // before the division
      const uint32_t sv = (fin || a.ring_in) && valid ? a.stage[u] : 0, m = slot / FP;
      const uint64_t r0 = (fin || a.ring_in) && valid ? a.rel0[m] : 0;
      // churn: heartbeat indices [0, kl] lie in the message's lifetime (none
      // when its publisher was offline at t_pub: nobody holds it)
      const bool alive = a.ring_in && valid && slot % FP < a.F && a.hist && a.malive[m];
      const uint64_t kl = alive ? a.q0[m] + a.horizon - a.habs0[m] : 0;
      if (a.ring_in) {
        // receiver-centric (churn, heartbeats k < gs_switch): a lane without a
        // key before this bucket lists itself when an IHAVE of one of its
        // message's heartbeats T_k can reach its peer inside [lo, hi) (T_k +
        // min / max latency into its stage), up to the message's lifetime
        if (alive && !(pending && t < lo) && a.gs_switch > 0 && hi <= a.g0) {
          gnext = a.g0;  // before the batch's first heartbeat + the smallest latency no IHAVE lands
        } else if (alive && !(pending && t < lo) && a.gs_switch > 0) {
          const uint64_t imn = L.imin[sv], imx = L.imax[sv];
          const uint64_t kr = kl < a.gs_switch - 1 ? kl : a.gs_switch - 1;  // last receiver-centric heartbeat
          const uint64_t k0 = lo > r0 + imx ? udiv53(lo - r0 - imx + a.hb_ns - 1, a.hb_ns) : 0;
          // an IHAVE to a peer offline at its arrival is lost: with windows
          // shorter than a heartbeat, a window lies in the epoch of its T_k,
          // so the peer's offline epochs are skipped (its tile sleeps)
          const bool one_ep = imx < a.hb_ns;
          const uint64_t hab0 = a.habs0[m];
          gwork = k0 <= kr && r0 + k0 * a.hb_ns + imn < hi && !(one_ep && ep_off(a, hab0 + k0, u));
          // the next bucket that can hold one of these arrivals: the first
          // window still open at hi (a window spans several buckets) with the
          // peer online
          uint64_t k1 = hi > r0 + imx ? udiv53(hi - r0 - imx + a.hb_ns - 1, a.hb_ns) : 0;
          if (one_ep && k1 <= kr && ep_off(a, hab0 + k1, u)) k1++;  // (one step: later ones are found then)
          if (k1 <= kr) gnext = r0 + k1 * a.hb_ns + imn > hi ? r0 + k1 * a.hb_ns + imn : hi;
        }
      }
      if (a.hwin && pending && t >= lo && t < hi) {  // receiver-centric gossip reads it for senders
        const uint64_t j = t <= r0 ? 0 : t <= r0 + a.hb_ns ? 1 : first_hb(t, r0, a.hb_ns);
        a.hwin[gid] = (uint8_t)(j < 254 ? j : 254);
      }
      if (a.ring_in) {
        // holders: a lane finalised in this bucket that gossips at a heartbeat
        // k >= gs_switch (its first gossip heartbeat j0 >= gs_switch - hist + 1,
        // i.e. t > T_(gs_switch - hist)) joins the holder list; so does the
        // publisher's own lane (key 0) when gs_switch < hist
        const bool act = pending && t >= lo && t < hi && alive;
        swork = act && (a.gs_switch < a.hist || t > r0 + (uint64_t)(a.gs_switch - a.hist) * a.hb_ns);
      } else if (fin && a.hist && (t > r0 ? t : r0) + hspan + L.lmax[sv] >= lo) {
        // sender-centric (frozen mesh): a final lane gossips at its
        // history_gossip heartbeats T_k >= t
        const uint64_t lmn = L.lmin[sv], lmx = L.lmax[sv];
        const uint64_t j0 = first_hb(t, r0, a.hb_ns);
        const uint64_t tlast = r0 + (j0 + a.hist - 1) * a.hb_ns;
        if (tlast + lmx >= lo) {
          for (uint32_t k = 0; k < a.hist; k++) {
            const uint64_t T = r0 + (j0 + k) * a.hb_ns;
            gwork |= (T + lmx >= lo && T + lmn < hi);
            if (T + lmx >= hi)
              for (uint32_t s = 0; s < a.S; s++) {
                const uint64_t x = T + L.lat[sv * a.S + s];
                if (x >= hi && x < gnext) gnext = x;
              }
          }
        }
      }
      if (gnext != INF64) {
        if (gnext > a.tmax) err |= ERR_TIME;
        const uint64_t gk = gnext << a.tshift;
        nmin = gk < nmin ? gk : nmin;
      }
      const uint64_t gm = __ballot(gwork);
      if (gwork) {
        const uint32_t pos = gcnt + (uint32_t)__popcll(gm & ((1ull << lane) - 1));
        a.gl_idx[gseg + pos] = (uint32_t)gid;
        if (a.gl_key) a.gl_key[gseg + pos] = key;
      }
      gcnt += (uint32_t)__popcll(gm);
      const uint64_t sm = __ballot(swork);
      if (swork) {  // to this wave's scratch segment; copied to the list at the end
        const uint32_t pos = scnt + (uint32_t)__popcll(sm & ((1ull << lane) - 1));
        a.hs_idx[gseg + pos] = (uint32_t)gid;
        a.hs_key[gseg + pos] = key;
        // its first IHAVE arrival: heartbeat max(j0, gs_switch) + the smallest
        // latency out of its stage (k_gossip's walk test)
        const uint64_t j0 = first_hb(t, r0, a.hb_ns);
        const uint64_t k = j0 > a.gs_switch ? j0 : a.gs_switch;
        if (k < j0 + a.hist && k <= kl) {
          const uint64_t lb = r0 + k * a.hb_ns + L.lmin[sv];
          hmin = lb < hmin ? lb : hmin;
        }
      }
      scnt += (uint32_t)__popcll(sm);
      if constexpr (SKIP) {  // the tile's gossip state for later skips
        const uint64_t tg = wave_min(gnext);
        const uint32_t nf = (uint32_t)__popcll(__ballot(valid && !fin && slot % FP < a.F));
        if (lane == 0) {
          a.tgmin[tile] = tg;
          a.tnf[tile] = nf;
          a.tstamp[tile] = a.launch + 1;
        }
      }
    }
    const uint64_t am = __ballot(active);
    if (am == 0) continue;
    if constexpr (FP == 1) {
      const uint32_t pos = cnt + (uint32_t)__popcll(am & ((1ull << lane) - 1));
      if (active) {
        a.fr_idx[seg + pos] = (uint32_t)gid;
        a.fr_key[seg + pos] = key;
      }
      cnt += (uint32_t)__popcll(am);
    } else {
      constexpr uint64_t gmask = (FP == 64) ? ~0ull : ((1ull << FP) - 1);
      const bool leader = (lane & (FP - 1)) == 0 && ((am >> lane) & gmask) != 0;
      const uint64_t lm = __ballot(leader);
      if (leader) a.fr_idx[seg + cnt + (uint32_t)__popcll(lm & ((1ull << lane) - 1))] = (uint32_t)(gid / FP);
      cnt += (uint32_t)__popcll(lm);
    }
   }
  }
  if (lane == 0) a.fr_cnt[wave] = cnt;
  nmin = wave_min(nmin);
  if constexpr (GOSSIP) {
    nonfin = wave_sum(nonfin);
    for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
    if (lane == 0) {
      a.gl_cnt[wave] = gcnt;
      if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
    }
    if (a.hl_idx) {  // holders: one list claim per block, waves copy their scratch
      __shared__ uint32_t s_hn[TB / 64];
      __shared__ uint64_t s_hm[TB / 64];
      __shared__ unsigned long long s_base;
      const int wv = threadIdx.x >> 6;
      hmin = wave_min(hmin);
      if (lane == 0) { s_hn[wv] = scnt; s_hm[wv] = hmin; }
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t tot = 0;
        uint64_t mn = INF64;
        for (int i = 0; i < TB / 64; i++) { tot += s_hn[i]; mn = s_hm[i] < mn ? s_hm[i] : mn; }
        s_base = tot ? atomicAdd(a.hl_cnt, (unsigned long long)tot) : 0;
        if (mn != INF64) atomicMin((unsigned long long*)&a.hl_min[a.launch % 3], (unsigned long long)mn);
      }
      __syncthreads();
      uint64_t base = s_base;
      for (int i = 0; i < wv; i++) base += s_hn[i];
      for (uint32_t i = lane; i < scnt; i += 64) {
        a.hl_idx[base + i] = a.hs_idx[gseg + i];
        a.hl_key[base + i] = a.hs_key[gseg + i];
      }
    }
  }
  __shared__ uint64_t s_red[TB / 64 * 5];
  const uint64_t ws[4] = {nonfin, GOSSIP ? (uint64_t)gcnt + scnt : 0, nscan, nscan_g};
  unsigned long long* const ps[4] = {GOSSIP ? (unsigned long long*)&a.nonfinal[a.launch % 3] : nullptr,
                                     (unsigned long long*)&a.counters[C_GLISTED],
                                     (unsigned long long*)&a.counters[C_TSCANNED],
                                     (unsigned long long*)&a.counters[C_TSCANNED_G]};
  block_flush<TB / 64, 4>(nmin, ws, (unsigned long long*)&a.ctrl[(a.launch + 1) % 3], ps, s_red, 5);
}

// Lazy gossip of one bucket: for every listed final lane
// (v, m, f) and each of its gossip heartbeats with an IHAVE arrival in
// [lo, hi): recompute gossip_targets(v, h); a target w that has not seen
// (m, f) by the IHAVE's arrival t_i sends IWANT, and v's answer is pushed with
// key (t_i + lat(w,v) + ser_up(v) + lat(v,w) + dn, hops_v + 1, v). Deciding
// here is exact: every key below hi is final, and every answer lands >= hi.
constexpr uint32_t GOSSIP_R_REG = 8;
__device__ __forceinline__ bool pair_lt(uint64_t k1, uint32_t w1, uint64_t k2, uint32_t w2) {
  return k1 < k2 || (k1 == k2 && w1 < w2);
}

// gossip_targets(u, hab) (libp2p-gossipsub emit_gossip, upstream; DESIGN.md
// §2.7): the r smallest (rng(GOSSIP, u, h, w), w) among u's non-mesh
// connections (online ones under churn, over the epoch's mesh), r =
// max(D_lazy, floor(factor * |non-mesh|)) capped at |non-mesh|; fn(e) per
// target in that order, e = stage << STAGE_SHIFT | id (as a mesh entry). The
// caller checks that u gossips at hab.
template <class Fn>
__device__ __forceinline__ void for_each_gossip_target(const RelaxArgs& a, uint32_t u, uint64_t hab, Fn&& fn) {
  const uint32_t h = (uint32_t)hab;
  uint32_t mrow[MESH_W];
  const uint32_t* mrp = a.mesh + (size_t)u * MESH_W;
  if (a.churn) mrp = ep_mesh(a, hab, u);
  const uint4* rp = reinterpret_cast<const uint4*>(mrp);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 x = rp[q];
    mrow[4 * q] = x.x & 0xFFFFFFu; mrow[4 * q + 1] = x.y & 0xFFFFFFu;
    mrow[4 * q + 2] = x.z & 0xFFFFFFu; mrow[4 * q + 3] = x.w & 0xFFFFFFu;
  }
  // r smallest (rng(GOSSIP, u, h, w), w) among non-mesh connections. The
  // first GOSSIP_R_REG stay sorted in registers (static indices: no
  // scratch); r depends on |non-mesh|, so it is cut after counting, and
  // the rare targets beyond GOSSIP_R_REG are found by rescanning for the
  // next smallest pair.
  uint64_t kk[GOSSIP_R_REG];
  uint32_t ww[GOSSIP_R_REG];
#pragma unroll
  for (int q = 0; q < (int)GOSSIP_R_REG; q++) { kk[q] = ~0ull; ww[q] = ~0u; }
  uint32_t nonmesh = 0;
  const uint64_t e0 = a.row[u], e1 = a.row[u + 1];
  auto eligible = [&](uint32_t w) {
    bool inm = false;
#pragma unroll
    for (int q = 0; q < (int)MESH_W; q++) inm |= mrow[q] == w;
    return !inm && !(a.churn && ep_off(a, hab, w));
  };
  const uint64_t pre = rng_pre(a.seed, P_GOSSIP, u);
  for (uint64_t e = e0; e < e1; e++) {
    const uint32_t w = a.col[e];
    if (!eligible(w)) continue;
    nonmesh++;
    const uint64_t rk = rng_fin(pre, h, w);
    if (!pair_lt(rk, w, kk[GOSSIP_R_REG - 1], ww[GOSSIP_R_REG - 1])) continue;
#pragma unroll
    for (int q = (int)GOSSIP_R_REG - 1; q > 0; q--) {  // insert, shifting the larger pairs up
      if (pair_lt(rk, w, kk[q - 1], ww[q - 1])) { kk[q] = kk[q - 1]; ww[q] = ww[q - 1]; }
      else if (pair_lt(rk, w, kk[q], ww[q])) { kk[q] = rk; ww[q] = w; }
    }
    if (pair_lt(rk, w, kk[0], ww[0])) { kk[0] = rk; ww[0] = w; }
  }
  uint32_t r = (uint32_t)(((uint64_t)nonmesh * a.gf_milli) / 1000);
  if (r < a.d_lazy) r = a.d_lazy;
  if (r > nonmesh) r = nonmesh;
#pragma unroll
  for (int q = 0; q < (int)GOSSIP_R_REG; q++)
    if ((uint32_t)q < r) fn(((uint32_t)a.stage[ww[q]] << STAGE_SHIFT) | ww[q]);
  uint64_t pk = kk[GOSSIP_R_REG - 1];
  uint32_t pw = ww[GOSSIP_R_REG - 1];
  for (uint32_t q = GOSSIP_R_REG; q < r; q++) {  // rare: more than GOSSIP_R_REG targets
    uint64_t bk = ~0ull;
    uint32_t bw = ~0u;
    for (uint64_t e = e0; e < e1; e++) {
      const uint32_t w = a.col[e];
      if (!eligible(w)) continue;
      const uint64_t rk = rng_fin(pre, h, w);
      if (pair_lt(pk, pw, rk, w) && pair_lt(rk, w, bk, bw)) { bk = rk; bw = w; }
    }
    fn(((uint32_t)a.stage[bw] << STAGE_SHIFT) | bw);
    pk = bk;
    pw = bw;
  }
}

// Receiver-centric lazy gossip of one bucket (churn): every listed lane
// (w, m, f) — no key before the bucket — reads, for each of its message's
// heartbeats T_k whose IHAVEs can reach w inside [lo, hi), the inverse IHAVE
// list of (w, epoch of T_k): each sender v that holds (m, f) by T_k with T_k
// among its history_gossip heartbeats (v's final key) sent an IHAVE arriving
// at t_i = T_k + lat(v, w); if w has not seen (m, f) by t_i (its own key) and
// neither the IHAVE nor the answer is lost, that is one IWANT and a candidate
// answer key. The lane keeps the smallest (one atomicMin). Exactly the IHAVE
// decisions of the sender-centric form, without touching the ~97 % of IHAVEs
// whose target already has the message.
template <int FP>
__device__ __forceinline__ void gossip_receiver(const RelaxArgs& a, const BucketLds& L, uint64_t lo, uint64_t hi,
                                                uint32_t gid, uint64_t kw, uint64_t& nmin, uint64_t& iw,
                                                uint32_t& err) {
  const uint32_t LL = a.L, S = a.S;
  const uint64_t tw = kw == INF64 ? INF64 : kw >> a.tshift;
  const uint32_t w = row_of(gid, LL), slot = (uint32_t)(gid - (uint64_t)w * LL);
  const uint32_t m = slot / FP, sw = a.stage[w];
  const uint64_t r0 = a.rel0[m], hb = a.hb_ns, lim = a.q0[m] + a.horizon;
  const uint64_t imn = L.imin[sw], imx = L.imax[sw], sdw = L.sd[sw];
  uint64_t best = INF64;
  uint64_t k = lo > r0 + imx ? udiv53(lo - r0 - imx + hb - 1, hb) : 0;
  for (;; k++) {
    const uint64_t T = r0 + k * hb;
    const uint64_t hab = a.habs0[m] + k;
    if (T + imn >= hi || hab > lim || k >= a.gs_switch) break;  // later heartbeats: sender-centric
    if (imx < hb && ep_off(a, hab, w)) continue;  // every IHAVE of this heartbeat reaches w offline
    auto ihave = [&](uint32_t e) {  // the IHAVE v -> w of heartbeat hab
      const uint32_t v = e & 0xFFFFFFu, sv = e >> STAGE_SHIFT;
      const uint64_t lvw = L.lat[sv * S + sw];
      const uint64_t ti = T + lvw;
      if (ti < lo || ti >= hi || tw <= ti) return;  // another bucket, or w has seen it
      const uint64_t hi_ = ep_plus(hab, lvw, hb);
      if (hi_ > lim || ep_off(a, hi_, w)) return;  // IHAVE lost
      // v's final bit clear: its key is >= hi > T (a tile the last scan skipped
      // has no pending key below hi; pushes land >= hi), no key read
      const size_t vi = (size_t)v * LL + slot;
      if (!a.hwin && a.tstamp && !((a.fbits[vi >> 6] >> (vi & 63)) & 1)) return;
      // v holds (m, f) at T and T is one of its gossip heartbeats: j0 <= k <
      // j0 + hist, j0 = the first heartbeat at or after its final key time
      // (hwin, written when the scan finalised it; else from the key)
      uint64_t kv = INF64, j0;
      if (a.hwin) {
        j0 = a.hwin[vi];
        if (j0 == 255) return;  // not final: does not hold it
      } else {
        kv = a.keys[vi];
        if (kv == INF64 || (kv >> a.tshift) > T) return;  // v does not hold it at T
        j0 = first_hb(kv >> a.tshift, r0, hb);
      }
      if (k < j0 || k >= j0 + a.hist) return;  // T is not one of v's gossip heartbeats
      const uint64_t ser = L.su[sv];
      const uint64_t A = ti + L.lat[sw * S + sv] + ser + lvw + (sdw > ser ? sdw - ser : 0);
      const uint64_t ha = ep_plus(hab, A - T, hb);
      if (ha > lim || ep_off(a, ha, w)) return;  // answer lost
      iw++;
      if (A > a.tmax) err |= ERR_TIME;
      // the answer's key needs v's hops only if its time can beat (or tie) the
      // best answer so far and w's own key
      const uint64_t cur = best < kw ? best : kw;
      if (cur != INF64 && A > (cur >> a.tshift)) return;
      if (kv == INF64) kv = a.keys[vi];
      const uint32_t hp = (uint32_t)((kv >> a.sb) & ((1u << HOP_BITS) - 1));
      if (hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
      const uint64_t nk = (A << a.tshift) | ((uint64_t)(hp + 1) << a.sb) | v;
      best = nk < best ? nk : best;
    };
    // epoch-major lists ([R][N][GT_IN]; receiver-major measured 5 % slower on
    // config #3 although a tile's lanes then read one contiguous run)
    const size_t li = (size_t)((uint32_t)hab % a.ring_R) * a.N + w;
    // the list: senders first, EMPTY after them; GT_REDO in entry 0: more
    // senders than it holds (k_gossip_in_gather)
    const uint4* lp = reinterpret_cast<const uint4*>(a.ring_in + li * GT_IN);
    const uint4 x0 = lp[0];
    if (x0.x != GT_REDO) {
      for (uint32_t q0 = 0; q0 < GT_IN; q0 += 4) {
        const uint4 x = q0 ? lp[q0 / 4] : x0;
        if (x.x == EMPTY) break;
        ihave(x.x);
        if (x.y == EMPTY) break;
        ihave(x.y);
        if (x.z == EMPTY) break;
        ihave(x.z);
        if (x.w == EMPTY) break;
        ihave(x.w);
      }
    } else {  // more senders than the list holds (rare): w's online non-mesh neighbours that pick w
      for (uint64_t e = a.row[w]; e < a.row[w + 1]; e++) {
        const uint32_t v = a.col[e];
        if (ep_off(a, hab, v)) continue;
        for_each_gossip_target(a, v, hab, [&](uint32_t x) {
          if ((x & 0xFFFFFFu) == w) ihave(((uint32_t)a.stage[v] << STAGE_SHIFT) | v);
        });
      }
    }
  }
  if (best < kw) {
    atomicMin((unsigned long long*)&a.keys[gid], (unsigned long long)best);
    if (a.tstamp) a.touched[gid >> 6] = 1;
    nmin = best < nmin ? best : nmin;
  }
}

// Sender-centric lazy gossip of one listed final lane (v, m, f): each of its
// history_gossip heartbeats (index >= kmin) with an IHAVE arrival in [lo, hi)
// re-selects v's targets; a target that has not seen (m, f) by the arrival
// sends IWANT and v's answer is pushed into its key.
// With `next` (the holder list) the lane's next IHAVE arrival at or after hi
// is folded into *next as well (the scan does that for listed lanes).
template <int FP>
__device__ __forceinline__ void gossip_sender(const RelaxArgs& a, const BucketLds& L, uint64_t lo, uint64_t hi,
                                              uint64_t gid, uint64_t key, uint64_t kmin, uint64_t* next,
                                              uint64_t& nmin, uint64_t& iw, uint32_t& err) {
  const uint32_t LL = a.L, S = a.S;
  const uint64_t t = key >> a.tshift;
  const uint32_t u = row_of(gid, LL), slot = (uint32_t)(gid - (uint64_t)u * LL);
  const uint32_t m = slot / FP, sv = a.stage[u];
  const uint32_t hp = (uint32_t)((key >> a.sb) & ((1u << HOP_BITS) - 1));
  const uint64_t ser = L.su[sv];
  const uint64_t r0 = a.rel0[m];
  const uint64_t j0 = first_hb(t, r0, a.hb_ns);
  for (uint32_t k = 0; k < a.hist; k++) {
    if (j0 + k < kmin) continue;
    const uint64_t T = r0 + (j0 + k) * a.hb_ns;
    const uint64_t hab = a.habs0[m] + j0 + k;
    if (next && T + L.lmax[sv] >= hi && !(a.churn && hab > a.q0[m] + a.horizon))
      for (uint32_t s = 0; s < S; s++) {
        const uint64_t x = T + L.lat[sv * S + s];
        if (x >= hi && x < *next) *next = x;
      }
    if (T + L.lmax[sv] < lo || T + L.lmin[sv] >= hi) continue;
    auto ihave = [&](uint32_t e) {  // v's IHAVE to w; IWANT + answer if w has not seen it
      const uint32_t w = e & 0xFFFFFFu, sw = e >> STAGE_SHIFT;
      const uint64_t lvw = L.lat[sv * S + sw];
      const uint64_t ti = T + lvw;
      if (ti < lo || ti >= hi) return;
      const uint64_t sd = L.sd[sw];
      const uint64_t A = ti + L.lat[sw * S + sv] + ser + lvw + (sd > ser ? sd - ser : 0);
      if (a.churn) {  // IHAVE or answer lost: epochs counted from the heartbeat's (= ev_epoch)
        const uint64_t lim = a.q0[m] + a.horizon;
        const uint64_t hi_ = ep_plus(hab, lvw, a.hb_ns), ha = ep_plus(hab, A - T, a.hb_ns);
        if (hi_ > lim || ep_off(a, hi_, w) || ha > lim || ep_off(a, ha, w)) return;
      }
      const size_t dst = (size_t)w * LL + slot;
      // final before this bucket (its tile's final bit from an earlier scan:
      // key time < that bucket's end <= lo <= t_i): seen, no key read
      if (a.tstamp && ((a.fbits[dst >> 6] >> (dst & 63)) & 1) && a.tstamp[dst >> 6] != a.launch + 1) return;
      const uint64_t kw = a.keys[dst];
      if (kw != INF64 && (kw >> a.tshift) <= ti) return;  // already seen: no IWANT
      iw++;
      if (A > a.tmax) err |= ERR_TIME;
      if (hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
      const uint64_t nk = (A << a.tshift) | ((uint64_t)(hp + 1) << a.sb) | u;
      if (nk < kw) {
        atomicMin((unsigned long long*)&a.keys[dst], (unsigned long long)nk);
        if (a.tstamp) a.touched[dst >> 6] = 1;
        nmin = nk < nmin ? nk : nmin;
      }
    };
    // v gossips only while online, within the message's lifetime
    if (a.churn && (hab > a.q0[m] + a.horizon || ep_off(a, hab, u))) continue;
    for_each_gossip_target(a, u, hab, ihave);
  }
}

template <int FP>
__global__ __launch_bounds__(TB) void k_gossip(RelaxArgs a) {
  __shared__ BucketLds L;
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64 || gossip_done(a)) return;
  load_tables(L, a);
  __syncthreads();
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t n = __builtin_amdgcn_readfirstlane(a.gl_cnt[wave]);
  const size_t seg = (size_t)wave * a.gl_cap;
  uint64_t nmin = INF64, iw = 0;
  uint32_t err = 0;
  if (a.ring_in) {
    for (uint32_t i = lane; i < n; i += 64)
      gossip_receiver<FP>(a, L, lo, hi, a.gl_idx[seg + i], a.gl_key[seg + i], nmin, iw, err);
    // holders (heartbeats >= gs_switch): the entries finalised after the last
    // launch whose bucket ended before lo - (hist * hb + the largest latency),
    // the earliest finalisation time whose IHAVEs can still arrive at lo
    const uint64_t end = *a.hl_cnt;
    const uint64_t span = (uint64_t)a.hist * a.hb_ns + L.lmax_all;
    uint64_t start = 0;
    if (lo > span) {
      const uint64_t x = lo - span;
      uint32_t l0 = 0, l1 = a.launch;  // last launch with lo_l + delta <= x: binary search on [l0, l1)
      while (l0 < l1) {
        const uint32_t mid = (l0 + l1) >> 1;
        if (a.hl_lo[mid] + a.delta <= x) l0 = mid + 1; else l1 = mid;
      }
      start = l0 > 0 ? a.hl_end[l0 - 1] : 0;
    }
    const uint64_t hm = a.hl_min[a.launch % 3];
    uint64_t hnext = INF64;
    if (hm < hi) {
      const uint64_t nthreads = (uint64_t)gridDim.x * TB;
      for (uint64_t i = start + (uint64_t)blockIdx.x * TB + threadIdx.x; i < end; i += nthreads)
        gossip_sender<FP>(a, L, lo, hi, a.hl_idx[i], a.hl_key[i], a.gs_switch, &hnext, nmin, iw, err);
    } else if (blockIdx.x == 0 && threadIdx.x == 0) {
      hnext = hm;  // no holder's IHAVE lands in this bucket: the bound carries over
    }
    hnext = wave_min(hnext);
    if (hnext != INF64) {
      if (hnext > a.tmax) err |= ERR_TIME;
      const uint64_t gk = hnext << a.tshift;
      nmin = gk < nmin ? gk : nmin;
      if (lane == 0) atomicMin((unsigned long long*)&a.hl_min[(a.launch + 1) % 3], (unsigned long long)hnext);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      a.hl_lo[a.launch] = lo;
      a.hl_end[a.launch] = end;
    }
  } else {
    for (uint32_t i = lane; i < n; i += 64)
      gossip_sender<FP>(a, L, lo, hi, a.gl_idx[seg + i], a.keys[a.gl_idx[seg + i]], 0, nullptr, nmin, iw, err);
  }
  nmin = wave_min(nmin);
  iw = wave_sum(iw);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if (lane == 0) {
    if (nmin != INF64) atomicMin((unsigned long long*)&a.ctrl[(a.launch + 1) % 3], (unsigned long long)nmin);
    if (iw) atomicAdd((unsigned long long*)&a.counters[C_GOSSIP], (unsigned long long)iw);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
}

// Frontier: every lane carries one compacted arrival (FP lanes per group).
template <int FP, bool FILTER, bool TOUCH>
__global__ __launch_bounds__(TB) void k_frontier(RelaxArgs a) {
  __shared__ BucketLds L;
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64 || gossip_done(a)) return;
  load_tables(L, a);
  __syncthreads();
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t LL = a.L;
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t n = __builtin_amdgcn_readfirstlane(a.fr_cnt[wave]);
  const size_t seg = (size_t)wave * a.seg_cap;
  constexpr uint32_t GPW = 64 / FP;  // groups per wave-iteration
  uint64_t nmin = INF64, fd = 0, nr = 0, np = 0;
  uint32_t err = 0;
  for (uint32_t base = 0; base < n; base += GPW) {
    const uint32_t gi = base + (uint32_t)lane / FP;
    const bool valid = gi < n;
    uint64_t gid, key;
    if constexpr (FP == 1) {
      gid = valid ? a.fr_idx[seg + gi] : 0;
      key = valid ? a.fr_key[seg + gi] : INF64;
    } else {
      gid = valid ? (uint64_t)a.fr_idx[seg + gi] * FP + (lane & (FP - 1)) : 0;
      key = valid ? a.keys[gid] : INF64;
    }
    const uint64_t t = key >> a.tshift;
    const uint32_t u = row_of(gid, LL);
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t pm = valid ? a.pub[slot / FP] : EMPTY;
    const bool active = valid && key != INF64 && t >= lo && t < hi && u != pm;
    relax_lane<FP, FILTER, false, true, TOUCH>(a, L, active, key, u, slot, pm, nmin, fd, nr, np, err);
  }
  flush_wave(a, nmin, fd, nr, np, err);
}

// ------------------------------------------------------------- dispatch ----
template <int FP>
void relax_fp(uint32_t variant, const RelaxArgs& a, unsigned grid, hipStream_t s, hipEvent_t mid) {
  if (variant & 8) {
    if (a.gossip && (variant & 2)) k_scan<FP, true, true><<<grid, TB, 0, s>>>(a);
    else if (a.gossip) k_scan<FP, false, true><<<grid, TB, 0, s>>>(a);
    else if (variant & 2) k_scan<FP, true, false><<<grid, TB, 0, s>>>(a);
    else k_scan<FP, false, false><<<grid, TB, 0, s>>>(a);
    if (mid) (void)hipEventRecord(mid, s);  // splits scan / frontier time when timing
    switch (variant & 3) {
      case 0: k_frontier<FP, false, false><<<grid, TB, 0, s>>>(a); break;
      case 1: k_frontier<FP, true, false><<<grid, TB, 0, s>>>(a); break;
      case 2: k_frontier<FP, false, true><<<grid, TB, 0, s>>>(a); break;
      default: k_frontier<FP, true, true><<<grid, TB, 0, s>>>(a); break;
    }
    if (a.gossip) k_gossip<FP><<<grid, TB, 0, s>>>(a);
    return;
  }
  switch (variant & 7) {
    case 0: k_relax<FP, false, false, false><<<grid, TB, 0, s>>>(a); break;
    case 1: k_relax<FP, true, false, false><<<grid, TB, 0, s>>>(a); break;
    case 2: k_relax<FP, false, true, false><<<grid, TB, 0, s>>>(a); break;
    case 3: k_relax<FP, true, true, false><<<grid, TB, 0, s>>>(a); break;
    case 4: k_relax<FP, false, false, true><<<grid, TB, 0, s>>>(a); break;
    case 5: k_relax<FP, true, false, true><<<grid, TB, 0, s>>>(a); break;
    case 6: k_relax<FP, false, true, true><<<grid, TB, 0, s>>>(a); break;
    default: k_relax<FP, true, true, true><<<grid, TB, 0, s>>>(a); break;
  }
}

void relax_dispatch(uint32_t FP, uint32_t variant, const RelaxArgs& a, unsigned grid, hipStream_t s,
                    hipEvent_t mid = nullptr) {
  switch (FP) {
    case 1: relax_fp<1>(variant, a, grid, s, mid); break;
    case 2: relax_fp<2>(variant, a, grid, s, mid); break;
    case 4: relax_fp<4>(variant, a, grid, s, mid); break;
    case 8: relax_fp<8>(variant, a, grid, s, mid); break;
    default: relax_fp<16>(variant, a, grid, s, mid); break;
  }
}
