// gs_lpull_kernel.h — owner-computes Delta-window pass over per-row candidate
// lists, the default eager path when its bounds hold.
// Included by gs_relax.hip after gs_pull_kernel.h (namespace gs::{anon}).
//
// Why: k_pull keeps every (peer, message) key in a dense row and re-reads the
// live 64-lane chunks of the row in every window pass. At the peak of a
// 1024-message batch every chunk holds a due key, so each of the ~17 windows
// re-reads the whole 8 KB row and writes back every 64-B sector holding a
// changed lane: 2.3x the algorithmic bytes (profiles/r02_v5). Here a lane's
// state is never kept in a dense row during the passes:
//
//  - fin[w]: one bit per lane, set when the lane's key is final (emitted),
//    held transposed in registers (lane j: bit q for lane q*64 + j) while the
//    row is processed;
//  - candidates that do not fall in the window being emitted are appended to
//    the row's list for their destination window c' (slot c' % K of a ring of
//    K lists of up to L entries); st[w] holds the K list lengths and the
//    length of the row's final log, and is read with the row's header, so
//    the pass that emits window c knows where its entries are without a
//    dependent load;
//  - final keys are appended to a per-row log (the keys buffer, emission
//    order, lanes in flane) and scattered back to the dense [N][L] layout
//    once per batch (k_lfinal) for k_complete.
//
// A pass PULLing window b's records (emitting c = b+1) min-reduces, per lane
// in LDS, the entries listed for c and this pass's candidates from the
// neighbours' records; final lanes are dropped when the minima are
// classified. A lane whose minimum lies in window c is final (Delta-stepping:
// every later candidate is >= the start of window c+1); a lane whose minimum
// lies later is appended once, as the best of this pass, to the list of its
// window. Candidates worse than a listed one are harmless: the lane is final
// by the time their window comes. The candidate arithmetic and the records are
// k_pull's, so the keys are bit-identical. A list that would outgrow L entries
// sets ERR_LIST and the host re-runs the batch on k_pull.
//
// Entry (u64): t - (c' * Delta) | hops | src | lane, the key's low (hops |
// src) bits kept as they are; the host checks the widths fit.
//
// IDONTWANT (go preset; template IDW, rows of one fragment):
// a final lane's key also goes to the dense keys[N][L] table (INF-initialised
// for such batches; no final log), and the emit step reads the key of the same
// lane at each mesh neighbour y: y is skipped when its key time + lat(y -> w)
// <= t. Such batches run with windows no wider than the smallest latency
// (gs_relax.hip), so only keys final in earlier windows — written by earlier
// passes, stable — can pass the test.
//
// Arrival record (every batch): the sender's row lists which of its mesh
// entries receive the lane (all but the source and the publisher, and for
// IDONTWANT the peers that said they have it) as a 16-bit inclusion mask:
//   start - window_lo (32) | hops (6) | inclusion mask (16) | lane (10);
// the receiver at index r of the sender's row takes it iff bit r is set, at
// FIFO position 1 + popcount(mask below r). A missing record reads 0: no bit.

// The record step reads through raw buffer resources whose word 3 (0x00020000:
// DATA_FORMAT 32, no swizzle, bounds check on) is the gfx9 / CDNA layout; its
// out-of-range reads return 0, which the step relies on.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "k_lpull's buffer resource layout is gfx950's (CDNA4); build with --offload-arch=gfx950"
#endif

constexpr uint32_t LP_KMAX = 12;  // ring of destination-window lists
constexpr uint32_t LP_SW = 16;    // u32 words of per-row state: list lengths [0..11] (slot = window % K), log length
constexpr uint32_t LP_LOG = 15;   // state word holding the final-log length
// state word set (k_lpubnb) on every batch publisher and its mesh (churn: CSR)
// neighbours: only those rows' emit step needs the publishers (LPullArgs::pubw)
constexpr uint32_t LP_PUB = 12;
static_assert(LP_KMAX <= LP_PUB && LP_PUB < LP_LOG, "row state words");
// arrival record (u64): start - window_lo (32) | hops (6) | inclusion mask (16) | lane (10)
constexpr uint32_t LP_IM_SHIFT = 10, LP_HOP_SHIFT = 26, LP_LANE_MASK = (1u << LP_IM_SHIFT) - 1;
static_assert(MESH_W <= LP_HOP_SHIFT - LP_IM_SHIFT && PULL_LMAX <= (1u << LP_IM_SHIFT) && HOP_BITS == 32 - LP_HOP_SHIFT,
              "record fields");

struct LPullArgs {
  uint64_t* keys;       // [N][L] final log during the passes; dense again after k_lfinal
  uint16_t* flane;      // [N][L] lane of each log entry
  uint64_t* busy;       // [N][B] uplink FIFO end per (peer, message), FP > 1
  uint64_t* blk;        // [K][N][ls] candidate lists per destination-window slot
  uint32_t* st;         // [N][LP_SW]
  uint32_t* fin;        // [N][64] u16 final bits, transposed: u16 j bit q = lane q*64 + j
  uint64_t* lrec;       // [2][N][L] per-row arrival records (k_pull's format)
  uint32_t* lcnt;       // [2][N]
  const uint32_t* mesh;
  const uint8_t* rpos;
  const uint32_t* pub;
  const uint8_t* stage;
  const uint32_t* tables;
  uint64_t* ctrl;       // [3][4] k_pull's pass control slots
  uint64_t* counters;
  uint64_t delta, tmax;
  uint32_t N, B, L, S, sb, tshift, pass, K, lb, dG;  // lb = lane bits, dG = Delta in key hi-word grains
  uint32_t ls, lcap;  // list stride (max(L, 256) entries) and capacity (ls; GS_LPULL_CAP lowers it)
  uint32_t idw;       // IDONTWANT batch (k_lpull<.., true>): finals go to dense keys[N][L], no log
  uint32_t self_log;  // k_lcomplete's latency stream: the publisher logs its own message
  uint64_t rmax;      // largest arrival offset of a forward after the lane's final time (the fragment
                      // FIFO + lat + dn + MESH_W ser): the emit step checks start + rmax <= tmax, so
                      // receivers need no time check
  // peer-partitioned pass (k_lpull<.., .., .., true>, gs_run_partitioned): this context's rows are
  // global peers [u0, u0 + N); every per-row array above is indexed by the local row, lrec / lcnt
  // receive only this part's records, and the previous pass's records of EVERY peer arrive packed
  // (rpk) with per-peer offsets (roff) and counts (rcg), exchanged by the host (gs_comm.hip)
  uint32_t u0;
  // batch slices (gs_relax.hip run_slices): rows [j * rN, (j + 1) * rN) are slice j, a
  // whole batch of its own over a copy of the graph (ids + j * rN); pub holds the
  // slices' publishers [S][B] as such row ids. 0: one batch
  uint32_t rN;
  uint32_t pubw;  // the LP_PUB state words are set (k_lpubnb): a row without it skips the publisher load
  uint32_t F, collide;  // k_lcomplete: fragments per message, defect D8 (no fragment group completes)
  const uint64_t* rpk;
  const uint64_t* roff;
  const uint32_t* rcg;
  // lazy gossip inside the passes (k_lpull<.., GOS>, k_lctl, k_gsend):
  // a lockstep batch (every message's heartbeat k at the same relative time
  // grel0 + k * ghb) on the frozen mesh, rows of single-fragment lanes
  uint64_t grel0, ghb;        // heartbeats, relative to every t_pub
  uint64_t glat_min, glat_max;  // IHAVE travel time bounds over the used link classes
  uint64_t gnf;               // non-publisher lanes of the batch, B * (N - 1)
  uint64_t gseed;
  uint32_t ghist, gd_lazy, ggf;  // history_gossip, D_lazy, gossip factor x 1000
  uint64_t* gctl;             // [GC_WORDS] pass and heartbeat control (k_lctl)
  uint32_t* gpl;              // [N][LP_FW] sender planes of the built heartbeat (fin's transposed layout)
  uint64_t* gse;              // [N][L] their entries in rank order: target mask | sender hops << 58
  uint32_t* rowdone;          // [(N + 31) / 32] rows whose every lane is final
  const uint64_t* row;        // CSR (non-mesh connections are the IHAVE peers)
  const uint32_t* col;
  const uint8_t* flags;
  const uint8_t* csrpos;      // position of the row's peer in its neighbour's row
  const uint64_t* habs0;      // [B] absolute index of each message's heartbeat 0
  // churn on the list pass (k_lpull<1, CH, false, false, GOS, true>; gs_cpull.h): a lockstep
  // batch whose lane m at relative time t is in epoch E0 + cq[m] + k(t), k(t) = floor((cr0 + t) / chb)
  const uint32_t* ccol;  // [N][64] CSR rows, stage << 24 | peer, EMPTY padded (the row header)
  const uint8_t* cpos;   // [N][64] position of the row's peer in that neighbour's CSR row
  const uint64_t* cmm;   // [N][cE] mesh of each epoch as a mask over the row's CSR entries
  const uint64_t* cgt;   // [N][cE] IHAVE targets per epoch, a mask over the CSR row (lazy gossip)
  const uint32_t* coff;  // [chz + 2][N][LP_FW] offline lanes per relative epoch (fin's layout)
  const uint32_t* cq;    // [B]
  const uint8_t* pubok;  // [B] the publisher was online at t_pub (k_lpub; nullptr: all)
  uint8_t* gnz;          // [N] GOS: the row's plane of the built heartbeat has a lane (k_gsend)
  uint16_t* gtag;        // [N] GOS: = GC_BK when a plane of the built heartbeat targets the row
  uint32_t gsw;          // CHN + GOS: heartbeats k >= gsw push their IHAVEs into the targets' lists
                         // (k_gsend: only those a target may still need, per-target cap); k < gsw:
                         // every target scans the planes
  uint32_t* gpc;         // [N] CHN + GOS: IHAVE entries pushed to the row this heartbeat, bk << 16 | count
  const uint32_t* calive;  // [LP_FW] churn: the published lanes (publisher online at t_pub), fin's layout
  uint64_t* luni;        // [2][N] per pass: OR of the receiver masks of a row's records (a receiver
                         // reads a neighbour's records only when its own bit is set)
  uint64_t cr0, chb;
  uint32_t cE, chz;      // epochs per row of cmm / cgt; the lifetime in epochs (churn_horizon)
  uint32_t ghoff;        // GOS: relative epoch of heartbeat 0 (habs0 - q0: 0 or 1)
  uint32_t ghk;          // GOS: last heartbeat index whose IHAVEs are inside the lifetime (~0u: no cap)
};

// gctl words (k_lctl writes them between passes; k_gsend / k_lpull only read)
enum : uint32_t {
  GC_FD0 = 0,    // counters[C_FD] at the start of the batch
  GC_TLAST = 1,  // bound on the latest final time: the end of the last window that finalised a lane
  GC_E = 2,      // end of the last emitted window
  GC_DONE = 3,   // the batch's passes are over
  GC_GB = 4,     // next heartbeat whose senders are not yet known final
  GC_BK = 5,     // heartbeat + 1 whose sender planes are built (0: none)
  GC_BUILD = 6,  // heartbeat + 1 to build before this pass (0: none)
  GC_GW = 7,     // this pass's window holds IHAVE arrivals of heartbeat GC_BK - 1
  GC_FDP = 8,    // counters[C_FD] at the previous decision
  GC_WORDS = 9
};
constexpr uint32_t GSE_HOPS = 58;  // entry bits [0, 58): target mask over the sender's CSR row

constexpr uint32_t LP_FW = PULL_LMAX / 32;  // u32 final-bit words per row
constexpr uint32_t CELL_W = 64;             // churn: CSR entries per 64-wide ELL row header (the mask width)
// churn records (CHN) are 16 B: the word above with the 16 mask bits unused, then
// the sender's 64-bit receiver mask over its CSR row

__device__ __forceinline__ uint32_t sat32(uint64_t x) { return x > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)x; }

// Offset of key hi word hx from the emitted window c (window c + k starts at
// hi word sat32(hlo64 + k * dG)); for the saturated end of the time range only,
// where the division of the pass does not apply.
__device__ __forceinline__ uint32_t lp_rof(uint32_t hx, uint64_t hlo64, uint32_t dG, uint32_t K) {
  uint32_t r = 0;
  for (uint32_t k = 1; k <= K; k++) r += hx >= sat32(hlo64 + (uint64_t)k * dG) ? 1u : 0u;
  return r;  // r == K: beyond the ring (an error the host bound rules out)
}

// LDS of the pass per wave: CW = the row's candidate minima (CH 64-lane
// chunks), LST = compacted lane / group indices. CH = 16: 10 KB per wave, 4
// blocks (16 waves) per CU; CH = 8 (rows of <= 512 lanes): 5 KB, 8 blocks.
template <uint32_t CH>
struct LPullLds {
  uint64_t cw[PULL_WAVES][CH * 64];
  uint16_t lst[PULL_WAVES][CH * 64];
};

// Listed entries e[0..3] (entry = toff << (tshift + lb) | low << lb | lane, so
// key = (wlo << tshift) + (entry >> lb)) into the row's candidate minima. Bit 63
// marks an IHAVE entry (churn + lazy gossip, heartbeats >= gsw: glp_ihave_ent),
// not a candidate; the host keeps every entry below bit 63.
__device__ __forceinline__ void lp_apply_entries(uint64_t* CW, const uint64_t (&e)[4], uint32_t lmask, uint32_t lb,
                                                 uint64_t wlok, uint32_t& cb) {
#pragma unroll
  for (int u = 0; u < 4; u++) {
    if (e[u] >> 63) continue;  // no entry (~0) or an IHAVE entry
    const uint32_t li = (uint32_t)e[u] & lmask;
    atomicMin((unsigned long long*)&CW[li], (unsigned long long)(wlok + (e[u] >> lb)));
    cb |= 1u << (li >> 6);
  }
}

// ---- lazy gossip inside the passes (GOS batches) ----
//
// IHAVE rules (libp2p-gossipsub emit_gossip / handle_ihave / handle_iwant,
// upstream; gossip_lazy / gossip_factor at rust-test-node/src/main.rs:230,235;
// the oracle's sched_gossip): a peer v that first received m at t_v gossips
// it at the history_gossip heartbeats R_k >= t_v to the r smallest
// rng(GOSSIP, v, h, x) of its non-mesh connections x; the IHAVE reaches w at
// t_i = R_k + lat(v -> w); unless w holds m by t_i, w sends IWANT and v's
// answer arrives lat(w -> v) + ser_up(v) + lat(v -> w) + dn later with v's
// hops + 1 and src v. In a lockstep batch R_k is one relative time for every
// message, windows are no wider than the smallest latency (t_i never shares a
// window with R_k), so before the first pass that can see heartbeat k's IHAVEs
// every sender of k is final: k_gsend writes each row's sender plane (which
// lanes v gossips at k) and its entries (the lane's target mask over v's CSR
// row, v's hops), and the passes decide the IHAVEs receiver-side (glp_ihave).

// IHAVE targets of v at heartbeat h among its non-mesh connections (bit e of
// nmm: CSR entry e, held by lane e in x): the r smallest (rng, id) pairs, as a
// mask over v's CSR row. The CSR walk is wave-uniform, h is the lane's own.
// pre = rng_pre(seed, P_GOSSIP, v): one mix per candidate.
__device__ __forceinline__ uint64_t glp_targets(uint64_t pre, uint32_t h, uint32_t x, uint64_t nmm, uint32_t deg,
                                                uint32_t r) {
  auto lt = [](uint64_t k1, uint32_t w1, uint64_t k2, uint32_t w2) { return k1 < k2 || (k1 == k2 && w1 < w2); };
  uint64_t kk[GT_W];
  uint32_t ww[GT_W], pp[GT_W];
#pragma unroll
  for (int q = 0; q < (int)GT_W; q++) { kk[q] = INF64; ww[q] = ~0u; pp[q] = 0; }
  for (uint32_t e = 0; e < deg; e++) {
    if (!((nmm >> e) & 1)) continue;  // wave-uniform
    const uint32_t w = __builtin_amdgcn_readlane(x, e);
    const uint64_t rk = rng_fin(pre, h, w);
    if (!lt(rk, w, kk[GT_W - 1], ww[GT_W - 1])) continue;
#pragma unroll
    for (int q = (int)GT_W - 1; q > 0; q--) {  // insert, shifting the larger pairs up
      if (lt(rk, w, kk[q - 1], ww[q - 1])) { kk[q] = kk[q - 1]; ww[q] = ww[q - 1]; pp[q] = pp[q - 1]; }
      else if (lt(rk, w, kk[q], ww[q])) { kk[q] = rk; ww[q] = w; pp[q] = e; }
    }
    if (lt(rk, w, kk[0], ww[0])) { kk[0] = rk; ww[0] = w; pp[0] = e; }
  }
  uint64_t mask = 0;
#pragma unroll
  for (int q = 0; q < (int)GT_W; q++)
    if ((uint32_t)q < r) mask |= 1ull << pp[q];
  uint64_t pk = kk[GT_W - 1];
  uint32_t pw = ww[GT_W - 1];
  for (uint32_t q = GT_W; q < r; q++) {  // rare: more than GT_W targets, the next pair by a rescan
    uint64_t bk = INF64;
    uint32_t bw = ~0u, bp = 0;
    for (uint32_t e = 0; e < deg; e++) {
      if (!((nmm >> e) & 1)) continue;
      const uint32_t w = __builtin_amdgcn_readlane(x, e);
      const uint64_t rk = rng_fin(pre, h, w);
      if (lt(pk, pw, rk, w) && lt(rk, w, bk, bw)) { bk = rk; bw = w; bp = e; }
    }
    mask |= 1ull << bp;
    pk = bk;
    pw = bw;
  }
  return mask;
}

// Receiver side, row w in a window c = [wlo, wlo + Delta) holding IHAVE
// arrivals of heartbeat k (at gR): every non-mesh connection v whose t_i =
// gR + lat(v -> w) lies in c offers the lanes of its plane; for a lane of w
// not final before c that v targets, CW (the window's entries and records)
// says whether w has the message by t_i — if not, IWANT, and v's answer goes
// into CW as a candidate (it lands after window c).
__device__ __forceinline__ void glp_ihave(const LPullArgs& a, uint64_t* CW, uint32_t w, uint32_t sw, uint32_t finT,
                                          uint64_t wlo, uint64_t gR, const uint32_t* lat, const uint32_t* sup,
                                          const uint32_t* sdn, uint32_t& cb, uint64_t& niw, uint32_t& err) {
  const int lane = threadIdx.x & 63;
  const uint32_t S = a.S;
  wave_lds_sync();  // the window's entries and records are in CW
  // batch slices: the CSR by the peer (w - soff), the senders' planes by their slice rows
  const uint32_t soff = a.rN ? (w / a.rN) * a.rN : 0u;
  const uint64_t rb = a.row[w - soff], deg = a.row[w - soff + 1] - rb;  // the host checked deg <= GSE_HOPS
  uint32_t vx = 0, cp = 0, tio = 0, aoff = 0;
  bool ok = false;
  if ((uint64_t)lane < deg) {
    vx = a.col[rb + lane];
    const uint8_t fl = a.flags[rb + lane];
    cp = a.csrpos[rb + lane];
    const uint32_t sv = a.stage[vx];
    tio = lat[sv * S + sw];  // t_i - R_k
    const uint64_t ti = gR + tio;
    ok = !(fl & F_MESH) && ti >= wlo && ti < wlo + a.delta;
    const uint32_t su = sup[sv], sd = sdn[sw];
    aoff = lat[sw * S + sv] + su + tio + (sd > su ? sd - su : 0u);  // IWANT + answer: t_i -> arrival
  }
  uint64_t gm = __ballot(ok);
  const uint32_t nfl = ~finT & 0xFFFFu;  // lanes not final before window c
  while (gm) {  // wave-uniform: one IHAVE sender at a time
    const int e = __builtin_ctzll(gm);
    gm &= gm - 1;
    const uint32_t v = __builtin_amdgcn_readlane(vx, e) + soff;
    const uint32_t p = __builtin_amdgcn_readlane(cp, e);
    const uint64_t ti = gR + (uint32_t)__builtin_amdgcn_readlane(tio, e);
    const uint64_t A = ti + (uint32_t)__builtin_amdgcn_readlane(aoff, e);
    const uint32_t plj = reinterpret_cast<const uint16_t*>(a.gpl + (size_t)v * LP_FW)[lane];
    uint32_t c = plj & nfl;
    if (__ballot(c != 0) == 0) continue;
    // rank of (lane j, bit q) among v's entries: the lanes below j first, then q ascending
    const uint32_t own = (uint32_t)__popc(plj);
    uint32_t pre = own;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(pre, off);
      if (lane >= off) pre += y;
    }
    pre -= own;
    const uint64_t* ge = a.gse + (size_t)v * a.L;
    const uint64_t kb = (A << a.tshift) | v;
    const bool tbad = A > a.tmax;
    while (c) {
      const int q = __builtin_ctz(c);
      c &= c - 1;
      const uint64_t en = ge[pre + (uint32_t)__popc(plj & ((1u << q) - 1u))];
      if (!((en >> p) & 1)) continue;  // w is not among v's targets at heartbeat k
      const uint32_t i = (uint32_t)q * 64 + lane;
      const uint64_t x = CW[i];
      if (x != INF64 && (x >> a.tshift) <= ti) continue;  // w has it by t_i (arrivals first at equal time)
      niw++;
      const uint32_t hv = (uint32_t)(en >> GSE_HOPS) + 1;
      if (hv >= (1u << HOP_BITS)) err |= ERR_HOPS;
      if (tbad) err |= ERR_TIME;
      atomicMin((unsigned long long*)&CW[i], (unsigned long long)(kb | ((uint64_t)hv << a.sb)));
      cb |= 1u << q;
    }
  }
}

// Receiver side under churn (CHN): the epoch's mesh differs per lane, so every
// CSR neighbour v (lane e of the row header: ej / rj) may send IHAVEs; v's entry
// says whether w is a target (targets are online connections outside v's mesh
// at the heartbeat's epoch kh), lanes where w is offline at kh get none (offh),
// and an answer landing at or after gB1 (the start of epoch kh + 1) is lost
// where w is offline then or past the lifetime (offa): no IWANT is counted for
// it (the oracle's lost_a).
__device__ __forceinline__ void glp_ihave_chn(const LPullArgs& a, uint64_t* CW, uint32_t sw, uint32_t nfl, uint64_t wlo,
                                              uint64_t gR, uint32_t ej, uint32_t rj, uint32_t offa,
                                              uint64_t gB1, const uint32_t* lat, const uint32_t* sup,
                                              const uint32_t* sdn, uint32_t& cb, uint64_t& niw, uint32_t& err) {
  const int lane = threadIdx.x & 63;
  const uint32_t S = a.S;
  wave_lds_sync();  // the window's entries and records are in CW
  uint32_t tio = 0, aoff = 0;
  bool ok = false;
  if (ej != EMPTY) {
    const uint32_t sv = ej >> STAGE_SHIFT;
    tio = lat[sv * S + sw];  // t_i - R_k
    const uint64_t ti = gR + tio;
    // a sender whose plane is empty (k_gsend's gnz) offers nothing
    ok = ti >= wlo && ti < wlo + a.delta && a.gnz[ej & 0xFFFFFFu];
    const uint32_t su = sup[sv], sd = sdn[sw];
    aoff = lat[sw * S + sv] + su + tio + (sd > su ? sd - su : 0u);  // IWANT + answer: t_i -> arrival
  }
  uint64_t gm = __ballot(ok);
  constexpr int GV = 8;  // senders whose plane loads are in flight together
  while (gm) {  // wave-uniform
    uint32_t V[GV], P[GV], PL[GV];
    int E[GV];
    int nv = 0;
#pragma unroll
    for (int q = 0; q < GV; q++) {
      E[q] = gm ? __builtin_ctzll(gm) : 0;
      if (gm) { gm &= gm - 1; nv = q + 1; }
      V[q] = __builtin_amdgcn_readlane(ej, E[q]) & 0xFFFFFFu;
      P[q] = __builtin_amdgcn_readlane(rj, E[q]);
    }
#pragma unroll
    for (int q = 0; q < GV; q++)
      PL[q] = q < nv ? reinterpret_cast<const uint16_t*>(a.gpl + (size_t)V[q] * LP_FW)[lane] : 0u;
#pragma unroll
    for (int q = 0; q < GV; q++) {
      const uint32_t plj = PL[q];
      uint32_t c = plj & nfl;
      if (__ballot(c != 0) == 0) continue;  // wave-uniform (also q >= nv)
      const uint32_t v = V[q], p = P[q];
      const uint64_t ti = gR + (uint32_t)__builtin_amdgcn_readlane(tio, E[q]);
      const uint64_t A = ti + (uint32_t)__builtin_amdgcn_readlane(aoff, E[q]);
      c &= ~(A >= gB1 ? offa : 0u);  // lanes whose answer reaches w offline / past the lifetime
      const uint64_t* ge = a.gse + (size_t)v * a.L + lane;  // v's entry of lane q*64 + lane: ge[q * 64]
      const uint64_t kb = (A << a.tshift) | v;
      const bool tbad = A > a.tmax;
      while (c) {  // four of the lane's entries per round trip
        int qv[4];
        uint64_t en[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
          qv[t] = c ? __builtin_ctz(c) : -1;
          c &= c ? c - 1 : 0u;
          en[t] = qv[t] >= 0 ? ge[(size_t)qv[t] * 64] : 0ull;
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
          if (qv[t] < 0 || !((en[t] >> p) & 1)) continue;  // w is not among v's targets at heartbeat k
          const uint32_t i = (uint32_t)qv[t] * 64 + lane;
          const uint64_t x = CW[i];
          if (x != INF64 && (x >> a.tshift) <= ti) continue;  // w has it by t_i (arrivals first at equal time)
          niw++;
          const uint32_t hv = (uint32_t)(en[t] >> GSE_HOPS) + 1;
          if (hv >= (1u << HOP_BITS)) err |= ERR_HOPS;
          if (tbad) err |= ERR_TIME;
          atomicMin((unsigned long long*)&CW[i], (unsigned long long)(kb | ((uint64_t)hv << a.sb)));
          cb |= 1u << qv[t];
        }
      }
    }
  }
}

// Pushed IHAVE entries (churn, heartbeats k >= gsw): k_gsend appended, for
// every (sender v, lane m, target w), an entry t_i | hops + 1 | v | m flagged
// by bit 63 to w's list of the window holding t_i. With the window's entries
// and records in CW, w decides as glp_ihave does: no IWANT when the lane is
// final before the window or CW holds a time <= t_i; else IWANT (counted
// unless the answer lands in the next epoch where w is offline, or past the
// lifetime), and v's answer at t_i + lat(w -> v) + ser_up(v) + lat(v -> w) + dn
// is one more candidate.
__device__ __forceinline__ void glp_ihave_ent(const LPullArgs& a, uint64_t* CW, uint32_t w, uint32_t sw, uint32_t finT,
                                              const uint64_t* lst, uint32_t due, uint64_t wlok, const uint32_t* lat,
                                              const uint32_t* sup, const uint32_t* sdn, uint32_t& cb, uint64_t& niw,
                                              uint32_t& err) {
  const int lane = threadIdx.x & 63;
  const uint32_t S = a.S, lmask = (1u << a.lb) - 1;
  const uint64_t smask = (1ull << a.sb) - 1;
  // a row the pushes of the built heartbeat overflowed scans its neighbours'
  // planes instead (glp_ihave_chn): its pushed entries of that heartbeat are
  // left to the scan (pushed entries are taken while GC_BK is their heartbeat's)
  if (a.gtag[w] == (uint16_t)a.gctl[GC_BK]) return;
  wave_lds_sync();
  for (uint32_t f0 = 0; f0 < due; f0 += 64) {
    const uint32_t f = f0 + lane;
    const uint64_t en = f < due ? lst[f] : 0ull;
    const bool ih = (en >> 63) != 0;
    if (__ballot(ih) == 0) continue;
    const uint32_t li = ih ? (uint32_t)en & lmask : 0u;
    // lane li's final bit lives in lane li & 63 (bit li >> 6)
    const uint32_t fb = (uint32_t)__shfl((int)finT, (int)(li & 63u));
    if (!ih || ((fb >> (li >> 6)) & 1u)) continue;  // final before window c: w has it
    const uint64_t key = wlok + ((en & ~(1ull << 63)) >> a.lb);
    const uint64_t ti = key >> a.tshift;
    const uint64_t x = CW[li];
    if (x != INF64 && (x >> a.tshift) <= ti) continue;  // w has it by t_i
    const uint32_t v = (uint32_t)(key & smask), hv = (uint32_t)(key >> a.sb) & ((1u << HOP_BITS) - 1);
    const uint32_t sv = a.stage[v];
    const uint32_t su = sup[sv], sd = sdn[sw];
    const uint64_t A = ti + lat[sw * S + sv] + su + lat[sv * S + sw] + (sd > su ? sd - su : 0u);
    const uint64_t kt = udiv53(a.cr0 + ti, a.chb), B1 = (kt + 1) * a.chb - a.cr0;
    if (A >= B1) {  // the answer lands in epoch kt + 1: lost where w is offline then (or past the lifetime)
      const uint32_t ko = kt + 1 <= a.chz + 1 ? (uint32_t)kt + 1 : a.chz + 1;
      const uint32_t ob = reinterpret_cast<const uint16_t*>(a.coff + ((size_t)ko * a.N + w) * LP_FW)[li & 63u];
      if ((ob >> (li >> 6)) & 1u) continue;
    }
    niw++;
    if (A > a.tmax) err |= ERR_TIME;
    atomicMin((unsigned long long*)&CW[li], (unsigned long long)((A << a.tshift) | ((uint64_t)hv << a.sb) | v));
    cb |= 1u << (li >> 6);
  }
}

// Record step: groups of NG = 4 neighbours, RCH = 2 chunks of 64 records each
// per iteration (8 loads in flight per lane; 8 x 64 measured 2 % slower,
// profiles/r03_v1/ab_record_groups.txt). GS_LP_NG / GS_LP_RCH: A/B builds.
#ifndef GS_LP_NG
#define GS_LP_NG 4
#endif
#ifndef GS_LP_NT  // nontemporal stores of the final log (A/B: -DGS_LP_NT=0)
#define GS_LP_NT 1
#endif
#ifndef GS_LP_NTR  // nontemporal stores of the records (A/B variant; off)
#define GS_LP_NTR 0
#endif
#ifndef GS_LP_RCH
#define GS_LP_RCH 2
#endif
#ifndef GS_LP_SKIP  // record chunks past a neighbour's count skipped by a scalar branch (off: +1.3 % per step, r06)
#define GS_LP_SKIP 0
#endif
template <int FP, uint32_t CH, bool IDW = false, bool PART = false, bool GOS = false, bool CHN = false>
__global__ __launch_bounds__(TB, (CH <= 8 ? 6 : 4)) void k_lpull(LPullArgs a) {
  constexpr uint32_t NG = GS_LP_NG, RCH = GS_LP_RCH;
  static_assert(!IDW || FP == 1, "IDONTWANT on the list pass: rows of single-fragment lanes");
  static_assert(!GOS || !PART, "gossip on the list pass: gs_run's rows");
  static_assert(!CHN || (!IDW && !PART), "churn on the list pass: gs_run's rows (fragment groups included)");
  // row header: the mesh row (frozen mesh) or, under churn, the CSR row (the
  // mesh of a lane's epoch is a mask over it)
  constexpr uint32_t HW = CHN ? CELL_W : MESH_W;
  constexpr uint32_t LMAX = CH * 64;
  __shared__ LPullLds<CH> Ls;
  uint64_t* me = a.ctrl + (a.pass % 3) * 4;
  uint64_t lo, mode;
  if constexpr (GOS) {  // k_lctl decided this pass (gossip windows need the heartbeat state)
    lo = me[0];
    mode = me[1];
  } else {  // ---- decide this pass from the previous slot (grid-uniform; k_pull's rule) ----
    const uint64_t* pv = a.ctrl + ((a.pass + 2) % 3) * 4;
    if (pv[1] != PM_DONE && pv[2]) { mode = PM_PULL; lo = pv[1] == PM_PULL ? pv[0] + a.delta : pv[0]; }
    else if (pv[3] != INF64) { mode = PM_EMIT; lo = ((pv[3] >> a.tshift) / a.delta) * a.delta; }
    else { mode = PM_DONE; lo = pv[0]; }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      me[0] = lo;
      me[1] = mode;
      uint64_t* nx = a.ctrl + ((a.pass + 1) % 3) * 4;
      nx[2] = 0;
      nx[3] = INF64;
      if (mode != PM_DONE) atomicAdd((unsigned long long*)&a.counters[C_PASSES], 1ull);
      if (mode == PM_PULL) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
    }
  }
  if (mode == PM_DONE) return;

  const bool pull = mode == PM_PULL;
  const uint64_t wlo = pull ? lo + a.delta : lo;  // the window this pass emits
  const uint64_t c = wlo / a.delta;                // its index (scalar division, once)
  const uint32_t K = a.K, LL = a.L, S = a.S;
  const uint32_t cslot = (uint32_t)(c % K);
  const uint64_t hlo64 = c * a.dG;
  const uint32_t hlo = sat32(hlo64), hspan = a.dG;  // hi words of window c: [hlo, hlo + dG)
  // window offsets of pending minima by division when no threshold of the
  // ring saturates (lp_rof's count of window starts <= hx is then floor((hx - hlo) / dG))
  const bool rdiv = hlo64 + (uint64_t)(K + 1) * a.dG < 0xFFFFFFFFull;
  const float rinv = 1.0f / (float)a.dG;
  const size_t NL = (size_t)a.N * LL;
  const uint32_t pb = (a.pass + 1) & 1, nb = a.pass & 1;  // records read / written
  constexpr uint32_t RW = CHN ? 2 : 1;  // u64 words per record
  const uint64_t* rrec = PART ? a.rpk : a.lrec + pb * NL * RW;
  const uint32_t* rcnt = PART ? a.rcg : a.lcnt + (size_t)pb * a.N;  // indexed by global peer id
  uint64_t* wrec = a.lrec + nb * NL * RW;
  const uint64_t* runi = CHN ? a.luni + (size_t)pb * a.N : nullptr;
  uint64_t* wuni = CHN ? a.luni + (size_t)nb * a.N : nullptr;
  uint32_t* wcnt = a.lcnt + (size_t)nb * a.N;
  const uint32_t* lat = a.tables;
  const uint32_t* sup = a.tables + S * S;
  const uint32_t* sdn = a.tables + S * S + S;
  // lazy gossip: does this window hold IHAVE arrivals of the built heartbeat (k_lctl)?
  bool gw = false;
  uint64_t gR = 0;  // that heartbeat, relative to every t_pub
  uint16_t gbk = 0;  // CHN: the gtag of rows the built heartbeat's planes target
  if constexpr (GOS) {
    gw = a.gctl[GC_GW] != 0;
    gR = a.grel0 + (a.gctl[GC_BK] - 1) * a.ghb;
    gbk = (uint16_t)a.gctl[GC_BK];
  }
  uint64_t niw = 0;  // IWANTs sent
  // churn (CHN): the epoch boundaries the pass can meet. A record landing at
  // or after xBs (time) is lost where the receiver is offline in ks + 1 (offn):
  // a sender that received in ks used ks's mesh (peers online in ks), one that
  // received in ks + 1 only reaches peers online then, so the test needs no
  // sender epoch (with fragments the uplink FIFO can start a send of a lane
  // received in ks after xBs; rmax covers that FIFO). Window c
  // starts in relative epoch kc and, when it straddles a boundary, its lanes
  // final at or after eBc forward with the mesh of kc + 1.
  uint64_t xBs = INF64, eBc = INF64;
  uint32_t kc = 0;
  const uint32_t* offn = nullptr;
  uint32_t gkh = 0;     // GOS + CHN: relative epoch of the built heartbeat
  uint32_t calT = 0;    // GOS + CHN: the published lanes (lane j: bit q = lane q*64 + j)
  uint64_t gB1 = INF64;  // its next epoch's start (relative time)
  if constexpr (CHN) {
    const uint64_t ks = udiv53(a.cr0 + lo, a.chb), Bs = (ks + 1) * a.chb - a.cr0;
    if (pull && Bs < lo + a.delta + a.rmax) {
      xBs = Bs << a.tshift;
      offn = a.coff + (size_t)(ks + 1 <= a.chz + 1 ? ks + 1 : a.chz + 1) * a.N * LP_FW;
    }
    kc = (uint32_t)udiv53(a.cr0 + wlo, a.chb);
    const uint64_t Bc = ((uint64_t)kc + 1) * a.chb - a.cr0;
    if (Bc < wlo + a.delta) eBc = Bc;
    if constexpr (GOS) {
      calT = reinterpret_cast<const uint16_t*>(a.calive)[threadIdx.x & 63];
      gkh = a.ghoff + (uint32_t)(a.gctl[GC_BK] ? a.gctl[GC_BK] - 1 : 0);
      if (gkh > a.chz) gkh = a.chz;
      gB1 = ((uint64_t)gkh + 1) * a.chb - a.cr0;
    }
  }

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* CW = Ls.cw[wv];
  uint16_t* LST = Ls.lst[wv];
  const uint64_t smask = (1ull << a.sb) - 1;
  const uint32_t hmask = (1u << HOP_BITS) - 1;
  const uint64_t lanelt = (1ull << lane) - 1;
  const uint64_t lowmask = (1ull << a.tshift) - 1;
  // per state lane j < K: the window its counter slot stands for, as a hi word
  const uint32_t lwin = lane < (int)K ? (uint32_t)(((uint32_t)lane + K - cslot) % K) : 0u;
  const uint32_t lwhi = sat32(hlo64 + (uint64_t)lwin * a.dG);
  uint64_t fd = 0, nr = 0, np = 0, nrec = 0;
  uint32_t nmh = ~0u;
  uint32_t err = 0;
#ifdef GS_PULL_PROF
  uint64_t pp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

#pragma unroll
  for (int q = 0; q < (int)CH; q++) CW[q * 64 + lane] = INF64;
  wave_lds_sync();

  // The wave's rows are w0 + k * stride (local row; global peer a.u0 + w), taken
  // 64 at a time: step 0 finds, one row per lane, the rows with something to do
  // in this pass, and the wave visits only those (the near-empty first and last
  // passes of a batch would otherwise walk every row header one row at a time).
  const uint32_t stride = gridDim.x * PULL_WAVES;
  for (uint32_t base = blockIdx.x * PULL_WAVES + wv; base < a.N; base += 64 * stride) {
  // 0. lane l: row base + l * stride is active if a neighbour sent records
  //    (PULL), entries are due in window c, or it may take IHAVEs (a gossip
  //    window, a lane not final); an inactive row is only booked: no records
  //    from it next pass, its pending windows into nmh
  uint64_t am;
  {
    const uint32_t wl = base + (uint32_t)lane * stride;
    bool act = false;
    if (wl < a.N) {
      const uint4* sp = reinterpret_cast<const uint4*>(a.st + (size_t)wl * LP_SW);
      uint32_t s4[LP_KMAX];
#pragma unroll
      for (int k = 0; k < (int)LP_KMAX / 4; k++) {
        const uint4 v = sp[k];
        s4[k * 4] = v.x; s4[k * 4 + 1] = v.y; s4[k * 4 + 2] = v.z; s4[k * 4 + 3] = v.w;
      }
      // the nearest pending window; cs and kk pass through an empty asm so that
      // the per-slot offsets and tests are computed here, not hoisted out of the
      // row loop (24 more scalars live across every row: SGPR spills)
      uint32_t cs = cslot, kk = K, mo = ~0u;
      asm volatile("" : "+s"(cs), "+s"(kk));
#pragma unroll
      for (uint32_t j = 0; j < LP_KMAX; j++) {
        if (j >= kk || !s4[j]) continue;
        act |= j == cs;
        mo = umin32(mo, j >= cs ? j - cs : j + kk - cs);
      }
      const uint32_t mh = mo == ~0u ? ~0u : sat32(hlo64 + (uint64_t)mo * a.dG);
      if (GOS && gw) act |= !((a.rowdone[wl >> 5] >> (wl & 31)) & 1u) && (!CHN || a.gtag[wl] == gbk);
      if (pull && !act) {
        if constexpr (CHN) {  // CSR rows, 16 entries at a time until the padding
          const uint4* mp = reinterpret_cast<const uint4*>(a.ccol + (size_t)wl * CELL_W);
          for (int g = 0; g < (int)CELL_W / 16 && !act; g++) {
            uint32_t e[16];
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const uint4 m = mp[g * 4 + k];
              e[4 * k] = m.x; e[4 * k + 1] = m.y; e[4 * k + 2] = m.z; e[4 * k + 3] = m.w;
            }
#pragma unroll
            for (int u = 0; u < 16; u++)
              if (e[u] != EMPTY) act |= rcnt[e[u] & 0xFFFFFFu] != 0;
            if (e[15] == EMPTY) break;
          }
        } else {
          const uint4* mp = reinterpret_cast<const uint4*>(a.mesh + (size_t)(a.u0 + wl) * MESH_W);
#pragma unroll
          for (int k = 0; k < (int)MESH_W / 4; k++) {
            const uint4 m = mp[k];
            const uint32_t e[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
            for (int u = 0; u < 4; u++)
              if (e[u] != EMPTY) act |= rcnt[e[u] & 0xFFFFFFu] != 0;
          }
        }
      }
      if (!act) {
        wcnt[wl] = 0;
        nmh = umin32(nmh, mh);
      }
    }
    am = __ballot(act);
  }
  uint32_t w = a.N, wn = a.N;
  if (am) {
    w = base + (uint32_t)__builtin_ctzll(am) * stride;
    am &= am - 1;
  }
  uint32_t ej = EMPTY, cj = 0, rj = 0, sv = 0;
  uint64_t ro = 0, ro2 = 0;  // PART: offsets of the neighbours' packed records
  if constexpr (CHN) {
    if (w < a.N) {
      ej = a.ccol[(size_t)w * CELL_W + lane];
      rj = a.cpos[(size_t)w * CELL_W + lane];
      if (pull && ej != EMPTY) {
        cj = rcnt[ej & 0xFFFFFFu];
        if (!((runi[ej & 0xFFFFFFu] >> (rj & 63u)) & 1)) cj = 0;  // no record of it is for w
      }
      if (lane < (int)LP_SW) sv = a.st[(size_t)w * LP_SW + lane];
    }
  } else if (w < a.N && lane < (int)MESH_W) {
    ej = a.mesh[(size_t)(a.u0 + w) * MESH_W + lane];
    rj = a.rpos[(size_t)(a.u0 + w) * MESH_W + lane];
    if (pull && ej != EMPTY) {
      cj = rcnt[ej & 0xFFFFFFu];
      if constexpr (PART) ro = a.roff[ej & 0xFFFFFFu];
    }
    sv = a.st[(size_t)w * LP_SW + lane];
  }
  uint32_t dw = 0;  // gossip windows: the row-done word of row w (every lane reads it)
  if (GOS && gw && w < a.N) dw = a.rowdone[w >> 5];
  for (; w < a.N; w = wn) {
    PP_T(tA);
    wn = am ? base + (uint32_t)__builtin_ctzll(am) * stride : a.N;  // the next active row
    am &= am - 1;
    const uint32_t w2 = wn;
    uint32_t ej2 = EMPTY, rj2 = 0, cj2 = 0, sv2 = 0, dw2 = 0;
    if constexpr (CHN) {
      if (w2 < a.N) {
        ej2 = a.ccol[(size_t)w2 * CELL_W + lane];
        rj2 = a.cpos[(size_t)w2 * CELL_W + lane];
        if (lane < (int)LP_SW) sv2 = a.st[(size_t)w2 * LP_SW + lane];
      }
    } else if (w2 < a.N && lane < (int)MESH_W) {  // w2 < N is wave-uniform
      ej2 = a.mesh[(size_t)(a.u0 + w2) * MESH_W + lane];
      rj2 = a.rpos[(size_t)(a.u0 + w2) * MESH_W + lane];
      sv2 = a.st[(size_t)w2 * LP_SW + lane];
    }
    if (GOS && gw && w2 < a.N) dw2 = a.rowdone[w2 >> 5];
    const uint64_t cand = __ballot(cj != 0);
    // entries destined to window c; a count past the capacity means entries were
    // dropped (ERR_LIST, the batch re-runs on k_pull): read only what was written
    const uint32_t due = umin32(__builtin_amdgcn_readlane(sv, cslot), a.lcap);
    // gossip windows: a row with a lane not yet final may take IWANT answers
    bool gossip_row = GOS && gw && !((dw >> (w & 31)) & 1u) && (!CHN || a.gtag[w] == gbk);
    uint32_t gnfl = 0, goffa = 0;  // CHN: lanes that may take an IHAVE (not final, online at kh, published)
    if constexpr (GOS && CHN) {
      if (gossip_row) {
        const uint32_t fT = reinterpret_cast<const uint16_t*>(a.fin + (size_t)w * LP_FW)[lane];
        const uint32_t offh = reinterpret_cast<const uint16_t*>(a.coff + ((size_t)gkh * a.N + w) * LP_FW)[lane];
        goffa = reinterpret_cast<const uint16_t*>(a.coff + ((size_t)(gkh + 1) * a.N + w) * LP_FW)[lane];
        gnfl = ~fT & ~offh & calT & 0xFFFFu;
        gossip_row = __ballot(gnfl != 0) != 0;
      }
    }
    if (cand == 0 && due == 0 && !gossip_row) {  // nothing to apply, nothing due: the pending windows stay
      if (lane == 0) wcnt[w] = 0;
      if (lane < (int)K && sv) nmh = umin32(nmh, lwhi);
      if (pull && lane < (int)HW && ej2 != EMPTY) {
        cj2 = rcnt[ej2 & 0xFFFFFFu];
        if constexpr (PART) ro2 = a.roff[ej2 & 0xFFFFFFu];
        if constexpr (CHN) {
          if (!((runi[ej2 & 0xFFFFFFu] >> (rj2 & 63u)) & 1)) cj2 = 0;
        }
      }
      ej = ej2; rj = rj2; cj = cj2; sv = sv2; ro = ro2; dw = dw2;
      PP_T(tS);
      PP_ADD(0, tS - tA);
      continue;
    }
    PP_ADD(7, 1);
    const uint32_t sw = a.stage[a.u0 + w];
    // final bits transposed: lane j holds bit q for lane q*64 + j (u16 per lane)
    uint32_t finT = reinterpret_cast<const uint16_t*>(a.fin + (size_t)w * LP_FW)[lane];
    // churn: the row's lanes offline in the records' next epoch (crossing records)
    uint32_t onl = 0;
    if constexpr (CHN) {
      if (offn) onl = reinterpret_cast<const uint16_t*>(offn + (size_t)w * LP_FW)[lane];
    }
    // 1 + 2. the entries listed for window c and this pass's candidates from
    //    the neighbours' records of window lo, min-reduced per lane in CW (final
    //    lanes are dropped in step 3). The first 256 entries are applied after
    //    the first neighbour group's record loads are issued: one memory round
    //    trip for both instead of two in a row.
    uint32_t cb = 0;
    const uint64_t* lst = a.blk + ((size_t)cslot * a.N + w) * a.ls;
    const uint32_t lmask = (1u << a.lb) - 1;
    const uint64_t wlok = wlo << a.tshift;
    uint64_t e[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t f = u * 64 + lane;
      e[u] = f < due ? lst[f] : ~0ull;
    }
    bool ent = true;  // wave-uniform: the first entries still to apply
    // 2 (churn). 16-B records from the CSR neighbours: w's bit at its position
    //    p in the sender's row (rj), FIFO position 1 + the receivers below p; a
    //    record that crosses into the next epoch is dropped where w is offline
    //    there (onl; lane `slot`'s bit fetched from lane slot & 63)
    if constexpr (CHN) {
      if (pull) {
        const uint32_t sd = sdn[sw];
        uint64_t cmk = cand;
        while (cmk) {
          uint32_t U[NG], NN[NG], SER[NG], IB0[NG], IB1[NG], LM0[NG], LM1[NG];
          uint64_t BASE[NG];
          uint32_t maxn = 0;
#pragma unroll
          for (int k = 0; k < (int)NG; k++) {
            const uint64_t bit = cmk & (~cmk + 1);
            cmk ^= bit;
            const int j = bit ? (int)__builtin_ctzll(bit) : 0;
            const uint32_t e = __builtin_amdgcn_readlane(ej, j);
            U[k] = e & 0xFFFFFFu;
            const uint32_t r = __builtin_amdgcn_readlane(rj, j) & 63u;
            IB0[k] = r < 32 ? 1u << r : 0u;
            IB1[k] = r < 32 ? 0u : 1u << (r - 32);
            LM0[k] = r < 32 ? (1u << r) - 1u : ~0u;
            LM1[k] = r < 32 ? 0u : (1u << (r - 32)) - 1u;
            NN[k] = bit ? (uint32_t)__builtin_amdgcn_readlane(cj, j) : 0u;
            const uint32_t su0 = e >> STAGE_SHIFT, su = su0 < S ? su0 : 0u;
            SER[k] = sup[su];
            BASE[k] = ((lo + lat[su * S + sw] + (sd > SER[k] ? sd - SER[k] : 0)) << a.tshift) +
                      ((1ull << a.sb) | U[k]);
            maxn = NN[k] > maxn ? NN[k] : maxn;
          }
          __amdgpu_buffer_rsrc_t RS[NG];
#pragma unroll
          for (int k = 0; k < (int)NG; k++)
            RS[k] = __builtin_amdgcn_make_buffer_rsrc((void*)(rrec + (size_t)U[k] * LL * 2), (short)0,
                                                      (int)(NN[k] * 16u), 0x00020000);
          for (uint32_t i0 = 0; i0 < maxn; i0 += 64) {
            uint32_t rv[NG][4];
#pragma unroll
            for (int k = 0; k < (int)NG; k++) {
              const uint32_t i = i0 + lane;
              const auto v = __builtin_amdgcn_raw_buffer_load_b128(RS[k], i * 16u, 0, 0);
              rv[k][0] = v[0]; rv[k][1] = v[1]; rv[k][2] = v[2]; rv[k][3] = v[3];
            }
            if (ent) {
              ent = false;
              lp_apply_entries(CW, e, lmask, a.lb, wlok, cb);
            }
#pragma unroll
            for (int k = 0; k < (int)NG; k++) {
              const uint32_t lo32 = rv[k][0], so = rv[k][1];
              bool ok = ((rv[k][2] & IB0[k]) | (rv[k][3] & IB1[k])) != 0;
              const uint32_t slot = lo32 & LP_LANE_MASK;
              const uint32_t pos = (uint32_t)__popc(rv[k][2] & LM0[k]) + (uint32_t)__popc(rv[k][3] & LM1[k]) + 1u;
              const uint64_t off = (uint64_t)pos * SER[k] + so;
              const uint64_t nk = BASE[k] + (((off << HOP_BITS) | (lo32 >> LP_HOP_SHIFT)) << a.sb);
              if (offn) {  // wave-uniform: a record may cross into epoch ks + 1
                const uint32_t ob = (uint32_t)__shfl((int)onl, (int)(slot & 63u));
                if (nk >= xBs && ((ob >> (slot >> 6)) & 1u)) ok = false;
              }
              if (ok) {
                atomicMin((unsigned long long*)&CW[slot], (unsigned long long)nk);
                cb |= 1u << (slot >> 6);
              }
            }
          }
        }
      }
    }
    // 2. this pass's candidates from the neighbours' records of window lo
    if (!CHN && pull) {
      const uint32_t sd = sdn[sw];
      uint64_t cmk = cand;
      while (cmk) {
        uint32_t U[NG], NN[NG], SER[NG], IB[NG], LB[NG];
        uint64_t BASE[NG], RO[NG];
        uint32_t maxn = 0;
#pragma unroll
        // wave-uniform and branch-free (a missing neighbour has NN = 0): with
        // the assignments under `if (cmk)` the compiler kept the descriptors of
        // neighbours 1-3 in VGPRs and wrapped each of their buffer loads in a
        // readfirstlane waterfall loop (35 -> 11 v_readfirstlane, 118 -> 110
        // VGPRs for k_lpull<1, 16>)
        for (int k = 0; k < (int)NG; k++) {
          const uint64_t bit = cmk & (~cmk + 1);
          cmk ^= bit;
          const int j = bit ? (int)__builtin_ctzll(bit) : 0;
          const uint32_t e = __builtin_amdgcn_readlane(ej, j);
          U[k] = e & 0xFFFFFFu;
          if constexpr (PART)
            RO[k] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(ro >> 32), j) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane((uint32_t)ro, j);
          else
            RO[k] = (uint64_t)U[k] * LL;
          // w's bit in the record's inclusion mask, and the bits below it
          const uint32_t r = __builtin_amdgcn_readlane(rj, j);
          IB[k] = 1u << (LP_IM_SHIFT + r);
          LB[k] = ((1u << r) - 1u) << LP_IM_SHIFT;
          NN[k] = bit ? (uint32_t)__builtin_amdgcn_readlane(cj, j) : 0u;
          const uint32_t su0 = e >> STAGE_SHIFT, su = su0 < S ? su0 : 0u;  // a missing neighbour's EMPTY: class 0
          SER[k] = sup[su];
          // the candidate key less its record-dependent parts: (arrival base
          // << tshift) + (hops 1 | src); a record adds (start offset + FIFO
          // position * ser) << tshift and its hops << sb (no carries: the low
          // fields stay below 2^tshift, the sender checked the time field)
          BASE[k] = ((lo + lat[su * S + sw] + (sd > SER[k] ? sd - SER[k] : 0)) << a.tshift) +
                    ((1ull << a.sb) | U[k]);
          maxn = NN[k] > maxn ? NN[k] : maxn;
        }
        __amdgpu_buffer_rsrc_t RS[NG];  // wave-uniform: base = the neighbour's records, NN[k] of them
#pragma unroll
        for (int k = 0; k < (int)NG; k++)
          RS[k] = __builtin_amdgcn_make_buffer_rsrc((void*)(rrec + RO[k]), (short)0, (int)(NN[k] * 8u), 0x00020000);
        for (uint32_t i0 = 0; i0 < maxn; i0 += 64 * RCH) {
          uint64_t rec[NG][RCH];
#pragma unroll
          for (int k = 0; k < (int)NG; k++)
#pragma unroll
            for (int cc = 0; cc < (int)RCH; cc++) {
              // bounds-checked buffer load, 32-bit offset: past the
              // neighbour's NN records it reads 0, which no record is (a
              // forwarding sender has hops >= 1)
              const uint32_t i = i0 + cc * 64 + lane;
              if (GS_LP_SKIP && i0 + cc * 64 >= NN[k]) {  // wave-uniform: a chunk past every record
                rec[k][cc] = 0;
                continue;
              }
              const auto v = __builtin_amdgcn_raw_buffer_load_b64(RS[k], i * 8u, 0, 0);
              rec[k][cc] = ((uint64_t)v[1] << 32) | v[0];
            }
          if (ent) {  // the listed entries while the records are in flight
            ent = false;
            lp_apply_entries(CW, e, lmask, a.lb, wlok, cb);
          }
#pragma unroll
          for (int k = 0; k < (int)NG; k++)
#pragma unroll
            for (int cc = 0; cc < (int)RCH; cc++) {
              if (GS_LP_SKIP && i0 + cc * 64 >= NN[k]) continue;  // (nothing loaded: no record)
              const uint64_t rc = rec[k][cc];
              const uint32_t lo32 = (uint32_t)rc;
              // w receives it iff its bit of the inclusion mask is set (no
              // record reads 0: no bit), at FIFO position 1 + the receivers
              // before it; the time field cannot overflow (the sender checked
              // start + rmax)
              const bool ok = (lo32 & IB[k]) != 0;
              const uint32_t slot = lo32 & LP_LANE_MASK;
              const uint32_t pos = (uint32_t)__popc(lo32 & LB[k]) + 1u;
              const uint64_t off = (uint64_t)pos * SER[k] + (rc >> 32);
              // tshift = sb + HOP_BITS: time and hops are one field above src
              const uint64_t nk = BASE[k] + (((off << HOP_BITS) | (lo32 >> LP_HOP_SHIFT)) << a.sb);
              if (ok) {
                atomicMin((unsigned long long*)&CW[slot], (unsigned long long)nk);
                cb |= 1u << (slot >> 6);
              }
            }
        }
      }
    }
    if (ent) lp_apply_entries(CW, e, lmask, a.lb, wlok, cb);  // no records
    for (uint32_t f0 = 256; f0 < due; f0 += 256) {  // more than 256 entries (rare)
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t f = f0 + u * 64 + lane;
        e[u] = f < due ? lst[f] : ~0ull;
      }
      lp_apply_entries(CW, e, lmask, a.lb, wlok, cb);
    }
    PP_T(tG);
    PP_ADD(1, tG - tA);
    // 2b. lazy gossip (GOS): IHAVEs of the built heartbeat k landing in window c
    //     from the row's non-mesh connections v. Every entry and record of the
    //     window is in CW now, so w has the message by the IHAVE's arrival t_i
    //     iff CW holds a time <= t_i there; else w sends IWANT and v's answer
    //     (its key's hops + 1, src v) is one more candidate, after window c.
    if constexpr (GOS && CHN) {
      if (gossip_row) glp_ihave_chn(a, CW, sw, gnfl, wlo, gR, ej, rj, goffa, gB1, lat, sup, sdn, cb, niw, err);
      if (due) glp_ihave_ent(a, CW, w, sw, finT, lst, due, wlok, lat, sup, sdn, cb, niw, err);
    } else if constexpr (GOS) {
      if (gossip_row) glp_ihave(a, CW, w, sw, finT, wlo, gR, lat, sup, sdn, cb, niw, err);
    }
    for (int off = 32; off > 0; off >>= 1) cb |= __shfl_xor(cb, off);
    cb = __builtin_amdgcn_readfirstlane(cb);
    wave_lds_sync();
    if (pull && lane < (int)HW && ej2 != EMPTY) {  // next row's lists
      cj2 = rcnt[ej2 & 0xFFFFFFu];
      if constexpr (PART) ro2 = a.roff[ej2 & 0xFFFFFFu];
      if constexpr (CHN) {
        if (!((runi[ej2 & 0xFFFFFFu] >> (rj2 & 63u)) & 1)) cj2 = 0;
      }
    }
    // 3. classify the minima of the touched chunks: final lanes are dropped
    //    (candidates are not filtered on the way in), a minimum in window c is
    //    final now (logged, marked, its lane / group indexed from the front of
    //    LST), a later one is pending (indexed from the back). Keys stay where
    //    they are in CW.
    PP_T(tR);
    PP_ADD(2, tR - tG);
    const uint32_t log0 = __builtin_amdgcn_readlane(sv, LP_LOG);
    uint32_t logc = log0, cnt = 0, npend = 0, nfin = 0;  // the finals are logged in step 4
#pragma unroll
    for (int q = 0; q < (int)CH; q++) {
      if (!((cb >> q) & 1u)) continue;  // wave-uniform
      const uint32_t i = q * 64 + lane;
      const uint64_t x = CW[i];
      const bool fe = (finT & (1u << q)) != 0;  // final in an earlier window: dropped
      // (a fragment group's step 4 re-reads every lane of a final group)
      if (FP > 1 && fe && x != INF64) CW[i] = INF64;
      // the wave's masks from three single compares (a ballot of a compound
      // predicate cost a select + compare each), lane positions by mbcnt
      const bool inf = x == INF64, inw = ((uint32_t)(x >> 32) - hlo) < hspan;
      // llvm.amdgcn.icmp: the compare's lane mask as is (32 EQ, 33 NE, 36 ULT)
      const uint64_t dead = __builtin_amdgcn_uicmp(finT & (1u << q), 0u, 33) | __builtin_amdgcn_uicmpl(x, INF64, 32);
      const uint64_t bw = __builtin_amdgcn_uicmp((uint32_t)(x >> 32) - hlo, hspan, 36);
      const uint64_t am = bw & ~dead, pm = ~(bw | dead);
      const bool act = !fe && !inf && inw, pend = !fe && !inf && !inw;
      if (pend)
        LST[LMAX - 1 - (npend + __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u)))] =
            (uint16_t)i;
      npend += (uint32_t)__popcll(pm);
      if (am) {  // wave-uniform
        finT |= act ? 1u << q : 0u;
        nfin = 1;
        if constexpr (FP == 1) {
          if (act)
            LST[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u))] =
                (uint16_t)i;
          cnt += (uint32_t)__popcll(am);
        } else {
          constexpr uint64_t gmask = (FP == 64) ? ~0ull : ((1ull << FP) - 1);
          const int gb = lane & ~(FP - 1);
          const bool gact = ((am >> gb) & gmask) != 0;
          const uint64_t lm = __ballot(gact && (lane & (FP - 1)) == 0);  // group leaders
          if (gact && (lane & (FP - 1)) == 0) LST[cnt + (uint32_t)__popcll(lm & lanelt)] = (uint16_t)(i / FP);
          cnt += (uint32_t)__popcll(lm);
        }
      }
    }
    wave_lds_sync();
    PP_T(tC);
    PP_ADD(3, tC - tR);
    // 3b. the pending minima -> the lists of their windows c + r (r = 1..K-1),
    //     appended after the entries already there
    // lane j < K: entries appended to list slot j in this pass (lane-held, so
    // each group of 64 visits only the destination windows present in it)
    uint32_t addl = 0;
    // an EMIT pass's minima all lie in window c, except IWANT answers (GOS)
    if (!pull && !GOS && npend) err |= ERR_RING;
    if ((pull || GOS) && npend) {
      const uint32_t lmax = a.lcap;
      for (uint32_t j0 = 0; j0 < npend; j0 += 64) {
        const bool jv = j0 + lane < npend;
        const uint32_t li = jv ? LST[LMAX - 1 - (j0 + lane)] : 0u;
        const uint64_t x = jv ? CW[li] : INF64;
        uint32_t r = 0;
        if (jv) {
          if (rdiv) {  // floor((hx - hlo) / dG) capped at K: the float quotient is within 1
            const uint32_t d = (uint32_t)(x >> 32) - hlo;
            uint32_t q = (uint32_t)((float)d * rinv);
            if ((uint64_t)q * hspan > d) q--;
            else if (((uint64_t)q + 1) * hspan <= d) q++;  // widened first: q may be 0xFFFFFFFF
            r = q < K ? q : K;
          } else {
            r = lp_rof((uint32_t)(x >> 32), hlo64, a.dG, K);
          }
        }
        if (jv && r >= K) err |= ERR_RING;
        const bool ap = jv && r > 0 && r < K;
        uint32_t pos = 0, slot = 0;
        uint64_t rem = __builtin_amdgcn_uicmp(r - 1u, K - 1u, 36);  // ap: r in [1, K) (r = 0 off the list)
        while (rem) {                 // read from the lowest lane still waiting (wave-uniform)
          const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)__builtin_ctzll(rem));
          const uint32_t sl = (cslot + k) % K;
          const uint64_t bm = __builtin_amdgcn_uicmp(r, k, 32);  // k >= 1: only listed lanes
          rem &= ~bm;
          const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane(sv + addl, sl);
          if (ap && r == k) {
            pos = b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
            slot = sl;
          }
          addl += lane == (int)sl ? (uint32_t)__popcll(bm) : 0u;
        }
        if (ap) {
          if (pos >= lmax) err |= ERR_LIST;
          else {
            const uint64_t toff = (x >> a.tshift) - (wlo + (uint64_t)r * a.delta);
            a.blk[((size_t)slot * a.N + w) * a.ls + pos] = (toff << (a.tshift + a.lb)) | ((x & lowmask) << a.lb) | li;
          }
        }
      }
    }
    np += npend + cnt;
    PP_T(tP);
    PP_ADD(4, tP - tC);
    // 4. sparse: forward targets, uplink FIFO and one record per arrival (k_pull's step 4)
    uint32_t ecnt = 0;
    uint64_t uni = 0;  // churn: the receivers of any of the row's records
    if (cnt) {
      const uint32_t deg = (uint32_t)__popcll(__ballot(ej != EMPTY));  // rows are packed
      const uint32_t psl = a.rN ? (w / a.rN) * a.B : 0u;  // batch slices: this row's publishers
      const bool needp = !a.pubw || __builtin_amdgcn_readlane(sv, LP_PUB) != 0;
      const uint32_t serw = sup[sw];
      constexpr uint32_t GPW = 64 / FP;
      for (uint32_t g0 = 0; g0 < cnt; g0 += GPW) {
        const uint32_t gi = g0 + (uint32_t)lane / FP;
        const bool gv = gi < cnt;
        const uint32_t grp = gv ? LST[gi] : 0;
        const uint32_t i = grp * FP + (lane & (FP - 1));
        const uint64_t x = gv ? CW[i] : INF64;  // final lanes were set to INF in step 3
        // the message's publisher (excluded from the receivers); a row that is
        // no publisher nor a publisher's neighbour needs none (no load)
        uint32_t pm = EMPTY;
        if (needp) pm = gv ? a.pub[psl + grp] : EMPTY;
        // FP == 1: LST holds only lanes final in window c; a fragment group's
        // other lanes are re-checked
        const bool act = gv && (FP == 1 || (x != INF64 && ((uint32_t)(x >> 32) - hlo) < hspan)) && a.u0 + w != pm;
        const uint32_t src = (uint32_t)(x & smask);
        uint32_t xm = 0;  // excluded mesh indices: source, publisher (IDW: and IDONTWANT)
        uint64_t im64 = 0;  // churn: the receivers as a mask over the CSR row
        if constexpr (CHN) {  // the mesh of the epoch the lane was received in, less source and publisher
          const uint32_t kk = kc + ((x >> a.tshift) >= eBc ? 1u : 0u);
          const uint64_t mmv = act ? a.cmm[(size_t)w * a.cE + a.cq[grp] + kk] : 0ull;
          uint64_t xm64 = 0;
          for (uint32_t k = 0; k < deg; k++) {  // wave-uniform: entry k from lane k
            const uint32_t y = __builtin_amdgcn_readlane(ej, k) & 0xFFFFFFu;
            xm64 |= (y == src || y == pm) ? 1ull << k : 0ull;
          }
          im64 = mmv & ~xm64;
        } else if constexpr (IDW) {
          // IDONTWANT from y already here: ky + lat(y -> w) <= t_w. The keys of
          // IB mesh entries are loaded before any is tested (one round trip per
          // IB entries instead of one per entry; CH = 8 rows run at 80 VGPRs)
          constexpr uint32_t IB = CH == 8 ? 2 : 8;
          const uint64_t tw = x >> a.tshift;
          for (uint32_t k0 = 0; k0 < deg; k0 += IB) {  // wave-uniform: entry k from lane k
            uint64_t ky[IB];
#pragma unroll
            for (uint32_t u = 0; u < IB; u++) {
              const uint32_t k = k0 + u;
              const uint32_t y = k < deg ? (uint32_t)__builtin_amdgcn_readlane(ej, k) & 0xFFFFFFu : src;
              ky[u] = act && y != src && y != pm ? a.keys[(size_t)y * LL + i] : INF64;
            }
#pragma unroll
            for (uint32_t u = 0; u < IB; u++) {
              const uint32_t k = k0 + u;
              if (k >= deg) break;  // (wave-uniform)
              const uint32_t e = __builtin_amdgcn_readlane(ej, k);
              const uint32_t y = e & 0xFFFFFFu;
              const bool sk = y == src || y == pm ||
                              (ky[u] != INF64 && (ky[u] >> a.tshift) + lat[(e >> STAGE_SHIFT) * S + sw] <= tw);
              xm |= sk ? 1u << k : 0u;
            }
          }
        } else {
          for (uint32_t k = 0; k < deg; k++) {  // wave-uniform: entry k from lane k
            const uint32_t y = __builtin_amdgcn_readlane(ej, k) & 0xFFFFFFu;
            xm |= (y == src || y == pm) ? 1u << k : 0u;
          }
        }
        const uint32_t im = CHN ? 0u : ((1u << deg) - 1u) & ~xm;  // the receivers (deg <= MESH_W = 16)
        const uint32_t n = act ? (CHN ? (uint32_t)__popcll(im64) : (uint32_t)__popc(im)) : 0u;
        const uint64_t start = uplink_start<FP>(a.busy, (size_t)w * a.B + grp, act, x, n, serw, a.tshift);
        const uint32_t hp = (uint32_t)(x >> a.sb) & hmask;
        if (act) {
          fd++;
          nr += n;
          if (n && hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
          if (start - wlo >= (1ull << 32) || (n && start + a.rmax > a.tmax)) err |= ERR_TIME;
        }
        // act as lane masks: listed (gi < cnt) and not the message's publisher
        const uint64_t fm = FP == 1 ? (__builtin_amdgcn_uicmp(gi, cnt, 36) & __builtin_amdgcn_uicmp(pm, a.u0 + w, 33))
                                    : __ballot(act);  // final log: 64 entries per store
        if constexpr (IDW) {
          if (act) a.keys[(size_t)w * LL + i] = x;  // dense: the neighbours' IDONTWANT tests read it
        } else {
          if (act) {
            const uint32_t p =
                logc + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
            if (GS_LP_NT) {  // the final log is read after the passes (completion): stream it past the caches
              __builtin_nontemporal_store(x, &a.keys[(size_t)w * LL + p]);
              __builtin_nontemporal_store((uint16_t)i, &a.flane[(size_t)w * LL + p]);
            } else {
              a.keys[(size_t)w * LL + p] = x;
              a.flane[(size_t)w * LL + p] = (uint16_t)i;
            }
          }
          logc += (uint32_t)__popcll(fm);
        }
        const bool want = act && n != 0;
        const uint64_t wm = fm & __builtin_amdgcn_uicmp(n, 0u, 33);
        if (want) {
          const size_t ri = (size_t)w * LL + ecnt +
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u));
          if constexpr (CHN) {
            uni |= im64;
            const uint64_t r0 = ((start - wlo) << 32) | ((uint64_t)hp << LP_HOP_SHIFT) | i;
            *reinterpret_cast<uint4*>(wrec + ri * 2) =
                make_uint4((uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)im64, (uint32_t)(im64 >> 32));
          } else {
            const uint64_t rv = ((start - wlo) << 32) | ((uint64_t)hp << LP_HOP_SHIFT) | ((uint64_t)im << LP_IM_SHIFT) | i;
            if (GS_LP_NTR) __builtin_nontemporal_store(rv, &wrec[ri]);
            else wrec[ri] = rv;
          }
        }
        ecnt += (uint32_t)__popcll(wm);
      }
    }
    PP_T(tD);
    PP_ADD(5, tD - tP);
    // 5. row state: final bits, pending list lengths, log length
    if (nfin) reinterpret_cast<uint16_t*>(a.fin + (size_t)w * LP_FW)[lane] = (uint16_t)finT;
    if constexpr (GOS) {  // every lane final: no IHAVE can matter to this row any more
      // (the lanes that can be final: F per message, one under defect D8; padding lanes never are)
      if (nfin && wave_sum((uint64_t)__popc(finT & 0xFFFFu)) == a.B * (a.collide ? 1u : a.F) && lane == 0)
        atomicOr(&a.rowdone[w >> 5], 1u << (w & 31));
    }
    {
      uint32_t nv = sv;  // lane j < K: slot j (window c + lwin), emptied if it is window c's
      if (lane < (int)K) nv = lane == (int)cslot ? 0u : sv + addl;
      if (lane == (int)LP_LOG) nv = logc;
      if (lane <= (int)LP_LOG) a.st[(size_t)w * LP_SW + lane] = nv;
      if (lane < (int)K && nv) nmh = umin32(nmh, lwhi);
    }
    if constexpr (CHN) {
      for (int off = 32; off > 0; off >>= 1) uni |= __shfl_xor(uni, off);
      if (lane == 0) wuni[w] = uni;
    }
    if (lane == 0) wcnt[w] = ecnt;
    nrec += ecnt;
    // 6. LDS back to INF for the next row: the touched chunks. cb passes
    //    through an empty asm so that the chunk tests are recomputed here from
    //    the scalar word (else the compiler keeps step 3's 16 chunk masks alive
    //    across the row: 32 SGPR spills to VGPR lanes and back per row)
    asm volatile("" : "+s"(cb));
#pragma unroll
    for (int q = 0; q < (int)CH; q++)
      if ((cb >> q) & 1u) CW[q * 64 + lane] = INF64;
    wave_lds_sync();
    ej = ej2; rj = rj2; cj = cj2; sv = sv2; ro = ro2; dw = dw2;
    PP_T(tE);
    PP_ADD(6, tE - tD);
  }
  }
#ifdef GS_PULL_PROF
  if (lane == 0)
    for (int k = 0; k < 8; k++) atomicAdd(&g_pull_prof[a.pass < 31 ? a.pass : 31][k], (unsigned long long)pp[k]);
#endif
  for (int off = 32; off > 0; off >>= 1) nmh = umin32(nmh, __shfl_xor(nmh, off));
  const uint64_t nmin = nmh == ~0u ? INF64 : (uint64_t)nmh << 32;
  fd = wave_sum(fd);
  nr = wave_sum(nr);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if (lane == 0) {
    if (nrec) atomicAdd((unsigned long long*)&me[2], (unsigned long long)nrec);
    if (nmin != INF64) atomicMin((unsigned long long*)&me[3], (unsigned long long)nmin);
    if (fd) atomicAdd((unsigned long long*)&a.counters[C_FD], (unsigned long long)fd);
    if (nr) atomicAdd((unsigned long long*)&a.counters[C_R_FWD], (unsigned long long)nr);
    if (np) atomicAdd((unsigned long long*)&a.counters[C_PUSH], (unsigned long long)np);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
  if constexpr (GOS) {
    niw = wave_sum(niw);
    if (lane == 0 && niw) atomicAdd((unsigned long long*)&a.counters[C_GOSSIP], (unsigned long long)niw);
  }
}

// Pass control of a GOS batch (one thread, before every pass): k_pull's rule
// (PULL the window whose records were just emitted, else EMIT the window of
// the min pending key, else DONE), where an EMIT also stops at the first
// window that can hold IHAVE arrivals while some lane is not final and some
// final lane still gossips (its first heartbeat + history_gossip - 1); then
// the heartbeats whose senders are all final now (R_k below the window):
// the one whose IHAVEs are still to come gets its planes built before the
// pass (k_gsend), and the pass learns whether its window holds its IHAVEs.
__global__ void k_lctl(LPullArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t* g = a.gctl;
  const uint64_t* pv = a.ctrl + ((a.pass + 2) % 3) * 4;
  uint64_t* me = a.ctrl + (a.pass % 3) * 4;
  uint64_t* nx = a.ctrl + ((a.pass + 1) % 3) * 4;
  const uint64_t D = a.delta, hb = a.ghb, r0 = a.grel0;
  const uint64_t fd = a.counters[C_FD];
  const uint64_t nf = a.gnf - (fd - g[GC_FD0]);  // lanes not final yet
  if (fd != g[GC_FDP]) {  // the last pass finalised lanes: all before the end of its window
    g[GC_TLAST] = g[GC_E];
    g[GC_FDP] = fd;
  }
  const uint64_t tl = g[GC_TLAST];
  uint64_t kmax = (tl <= r0 ? 0 : (tl - r0 + hb - 1) / hb) + a.ghist - 1;  // last heartbeat with a sender
  if (kmax > a.ghk) kmax = a.ghk;  // churn: no IHAVE past the messages' lifetime
  const bool gos = nf && a.ghist;
  uint64_t lo, mode;
  if (g[GC_DONE]) {
    mode = PM_DONE;
    lo = pv[0];
  } else if (pv[1] != PM_DONE && pv[2]) {
    mode = PM_PULL;
    lo = pv[1] == PM_PULL ? pv[0] + D : pv[0];
  } else {
    uint64_t e = pv[3] != INF64 ? ((pv[3] >> a.tshift) / D) * D : INF64;
    if (gos) {  // the next window with IHAVE arrivals: [R_k + lat_min, R_k + lat_max] from E on
      const uint64_t E = g[GC_E];
      const uint64_t k = E <= r0 + a.glat_max ? 0 : (E - r0 - a.glat_max + hb - 1) / hb;
      if (k <= kmax) {
        const uint64_t s = r0 + k * hb + a.glat_min;
        const uint64_t ws = s >= E ? (s / D) * D : E;  // E is a window boundary
        e = ws < e ? ws : e;
      }
    }
    if (e == INF64) {
      mode = PM_DONE;
      lo = pv[0];
      g[GC_DONE] = 1;
    } else {
      mode = PM_EMIT;
      lo = e;
    }
  }
  me[0] = lo;
  me[1] = mode;
  nx[2] = 0;
  nx[3] = INF64;
  g[GC_BUILD] = 0;
  g[GC_GW] = 0;
  if (mode == PM_DONE) return;
  atomicAdd((unsigned long long*)&a.counters[C_PASSES], 1ull);
  if (mode == PM_PULL) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
  const uint64_t wl = mode == PM_PULL ? lo + D : lo;  // the window this pass emits
  g[GC_E] = wl + D;
  for (uint64_t k = g[GC_GB]; r0 + k * hb < wl; k++) {  // every t_v <= R_k is final now
    if (gos && k <= kmax && r0 + k * hb + a.glat_max >= wl) {
      g[GC_BUILD] = k + 1;
      g[GC_BK] = k + 1;
    }
    g[GC_GB] = k + 1;
  }
  if (g[GC_BK] && gos) {
    const uint64_t R = r0 + (g[GC_BK] - 1) * hb;
    if (wl <= R + a.glat_max && wl + D > R + a.glat_min) g[GC_GW] = 1;
  }
}

// Sender planes of heartbeat k = GC_BUILD - 1, before the pass that first
// needs them. One wave per row v reads its final log (emission order: the
// entries with t <= R_k come first), keeps the lanes v gossips at k (first
// received in (R_(k - hist), R_k]), selects each one's IHAVE targets
// (glp_targets at heartbeat habs0[m] + k, the oracle's gossip_targets) and
// writes the plane and the entries (target mask | hops << 58) in rank order.
// A row none of whose non-mesh connections has a lane left to finalise is
// skipped: no pass reads its plane (row-done bits never clear within a batch).
// Pushed IHAVEs of sender row v at heartbeat k (churn, k >= gsw). Lane j holds
// the entries eq[q] (target mask | hops << 58) of v's lanes q*64 + j it gossips.
// For each connection t = ccx[e] (wave-uniform), the lanes whose targets
// include t and that t has not finalised yet (its final bits; most IHAVEs reach
// a peer that has the message, those are dropped here) become flagged entries
// t_i | hops + 1 | v | lane in t's list of the window holding t_i = R_k +
// lat(v -> t). A target that collects more than GP_CAP of them this heartbeat
// scans the planes instead (gtag; glp_ihave_ent then ignores its entries).
constexpr uint32_t GP_CAP = 192;
template <uint32_t CH>
__device__ __forceinline__ void glp_push(const LPullArgs& a, uint32_t v, uint64_t bk, uint64_t Rk, uint64_t wcur,
                                         const uint32_t* ccx, uint32_t deg, uint32_t plj, const uint64_t* eq,
                                         uint32_t calT, uint32_t& err) {
  const int lane = threadIdx.x & 63;
  const uint32_t S = a.S, sv = a.stage[v];
  const uint64_t dcur = udiv53(wcur, a.delta);  // the window the coming pass emits
  // connections whose targets include any offered lane, eight final-bit rows in flight at once
  uint64_t ce = 0;
  for (uint32_t e = 0; e < deg; e++) {  // wave-uniform
    uint32_t off = 0;
#pragma unroll
    for (int q = 0; q < (int)CH; q++) off |= (uint32_t)((eq[q] >> e) & 1) << q;
    if (__ballot((off & plj) != 0)) ce |= 1ull << e;
  }
  while (ce) {
    constexpr int GT = 8;
    uint32_t E[GT], FT[GT];
    int nt = 0;
#pragma unroll
    for (int g = 0; g < GT; g++) {
      E[g] = ce ? (uint32_t)__builtin_ctzll(ce) : 0u;
      if (ce) { ce &= ce - 1; nt = g + 1; }
    }
#pragma unroll
    for (int g = 0; g < GT; g++)
      FT[g] = g < nt ? reinterpret_cast<const uint16_t*>(a.fin + (size_t)(ccx[E[g]] & 0xFFFFFFu) * LP_FW)[lane] : 0xFFFFu;
    auto one = [&](uint32_t e, uint32_t ftg) {

    uint32_t off = 0;  // lane j: chunks q whose lane targets t
#pragma unroll
    for (int q = 0; q < (int)CH; q++) off |= (uint32_t)((eq[q] >> e) & 1) << q;
    off &= plj;
    const uint32_t xe = ccx[e], t = xe & 0xFFFFFFu;
    const uint32_t pj = off & ~ftg & calT;
    const uint32_t cj = (uint32_t)__popc(pj);
    uint32_t n = cj;
    for (int o = 32; o > 0; o >>= 1) n += (uint32_t)__shfl_xor((int)n, o);
    if (n == 0) return;
    uint32_t ok = 0, pos0 = 0, slot = 0;
    uint64_t toff = 0;
    if (lane == 0) {
      uint32_t old = a.gpc[t], nw;
      for (;;) {  // count the row's pushes of heartbeat bk (a stale tag restarts the count)
        const uint32_t cnt = (old >> 16) == (uint32_t)bk ? (old & 0xFFFFu) : 0u;
        nw = ((uint32_t)bk << 16) | (cnt + n < 0xFFFFu ? cnt + n : 0xFFFFu);
        const uint32_t o2 = atomicCAS(&a.gpc[t], old, nw);
        if (o2 == old) break;
        old = o2;
      }
      if ((nw & 0xFFFFu) > GP_CAP) {
        a.gtag[t] = (uint16_t)bk;  // t scans the planes of this heartbeat
      } else {
        const uint64_t ti = Rk + a.tables[sv * S + (xe >> STAGE_SHIFT)];
        const uint64_t d = udiv53(ti, a.delta);  // the window of t_i
        if (d < dcur || d >= dcur + a.K) {
          err |= ERR_RING;  // (k_lctl builds before the first window that can hold an IHAVE)
        } else {
          slot = (uint32_t)(d % a.K);
          toff = ti - d * a.delta;
          pos0 = atomicAdd(&a.st[(size_t)t * LP_SW + slot], n);
          ok = 1;
        }
      }
    }
    if (!__shfl((int)ok, 0)) return;
    pos0 = (uint32_t)__shfl((int)pos0, 0);
    slot = (uint32_t)__shfl((int)slot, 0);
    toff = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(toff >> 32), 0) << 32) | (uint32_t)__shfl((int)(uint32_t)toff, 0);
    uint32_t pre = cj;  // exclusive prefix of the lanes' counts
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)pre, o);
      if (lane >= o) pre += y;
    }
    pre -= cj;
    uint64_t* lst = a.blk + ((size_t)slot * a.N + t) * a.ls;
    uint32_t c = pj;
    while (c) {
      const int q = __builtin_ctz(c);
      c &= c - 1;
      const uint32_t pos = pos0 + pre++;
      if (pos >= a.lcap) { err |= ERR_LIST; continue; }
      const uint32_t hv = (uint32_t)(eq[q] >> GSE_HOPS) + 1;
      if (hv >= (1u << HOP_BITS)) { err |= ERR_HOPS; continue; }
      lst[pos] = (1ull << 63) | (toff << (a.tshift + a.lb)) | ((((uint64_t)hv << a.sb) | v) << a.lb) |
                 ((uint32_t)q * 64 + lane);
    }
    };
#pragma unroll
    for (int g = 0; g < GT; g++)
      if (g < nt) one(E[g], FT[g]);  // wave-uniform
  }
}

// Churn (CHN): a lane's epoch is E0 + cq[m] + kh (kh = ghoff + k, the
// heartbeat's relative epoch), its targets the ones k_cprep selected for (v,
// that epoch) (none when v is offline then), and nothing past the lifetime
// (kh > chz); lanes with no target get no plane bit.
template <uint32_t CH, bool CHN = false>
__global__ __launch_bounds__(TB) void k_gsend(LPullArgs a) {
  const uint64_t bk = a.gctl[GC_BUILD];
  if (!bk) return;  // grid-uniform: nothing to build before this pass
  __shared__ uint64_t ent[PULL_WAVES][CH * 64];
  __shared__ uint32_t sel[PULL_WAVES][CH * 64];
  __shared__ uint32_t pl[PULL_WAVES][LP_FW];
  __shared__ uint32_t cxs[PULL_WAVES][CHN ? CELL_W : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lanelt = (1ull << lane) - 1;
  const uint64_t k = bk - 1, Rk = a.grel0 + k * a.ghb;
  const uint64_t wcur = a.gctl[GC_E] - a.delta;  // start of the window the coming pass emits
  const uint32_t calT = CHN ? reinterpret_cast<const uint16_t*>(a.calive)[threadIdx.x & 63] : 0u;
  const bool haslo = k >= a.ghist;
  const uint64_t Rlo = haslo ? a.grel0 + (k - a.ghist) * a.ghb : 0;
  const uint32_t hmask = (1u << HOP_BITS) - 1;
  for (uint32_t v = blockIdx.x * PULL_WAVES + wv; v < a.N; v += gridDim.x * PULL_WAVES) {
    const uint32_t soff = a.rN ? (v / a.rN) * a.rN : 0u;  // batch slices: the slice's first row
    uint32_t deg, x = EMPTY;
    bool nm = false;
    uint32_t* ccx = cxs[wv];  // CHN: the row's CSR entries (stage << 24 | peer) for glp_push
    if constexpr (CHN) {
      const uint32_t xe = a.ccol[(size_t)v * CELL_W + lane];
      ccx[lane] = xe;
      nm = xe != EMPTY;  // any connection may be outside the lane's epoch mesh
      x = nm ? xe & 0xFFFFFFu : EMPTY;
      deg = (uint32_t)__popcll(__ballot(nm));
    } else {  // batch slices: the CSR and the rng by the peer, per-row arrays by the slice row
      const uint64_t rb = a.row[v - soff];
      deg = (uint32_t)(a.row[v - soff + 1] - rb);
      if ((uint32_t)lane < deg) {
        x = a.col[rb + lane];
        nm = !(a.flags[rb + lane] & F_MESH);
      }
    }
    bool need = false;
    if (nm) need = !((a.rowdone[(x + soff) >> 5] >> ((x + soff) & 31)) & 1u);
    if (__ballot(need) == 0) {  // wave-uniform
      if (CHN && lane == 0) a.gnz[v] = 0;
      continue;
    }
    if (lane < (int)LP_FW) pl[wv][lane] = 0;
    const uint64_t nmm = __ballot(nm);
    const uint64_t rpre = rng_pre(a.gseed, P_GOSSIP, v - soff);
    const uint32_t nonmesh = (uint32_t)__popcll(nmm);
    uint32_t r = (uint32_t)(((uint64_t)nonmesh * a.ggf) / 1000);
    if (r < a.gd_lazy) r = a.gd_lazy;
    if (r > nonmesh) r = nonmesh;
    // 1. the senders of k from the log: lane | hops << 16 (IDONTWANT batches keep
    //    dense final keys instead of a log: every lane of the row is looked at)
    const uint32_t n = a.idw ? a.L : a.st[(size_t)v * LP_SW + LP_LOG];
    uint32_t ns = 0;
    // the log is in window order: entries before the first one whose window
    // holds R_(k - hist) or later are not senders of k; 64 samples locate it
    uint32_t i_start = 0;
    if (haslo && n > 64 && !a.idw) {
      const uint32_t stride = (n + 63) / 64, ip = (uint32_t)lane * stride;
      const uint64_t T = (Rlo / a.delta) * a.delta;
      const uint64_t sk = ip < n ? a.keys[(size_t)v * a.L + ip] : INF64;
      const uint64_t sm = __ballot(ip >= n || (sk >> a.tshift) >= T);
      const uint32_t J = sm ? (uint32_t)__builtin_ctzll(sm) : 64u;
      i_start = J == 0 ? 0u : (J - 1) * stride + 1;
    }
    for (uint32_t i0 = i_start; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      const uint64_t key = i < n ? a.keys[(size_t)v * a.L + i] : INF64;
      const uint64_t t = key >> a.tshift;
      const bool s = i < n && key != INF64 && t <= Rk && (!haslo || t > Rlo);
      const uint64_t sm = __ballot(s);
      if (s)
        sel[wv][ns + (uint32_t)__popcll(sm & lanelt)] =
            (a.idw ? i : (uint32_t)a.flane[(size_t)v * a.L + i]) | ((uint32_t)(key >> a.sb) & hmask) << 16;
      ns += (uint32_t)__popcll(sm);
      // log entries of later windows have t > R_k: stop after a chunk with none at or below R_k + Delta
      if (!a.idw && __ballot(i < n && t <= Rk + a.delta) == 0) break;
    }
    wave_lds_sync();
    // 2. each sender lane's targets at its message's heartbeat habs0[m] + k
    uint64_t tu = 0;  // CHN: every target of the row's planes
    for (uint32_t j0 = 0; j0 < ns; j0 += 64) {
      const bool jv = j0 + lane < ns;
      const uint32_t s = jv ? sel[wv][j0 + lane] : 0u;
      const uint32_t m = s & 0xFFFFu;  // the lane (fragment lanes: message m / FP; every fragment is
                                       // gossiped on its own, at its message's heartbeats)
      const uint32_t h = jv ? (uint32_t)(a.habs0[(a.rN ? (v / a.rN) * a.B : 0u) + m / (a.L / a.B)] + k) : 0u;
      uint64_t mask;
      if constexpr (CHN) {  // the targets k_cprep selected for (v, the lane's epoch)
        const uint32_t kh = a.ghoff + (uint32_t)k;
        mask = jv && kh <= a.chz ? a.cgt[(size_t)v * a.cE + a.cq[m / (a.L / a.B)] + kh] : 0ull;
      } else {
        mask = glp_targets(rpre, h, x, nmm, deg, r);
      }
      if (jv && (!CHN || mask)) {
        const uint64_t en = mask | ((uint64_t)(s >> 16) << GSE_HOPS);
        if constexpr (CHN) {  // churn: entries at their lane's position
          a.gse[(size_t)v * a.L + m] = en;
          tu |= mask;
        }
        ent[wv][m] = en;
        atomicOr(&pl[wv][(m & 63) >> 1], 1u << (16 * (m & 1) + (m >> 6)));
      }
    }
    wave_lds_sync();
    // 3. the plane, and the entries in rank order (lane j's bits q ascending after the lanes below j)
    if (lane < (int)LP_FW) a.gpl[(size_t)v * LP_FW + lane] = pl[wv][lane];
    const uint32_t plj = (pl[wv][lane >> 1] >> (16 * (lane & 1))) & 0xFFFFu;
    if constexpr (CHN) {
      const bool nz = __ballot(plj != 0) != 0;
      if (lane == 0) a.gnz[v] = nz ? 1 : 0;
      if (nz && k < a.gsw) {  // every target of an early heartbeat scans the planes
        for (int off = 32; off > 0; off >>= 1) tu |= __shfl_xor(tu, off);
        if ((uint32_t)lane < deg && ((tu >> lane) & 1)) a.gtag[x] = (uint16_t)bk;
      } else if (nz) {  // later heartbeats push what a target may still need
        uint64_t eq[CH];
#pragma unroll
        for (int q = 0; q < (int)CH; q++) eq[q] = ((plj >> q) & 1) ? ent[wv][q * 64 + lane] : 0ull;
        uint32_t err = 0;
        glp_push<CH>(a, v, bk, Rk, wcur, ccx, deg, plj, eq, calT, err);
        if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
      }
      wave_lds_sync();
      continue;  // (entries are in place)
    }
    const uint32_t own = (uint32_t)__popc(plj);
    uint32_t pre = own;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(pre, off);
      if (lane >= off) pre += y;
    }
    pre -= own;
    uint32_t c = plj;
    while (c) {
      const int q = __builtin_ctz(c);
      c &= c - 1;
      a.gse[(size_t)v * a.L + pre++] = ent[wv][q * 64 + lane];
    }
    wave_lds_sync();
  }
}

// Seeds -> lists: k_seed appended the publishers' first sends (key, row << 11
// | lane) to a seed list; each goes to the list of its window d = 1..K (slot
// d % K) at a position taken from the row's list length. One thread per seed.
__global__ __launch_bounds__(TB) void k_lseed(LPullArgs a, const uint64_t* __restrict__ skey,
                                              const uint32_t* __restrict__ slane, const uint32_t* __restrict__ scnt) {
  const uint32_t n = *scnt, K = a.K;
  const uint64_t lowmask = (1ull << a.tshift) - 1;
  uint32_t err = 0;
  for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < n; i += gridDim.x * TB) {
    const uint64_t key = skey[i];
    const uint32_t w = slane[i] >> 11, l = slane[i] & 2047u;
    const uint32_t d = (uint32_t)(key >> 32) / a.dG;  // the window index (hi-word grain)
    if (d == 0 || d > K) { err |= ERR_RING; continue; }
    const uint32_t slot = d % K;
    const uint32_t pos = atomicAdd(&a.st[(size_t)w * LP_SW + slot], 1u);
    if (pos >= a.lcap) { err |= ERR_LIST; continue; }
    const uint64_t toff = (key >> a.tshift) - (uint64_t)d * a.delta;
    a.blk[((size_t)slot * a.N + w) * a.ls + pos] = (toff << (a.tshift + a.lb)) | ((key & lowmask) << a.lb) | l;
  }
  if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
}

// LP_PUB of every publisher of the batch and of its mesh neighbours (churn:
// its CSR neighbours, the emit step's receivers): one thread per (message,
// entry); entry `width` is the publisher itself. nmsg: the pub entries (slices: S x B).
__global__ __launch_bounds__(TB) void k_lpubnb(LPullArgs a, uint32_t nmsg) {
  const uint32_t width = a.ccol ? CELL_W : MESH_W;
  const uint64_t g = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (g >= (uint64_t)nmsg * (width + 1)) return;
  const uint32_t m = (uint32_t)(g / (width + 1)), k = (uint32_t)(g % (width + 1));
  const uint32_t p = a.pub[m];
  uint32_t x = p;
  if (k < width) {
    const uint32_t e = a.ccol ? a.ccol[(size_t)p * CELL_W + k] : a.mesh[(size_t)p * MESH_W + k];
    if (e == EMPTY) return;
    x = e & 0xFFFFFFu;
  }
  a.st[(size_t)x * LP_SW + LP_PUB] = 1u;
}

// The publishers' own lanes: final at time 0 (k_seed's key p), logged first.
__global__ void k_lpub(LPullArgs a, uint32_t Fe) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t FP = a.L / a.B;
  if (g >= a.B * Fe) return;
  const uint32_t m = g / Fe, f = g % Fe, i = m * FP + f;
  if (a.pub[m] - a.u0 >= a.N) return;  // partitioned: another part's publisher
  if (a.pubok && !a.pubok[m]) return;   // churn: an offline publisher publishes nothing
  const uint32_t p = a.pub[m] - a.u0;   // local row
  const uint32_t j = i & 63, q = i >> 6;  // transposed: lane j's u16, bit q
  atomicOr(&a.fin[(size_t)p * LP_FW + (j >> 1)], 1u << (16 * (j & 1) + q));
  if (a.idw) {  // dense keys (IDONTWANT batches)
    a.keys[(size_t)p * a.L + i] = (uint64_t)(p + a.u0);
    return;
  }
  const uint32_t pos = atomicAdd(&a.st[(size_t)p * LP_SW + LP_LOG], 1u);
  a.keys[(size_t)p * a.L + pos] = (uint64_t)(p + a.u0);
  a.flane[(size_t)p * a.L + pos] = (uint16_t)i;
}

// Final logs -> dense [N][L] key rows (INF where nothing arrived), in place:
// one wave per row reads its whole log into LDS before writing the row.
__global__ __launch_bounds__(TB) void k_lfinal(LPullArgs a) {
  __shared__ uint64_t row[PULL_WAVES][PULL_LMAX];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* R = row[wv];
  const uint32_t LL = a.L;
  for (uint32_t w = blockIdx.x * PULL_WAVES + wv; w < a.N; w += gridDim.x * PULL_WAVES) {
    for (uint32_t i = lane; i < LL; i += 64) R[i] = INF64;
    wave_lds_sync();
    const uint32_t n = a.st[(size_t)w * LP_SW + LP_LOG];
    for (uint32_t i0 = 0; i0 < n; i0 += 256) {
      uint64_t k4[4];
      uint32_t l4[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t i = i0 + u * 64 + lane;
        k4[u] = i < n ? a.keys[(size_t)w * LL + i] : INF64;
        l4[u] = i < n ? a.flane[(size_t)w * LL + i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (k4[u] != INF64) R[l4[u]] = k4[u];
    }
    wave_lds_sync();
    for (uint32_t i = lane; i < LL; i += 64) a.keys[(size_t)w * LL + i] = R[i];
    wave_lds_sync();
  }
}

// Completion from the final logs (results kept on the device): the counters
// and per-message reductions of k_complete<FP, false> without dense rows. One
// wave per row scatters the row's log into LDS; lane j keeps the reductions
// of messages j, j + 64, ... in registers over all its rows. A message's key
// at a row is the latest of its F fragments' keys (reassembly, main.rs:79-99:
// none unless all F arrived; never with colliding fragments, defect D8); at a
// non-publisher row it is a delivery; one flush per block through LDS.
// Batch slices (gs_relax.hip run_slices): block row y = slice y, whose rows
// are y * N + w of the key / log buffers, its publishers pub[y * B ..] (peer
// ids) and its reductions mstat[y * B ..].
constexpr uint32_t LC_WAVES = 16;
// With `lat` it also writes each row's logged latencies ([N][B] u16, the
// GS_WANT_LAT_MS stream; GS_LAT_NONE where nothing is logged; one slice).
__global__ __launch_bounds__(LC_WAVES * 64) void k_lcomplete(LPullArgs a, uint64_t* mstat, uint16_t* lat) {
  __shared__ uint64_t R[LC_WAVES][PULL_LMAX];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t B = a.B, stride = gridDim.x * LC_WAVES, FP = a.L / a.B, F = a.F;
  const size_t rbase = (size_t)blockIdx.y * a.N;
  const uint32_t* pub = a.pub + (size_t)blockIdx.y * B;
  if (mstat) mstat += (size_t)blockIdx.y * B * MS_COLS;
  uint64_t tm[PULL_CH];
  uint32_t ud[PULL_CH], pm[PULL_CH];
#pragma unroll
  for (int j = 0; j < (int)PULL_CH; j++) {
    const uint32_t m = j * 64 + lane;
    tm[j] = 0;
    ud[j] = 0;
    pm[j] = m < B ? pub[m] : EMPTY;
  }
  uint64_t deliv = 0, lsum = 0, lmax = 0;
  uint64_t* Rw = R[wv];
  // message m's key at this row (own: the publisher's own key, fragment 0)
  auto mkey = [&](uint32_t m, bool own) -> uint64_t {
    if (FP == 1 || own) return Rw[m * FP];
    if (a.collide) return INF64;
    uint64_t mk = 0;
    for (uint32_t f = 0; f < F; f++) {
      const uint64_t x = Rw[m * FP + f];
      if (x == INF64) return INF64;
      mk = x > mk ? x : mk;
    }
    return mk;
  };
  for (uint32_t w = blockIdx.x * LC_WAVES + wv; w < a.N; w += stride) {
    const size_t wr = rbase + w;
#pragma unroll
    for (int j = 0; j < (int)PULL_CH; j++) Rw[j * 64 + lane] = INF64;
    wave_lds_sync();
    const uint32_t n = a.st[wr * LP_SW + LP_LOG];
    for (uint32_t i0 = 0; i0 < n; i0 += 256) {
      uint64_t k4[4];
      uint32_t l4[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t i = i0 + u * 64 + lane;
        k4[u] = i < n ? a.keys[wr * a.L + i] : INF64;
        l4[u] = i < n ? a.flane[wr * a.L + i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (k4[u] != INF64) Rw[l4[u]] = k4[u];
    }
    wave_lds_sync();
    if (lat) {  // block-uniform
      bool big = false;
#pragma unroll
      for (int j = 0; j < (int)PULL_CH; j++) {
        const uint32_t m = j * 64 + lane;
        if (m >= B) continue;
        const bool own = pm[j] == a.u0 + w;
        const uint64_t x = mkey(m, own);
        uint32_t v = GS_LAT_NONE;
        if (own) {
          if (a.self_log && x != INF64) v = 0;
        } else if (x != INF64) {
          const uint64_t ms = (x >> a.tshift) / 1000000ull;
          big |= ms >= 0xFFFF;
          v = ms < 0xFFFF ? (uint32_t)ms : 0xFFFEu;
        }
        lat[(size_t)w * B + m] = (uint16_t)v;
      }
      if (big) atomicOr((unsigned*)&a.counters[C_ERR], ERR_LAT16);
    }
#pragma unroll
    for (int j = 0; j < (int)PULL_CH; j++) {
      const uint32_t m = j * 64 + lane;
      if (m >= B || pm[j] == a.u0 + w) continue;  // the publisher's own key is no delivery
      const uint64_t x = mkey(m, false);
      if (x == INF64) { ud[j]++; continue; }
      const uint64_t trel = x >> a.tshift, ms = trel / 1000000ull;
      deliv++;
      lsum += ms;
      lmax = ms > lmax ? ms : lmax;
      tm[j] = trel > tm[j] ? trel : tm[j];
    }
    wave_lds_sync();
  }
  deliv = wave_sum(deliv);
  lsum = wave_sum(lsum);
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t x = __shfl_xor(lmax, off);
    lmax = x > lmax ? x : lmax;
  }
  if (lane == 0 && deliv) {
    atomicAdd((unsigned long long*)&a.counters[C_DELIV], (unsigned long long)deliv);
    atomicAdd((unsigned long long*)&a.counters[C_LAT_SUM], (unsigned long long)lsum);
    atomicMax((unsigned long long*)&a.counters[C_LAT_MAX], (unsigned long long)lmax);
  }
  if (!mstat) return;  // block-uniform
  // per-message flush: the waves' values through LDS, one atomic per message and block
  __syncthreads();
#pragma unroll
  for (int j = 0; j < (int)PULL_CH; j++) R[wv][j * 64 + lane] = tm[j];
  __syncthreads();
  for (uint32_t m = threadIdx.x; m < B; m += LC_WAVES * 64) {
    uint64_t t = 0;
    for (uint32_t q = 0; q < LC_WAVES; q++) t = R[q][m] > t ? R[q][m] : t;
    if (t) atomicMax((unsigned long long*)&mstat[(size_t)m * MS_COLS + MS_TMAX], (unsigned long long)t);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < (int)PULL_CH; j++) R[wv][j * 64 + lane] = ud[j];
  __syncthreads();
  for (uint32_t m = threadIdx.x; m < B; m += LC_WAVES * 64) {
    uint64_t u = 0;
    for (uint32_t q = 0; q < LC_WAVES; q++) u += R[q][m];
    if (u) atomicAdd((unsigned long long*)&mstat[(size_t)m * MS_COLS + MS_UNDEL], (unsigned long long)u);
  }
}

// Chunks per row of the pass: 8 when a row has <= 512 lanes (half the LDS,
// twice the resident waves), else 16. GS_LPULL_CH=16 forces the wide form.
uint32_t lpull_chunks(uint32_t L) {
  const char* e = getenv("GS_LPULL_CH");  // per launch: A/B scripts switch it in one process
  return (L <= 512 && !(e && atoi(e) == 16)) ? 8u : 16u;
}

// Partitioned pass: this part's records of the pass (lrec[nb] / lcnt[nb], by
// local row) packed straight into its own range of the next pass's packed
// records of all parts: out = rpk + base (base = this part's offset there, the
// host knows every part's total after the pass) holds them row after row in
// the order rows claim space (one atomic per wave of 64 rows); roff[r] = base +
// the row's offset and rcg[r] = its count go to the own rows of the global
// offset / count tables. Only the other parts' ranges are then exchanged.
__global__ __launch_bounds__(TB) void k_lpack(const uint64_t* __restrict__ rec, const uint32_t* __restrict__ cnt,
                                              uint32_t N, uint32_t L, uint64_t base, uint64_t* __restrict__ out,
                                              uint64_t* __restrict__ roff, uint32_t* __restrict__ rcg,
                                              unsigned long long* cursor) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6), nw = gridDim.x * (TB / 64);
  for (uint32_t r0 = wave * 64; r0 < N; r0 += nw * 64) {
    const uint32_t r = r0 + lane;
    const uint32_t n = r < N ? cnt[r] : 0;
    uint32_t x = n;  // inclusive prefix over the wave's 64 rows
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    const uint32_t tot = __shfl(x, 63);
    unsigned long long b0 = 0;
    if (lane == 0 && tot) b0 = atomicAdd(cursor, (unsigned long long)tot);
    const uint64_t wb = ((uint64_t)__shfl((uint32_t)(b0 >> 32), 0) << 32) | __shfl((uint32_t)b0, 0);
    const uint64_t my = wb + x - n;
    if (r < N) {
      roff[r] = base + my;
      rcg[r] = n;
    }
    for (int j = 0; j < 64; j++) {  // copy row by row, 64 records per step
      const uint32_t nj = __shfl(n, j);
      const uint64_t oj = ((uint64_t)__shfl((uint32_t)(my >> 32), j) << 32) | __shfl((uint32_t)my, j);
      for (uint32_t i = lane; i < nj; i += 64) out[oj + i] = rec[(size_t)(r0 + j) * L + i];
    }
  }
}

// Routed record packing (GS_PART_ROUTE; gs_layout.h
// lp_route_bases): this part's records of a pass, for every destination part q
// the records with a receiver q owns (a bit of the record's inclusion mask at
// a mesh position whose peer is in q; the own part gets every record), each
// row's records contiguous and in emission order. One wave per 64 rows, the
// rows' records walked as one sequence 64 at a time (lane -> record);
// PM (4, 8 or 16) >= P destinations, the loops over them unrolled:
//  0. lane = row: per destination q the mask of the row's mesh entries q owns
//     (smq; bit 16: the own part), from comparisons with the parts' first
//     peers (no division);
//  1. lane = record: per destination one compare of (inclusion mask | valid
//     bit) with the row's mask gives the ballot; each row's run of lanes counts
//     its bits (popcounts of the ballots below the run's last lane), packed two
//     destinations per word, and the run's last lane adds them to LDS;
//  2. all destinations' claims in one atomic instruction (lane q claims
//     cursor[q] for the wave); the per-row offset / count tables are written;
//  3. lane = record again: per destination its position = the row's write
//     position + the run's lanes below it with that bit; the run's last lane
//     stores the row's advanced positions.
// The walk goes LP_RW chunks at a time: one LDS table maps each lane of the
// window to the row starting there, and the window's record loads are issued
// together (its chunks are independent until their LDS updates).
// Destination q's records go to d.out[q], its offset / count tables at this
// part's rows to d.roff[q][r] (+ d.ob[q]) / d.rcg[q][r]: for ranks, send
// segments and tables per destination (the own part: its gathered buffer at
// base 0 and its global tables); for loop-back parts on one device, straight
// into each destination context's gathered buffer and global tables.
constexpr uint32_t LP_PMAX = 16, LP_RW = 8;
struct RouteLo {
  uint32_t lo[LP_PMAX];  // lo[q]: the first peer of part q (gs_layout.h u0)
};
struct RouteDst {
  uint64_t* out[LP_PMAX];   // destination q's records of this part
  uint64_t* roff[LP_PMAX];  // their offsets, by local row
  uint32_t* rcg[LP_PMAX];   // their counts, by local row
  uint64_t ob[LP_PMAX];     // added to the offsets (the segment's base in q's buffer)
  // own_inplace: the own part's records stay where the pass wrote them (row r
  // at element own_off + r * L from the own gathered buffer, modulo 2^64: the
  // pass reads them through the same base + offset); only its tables are written
  uint64_t own_off;
  uint32_t own_inplace;
};
template <uint32_t PM>
__global__ __launch_bounds__(TB) void k_lpack_route(const uint64_t* __restrict__ rec, const uint32_t* __restrict__ cnt,
                                                    const uint32_t* __restrict__ mesh, uint32_t u0, uint32_t un,
                                                    uint32_t L, uint32_t P, uint32_t me, unsigned long long* cursor,
                                                    RouteLo rl, RouteDst d) {
  static_assert(MESH_W == 16 && PM % 4 == 0 && PM <= LP_PMAX, "17-bit masks, uint4 rows");
  constexpr uint32_t VB = 1u << MESH_W;                 // mask bit: a valid record (the own part's)
  __shared__ uint4 smq[TB / 64][64][PM / 4];            // per row: destination q's mask in word q
  __shared__ uint4 sco[TB / 64][64][PM / 4];            // per row: packed counts (16 bits each), then positions
  __shared__ uint32_t spre[TB / 64][64];                // exclusive prefix of the rows' record counts
  __shared__ uint64_t srow[TB / 64][LP_RW * 64 / 8];    // window lane -> the row whose records start there (bytes)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t wave = blockIdx.x * (TB / 64) + wv, nw = gridDim.x * (TB / 64);
  const uint64_t upto = lane == 63 ? ~0ull : (2ull << lane) - 1;  // lanes <= this one
  const uint64_t below = (1ull << lane) - 1;
  uint8_t* const srb = reinterpret_cast<uint8_t*>(srow[wv]);
  auto word = [](const uint4 (&a)[PM / 4], uint32_t q) -> uint32_t {  // (q a constant after unrolling)
    const uint4& h = a[q >> 2];
    return (q & 3) == 0 ? h.x : (q & 3) == 1 ? h.y : (q & 3) == 2 ? h.z : h.w;
  };
  for (uint32_t r0 = wave * 64; r0 < un; r0 += nw * 64) {
    // 0. lane j: row r0 + j — its record count and its destinations' masks
    const uint32_t r = r0 + (uint32_t)lane;
    const bool rv = r < un;
    const uint32_t n = rv ? cnt[r] : 0u;
    uint32_t mq[PM];
#pragma unroll
    for (uint32_t q = 0; q < PM; q++) mq[q] = q == me && !d.own_inplace ? VB : 0u;
    if (rv && d.own_inplace) {  // the own records in place: their row's offset and count
      d.roff[me][r] = d.own_off + (uint64_t)r * L;
      d.rcg[me][r] = n;
    }
    if (rv) {
      const uint4* mp = reinterpret_cast<const uint4*>(mesh + (size_t)(u0 + r) * MESH_W);
#pragma unroll
      for (int k4 = 0; k4 < (int)MESH_W / 4; k4++) {
        const uint4 m = mp[k4];
        const uint32_t e4[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t x = e4[u] & 0xFFFFFFu;  // (EMPTY entries: never a receiver bit)
#pragma unroll
          for (uint32_t q = 0; q < PM; q++) {
            const bool in = q < P && !(q == me && d.own_inplace) && (q == 0 || x >= rl.lo[q]) &&
                            (q + 1 >= P || x < rl.lo[q + 1]);
            mq[q] |= in ? 1u << (4 * k4 + u) : 0u;
          }
        }
      }
    }
#pragma unroll
    for (uint32_t q4 = 0; q4 < PM / 4; q4++) {
      smq[wv][lane][q4] = make_uint4(mq[4 * q4], mq[4 * q4 + 1], mq[4 * q4 + 2], mq[4 * q4 + 3]);
      sco[wv][lane][q4] = make_uint4(0, 0, 0, 0);
    }
    uint32_t x = n;  // inclusive prefix over the 64 rows
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    const uint32_t pre = x - n, T = __shfl(x, 63);
    spre[wv][lane] = pre;
    // One window of LP_RW chunks from t0: each lane's record xr and its mask
    // bits im (inclusion mask | VB if valid), its row j, whether it is its
    // run's last lane, and the run [p0, lane] / [p0, lane).
    struct Chunk {
      uint64_t xr, rle, rlt;
      uint32_t j, im;
      bool last;
    };
    auto window = [&](uint32_t t0, uint32_t& jc, Chunk (&ck)[LP_RW]) {
      srow[wv][lane] = ~0ull;  // no row starts here (yet)
      wave_lds_sync();
      if (n && pre >= t0 && pre - t0 < LP_RW * 64) srb[pre - t0] = (uint8_t)lane;
      wave_lds_sync();
#pragma unroll
      for (uint32_t w = 0; w < LP_RW; w++) {
        const uint32_t t = t0 + 64 * w + (uint32_t)lane;
        const uint32_t here = srb[64 * w + lane];  // the row starting at this lane, or 0xFF
        const uint64_t sm = __ballot(here != 0xFFu);
        const uint64_t sb = sm & upto;
        const uint32_t p0 = sb ? 63u - (uint32_t)__builtin_clzll(sb) : 0u;
        const uint32_t j = sb ? (uint32_t)__shfl((int)here, (int)p0) : jc;
        jc = (uint32_t)__builtin_amdgcn_readlane((int)j, 63);
        const bool v = t < T;
        const uint64_t from = ~((1ull << p0) - 1);
        ck[w].j = j;
        ck[w].rle = upto & from;
        ck[w].rlt = below & from;
        ck[w].last = v && (lane == 63 || ((sm >> (lane + 1)) & 1) || t + 1 == T);
        ck[w].xr = v ? rec[(size_t)(r0 + j) * L + (t - spre[wv][j])] : 0ull;
      }
#pragma unroll
      for (uint32_t w = 0; w < LP_RW; w++) {
        const bool v = t0 + 64 * w + (uint32_t)lane < T;
        ck[w].im = v ? ((((uint32_t)ck[w].xr >> LP_IM_SHIFT) & (VB - 1)) | VB) : 0u;
      }
    };
    // 1. counts per (row, destination)
    uint32_t jc = 0;  // the row continuing into the chunk (its start lies before it)
    for (uint32_t t0 = 0; t0 < T; t0 += LP_RW * 64) {
      Chunk ck[LP_RW];
      window(t0, jc, ck);
#pragma unroll
      for (uint32_t w = 0; w < LP_RW; w++) {
        if (t0 + 64 * w >= T) break;  // (wave-uniform)
        uint4 m[PM / 4];
#pragma unroll
        for (uint32_t q4 = 0; q4 < PM / 4; q4++) m[q4] = smq[wv][ck[w].j][q4];
        uint32_t pk[PM / 2];  // the run's counts so far, two destinations per word
#pragma unroll
        for (uint32_t q = 0; q < PM; q++) {
          const uint64_t bq = __ballot((ck[w].im & word(m, q)) != 0u);
          const uint32_t c = (uint32_t)__popcll(bq & ck[w].rle);
          pk[q >> 1] = (q & 1) ? pk[q >> 1] | (c << 16) : c;
        }
        if (ck[w].last) {
          uint32_t* row = reinterpret_cast<uint32_t*>(&sco[wv][ck[w].j][0]);
#pragma unroll
          for (uint32_t h = 0; h < PM / 2; h++) row[h] += pk[h];
        }
      }
      wave_lds_sync();  // (srow is rewritten by the next window)
    }
    // 2. offsets: one claim per destination, all in one instruction; sco
    // becomes each (row, destination)'s write position
    uint32_t pk[PM / 2];
    {
      const uint32_t* row = reinterpret_cast<const uint32_t*>(&sco[wv][lane][0]);
#pragma unroll
      for (uint32_t h = 0; h < PM / 2; h++) pk[h] = row[h];
    }
    uint32_t pos[PM], mytot = 0;
#pragma unroll
    for (uint32_t q = 0; q < PM; q++) {
      const uint32_t c = (pk[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
      uint32_t y = c;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t z = __shfl_up(y, off);
        if (lane >= off) y += z;
      }
      pos[q] = y - c;  // within the wave
      if (q < P && rv && !(q == me && d.own_inplace)) d.rcg[q][r] = c;
      const uint32_t tot = __shfl(y, 63);
      if ((uint32_t)lane == q) mytot = tot;
    }
    const unsigned long long b0 = mytot ? atomicAdd(&cursor[lane], (unsigned long long)mytot) : 0ull;
#pragma unroll
    for (uint32_t q = 0; q < PM; q++) {
      const uint64_t off = (((uint64_t)__shfl((uint32_t)(b0 >> 32), (int)q) << 32) | __shfl((uint32_t)b0, (int)q)) +
                           pos[q];
      pos[q] = (uint32_t)off;  // (< cap < 2^32)
      if (q < P && rv && !(q == me && d.own_inplace)) d.roff[q][r] = d.ob[q] + off;
    }
#pragma unroll
    for (uint32_t q4 = 0; q4 < PM / 4; q4++)
      sco[wv][lane][q4] = make_uint4(pos[4 * q4], pos[4 * q4 + 1], pos[4 * q4 + 2], pos[4 * q4 + 3]);
    wave_lds_sync();
    // 3. copy in emission order
    jc = 0;
    for (uint32_t t0 = 0; t0 < T; t0 += LP_RW * 64) {
      Chunk ck[LP_RW];
      window(t0, jc, ck);
#pragma unroll
      for (uint32_t w = 0; w < LP_RW; w++) {
        if (t0 + 64 * w >= T) break;  // (wave-uniform)
        const uint32_t j = ck[w].j;
        uint4 m[PM / 4], b[PM / 4];  // the row's masks and write positions (read before its last lane moves them)
#pragma unroll
        for (uint32_t q4 = 0; q4 < PM / 4; q4++) {
          m[q4] = smq[wv][j][q4];
          b[q4] = sco[wv][j][q4];
        }
        uint32_t nb[PM];
#pragma unroll
        for (uint32_t q = 0; q < PM; q++) {
          const bool s = (ck[w].im & word(m, q)) != 0u;
          const uint64_t bq = __ballot(s);
          const uint32_t base = word(b, q);
          if (s) d.out[q][(uint64_t)base + (uint32_t)__popcll(bq & ck[w].rlt)] = ck[w].xr;
          nb[q] = base + (uint32_t)__popcll(bq & ck[w].rle);
        }
        if (ck[w].last) {
#pragma unroll
          for (uint32_t q4 = 0; q4 < PM / 4; q4++)
            sco[wv][j][q4] = make_uint4(nb[4 * q4], nb[4 * q4 + 1], nb[4 * q4 + 2], nb[4 * q4 + 3]);
        }
      }
      wave_lds_sync();
    }
  }
}

// The receiver's offsets of the routed records: a foreign peer's offset is
// relative to its part's segment; add the segment's base in the gathered buffer.
struct RouteBases {
  uint64_t b[LP_PMAX];
};
__global__ __launch_bounds__(TB) void k_roff_fix(uint64_t* __restrict__ roff, uint32_t N, uint32_t P, uint32_t me,
                                                 RouteBases rb) {
  const uint32_t x = blockIdx.x * TB + threadIdx.x;
  if (x >= N) return;
  const uint32_t p = (uint32_t)((((uint64_t)x + 1) * P - 1) / N);  // gs_layout.h part_of
  if (p != me) roff[x] += rb.b[p];
}

// Loop-back parts on one device: after every part's pass, one wave combines
// the parts' pass control as the host would (gs_comm.hip run_batch_lp): lane
// p reads part p's slot {mode, records, min pending} and error word into
// st[p * 4 ..], and every part's slot gets the sum of the records and the min
// of the pending keys (part_lp_set's values) — one launch and one read-back
// instead of a read and a write per part.
struct PartCtl {
  uint64_t* ctrl[LP_PMAX];       // part p's pass control slots [3][4]
  const uint64_t* err[LP_PMAX];  // part p's error word (counters + C_ERR)
};
__global__ __launch_bounds__(64) void k_part_combine(PartCtl pc, uint32_t P, uint32_t slot, uint64_t* __restrict__ st) {
  const uint32_t p = threadIdx.x;
  const bool v = p < P;
  uint64_t* s = v ? pc.ctrl[p] + slot * 4 : nullptr;
  const uint64_t mode = v ? s[1] : 0, rec = v ? s[2] : 0, mn = v ? s[3] : INF64, er = v ? *pc.err[p] : 0;
  uint64_t sum = rec, lo = mn;
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(sum >> 32), off) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)sum, off);
    const uint64_t z = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(lo >> 32), off) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)lo, off);
    sum += y;
    lo = z < lo ? z : lo;
  }
  if (v) {
    st[p * 4 + 0] = mode;
    st[p * 4 + 1] = rec;
    st[p * 4 + 2] = mn;
    st[p * 4 + 3] = er;
    s[2] = sum;
    s[3] = lo;
  }
}

void lpull_dispatch_part(uint32_t FP, const LPullArgs& a, unsigned grid, hipStream_t s) {
  const bool ch8 = lpull_chunks(a.L) == 8;
#define GS_LPP(F)                                                      \
  if (ch8) k_lpull<F, 8, false, true><<<grid, TB, 0, s>>>(a);           \
  else k_lpull<F, 16, false, true><<<grid, TB, 0, s>>>(a);
  switch (FP) {
    case 1: GS_LPP(1) break;
    case 2: GS_LPP(2) break;
    case 4: GS_LPP(4) break;
    case 8: GS_LPP(8) break;
    default: GS_LPP(16) break;
  }
#undef GS_LPP
}

// One pass of a GOS batch: its control, the sender planes when a heartbeat's
// senders just became final, the pass itself (rows of one fragment).
// The churn list pass (CHN) by fragment lanes per message and chunks per row.
template <bool GOS>
void lpull_dispatch_chn(uint32_t FP, const LPullArgs& a, unsigned grid, hipStream_t s) {
#define GS_LPC(F)                                                                             \
  if (lpull_chunks(a.L) == 8) k_lpull<F, 8, false, false, GOS, true><<<grid, TB, 0, s>>>(a);  \
  else k_lpull<F, 16, false, false, GOS, true><<<grid, TB, 0, s>>>(a)
  switch (FP) {
    case 1: GS_LPC(1); break;
    case 2: GS_LPC(2); break;
    case 4: GS_LPC(4); break;
    case 8: GS_LPC(8); break;
    default: GS_LPC(16); break;
  }
#undef GS_LPC
}

void lpull_dispatch_gos(const LPullArgs& a, unsigned grid, hipStream_t s) {
  k_lctl<<<1, 64, 0, s>>>(a);
  const uint32_t FP = a.L / a.B;  // fragment lanes per message (rows of fragment groups: one lane per fragment)
  if (a.ccol) {  // churn
    if (lpull_chunks(a.L) == 8) k_gsend<8, true><<<grid, TB, 0, s>>>(a);
    else k_gsend<16, true><<<grid, TB, 0, s>>>(a);
    lpull_dispatch_chn<true>(FP, a, grid, s);
    return;
  }
  if (a.idw) {  // IDONTWANT (FP == 1: the host sends fragmented IDONTWANT batches to the push path)
    if (lpull_chunks(a.L) == 8) {
      k_gsend<8><<<grid, TB, 0, s>>>(a);
      k_lpull<1, 8, true, false, true><<<grid, TB, 0, s>>>(a);
    } else {
      k_gsend<16><<<grid, TB, 0, s>>>(a);
      k_lpull<1, 16, true, false, true><<<grid, TB, 0, s>>>(a);
    }
    return;
  }
  if (lpull_chunks(a.L) == 8) {
    k_gsend<8><<<grid, TB, 0, s>>>(a);
    switch (FP) {
      case 1: k_lpull<1, 8, false, false, true><<<grid, TB, 0, s>>>(a); break;
      case 2: k_lpull<2, 8, false, false, true><<<grid, TB, 0, s>>>(a); break;
      case 4: k_lpull<4, 8, false, false, true><<<grid, TB, 0, s>>>(a); break;
      case 8: k_lpull<8, 8, false, false, true><<<grid, TB, 0, s>>>(a); break;
      default: k_lpull<16, 8, false, false, true><<<grid, TB, 0, s>>>(a); break;
    }
  } else {
    k_gsend<16><<<grid, TB, 0, s>>>(a);
    switch (FP) {
      case 1: k_lpull<1, 16, false, false, true><<<grid, TB, 0, s>>>(a); break;
      case 2: k_lpull<2, 16, false, false, true><<<grid, TB, 0, s>>>(a); break;
      case 4: k_lpull<4, 16, false, false, true><<<grid, TB, 0, s>>>(a); break;
      case 8: k_lpull<8, 16, false, false, true><<<grid, TB, 0, s>>>(a); break;
      default: k_lpull<16, 16, false, false, true><<<grid, TB, 0, s>>>(a); break;
    }
  }
}

void lpull_dispatch(uint32_t FP, const LPullArgs& a, unsigned grid, hipStream_t s) {
  if (a.ccol) {  // churn without lazy gossip (rows of fragment groups: FP lanes per message)
    lpull_dispatch_chn<false>(FP, a, grid, s);
    return;
  }
  if (a.idw) {  // FP == 1 (the host sends fragmented IDONTWANT batches to the push path)
    if (lpull_chunks(a.L) == 8) k_lpull<1, 8, true><<<grid, TB, 0, s>>>(a);
    else k_lpull<1, 16, true><<<grid, TB, 0, s>>>(a);
    return;
  }
  if (lpull_chunks(a.L) == 8) {
    switch (FP) {
      case 1: k_lpull<1, 8><<<grid, TB, 0, s>>>(a); break;
      case 2: k_lpull<2, 8><<<grid, TB, 0, s>>>(a); break;
      case 4: k_lpull<4, 8><<<grid, TB, 0, s>>>(a); break;
      case 8: k_lpull<8, 8><<<grid, TB, 0, s>>>(a); break;
      default: k_lpull<16, 8><<<grid, TB, 0, s>>>(a); break;
    }
    return;
  }
  switch (FP) {
    case 1: k_lpull<1, 16><<<grid, TB, 0, s>>>(a); break;
    case 2: k_lpull<2, 16><<<grid, TB, 0, s>>>(a); break;
    case 4: k_lpull<4, 16><<<grid, TB, 0, s>>>(a); break;
    case 8: k_lpull<8, 16><<<grid, TB, 0, s>>>(a); break;
    default: k_lpull<16, 16><<<grid, TB, 0, s>>>(a); break;
  }
}
