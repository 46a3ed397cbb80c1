// gs_pull_kernel.h — owner-computes Delta-window pass, the default eager
// forwarding path. Included by gs_relax.hip after
// gs_relax_kernel.h (inside namespace gs::{anon}).
//
// Why: the push path (k_scan + k_frontier) issues one random 64-bit atomicMin
// per improving send. On gfx950 a random 8-byte atomic into an HBM-sized table
// runs at ~18 G/s chip-wide (scripts/ubench_mem.hip), and k_frontier sat on
// that floor. Here every key row is written by its owner only:
//
//   one wave owns peer w's row keys[w][0..L) for the pass; it
//    1. loads the row's live 64-lane chunks into registers (L <= 1024: up to
//       16 chunks of 64 lanes),
//    2. PULL passes: reads the arrival records its mesh neighbours u emitted
//       for window [lo, lo+D) in the previous pass — all neighbours' records
//       in one flattened loop — and re-derives each forward u -> w exactly as
//       relax_lane/k_precv do (w's position in mesh(u) \ {src, publisher},
//       u's uplink start, link latency), min-reducing them in an LDS buffer,
//    3. merges, writes changed lanes back, and emits its own arrivals of the
//       next window as 8-byte records for the pass after,
//    4. keeps chunkmin[w][q] = hi word of the min pending key of chunk q
//       beyond that window. A chunk is live in a pass (read from HBM) only if
//       it holds a key due in the emitted window or receives a candidate; rows
//       with neither cost one 64-B read. Windows on the rising and falling
//       edge of a batch touch a few of a row's 16 chunks, the peak windows
//       all of them.
//
// Record (u64): start - window_lo (32) | hops (6) | j_src (5) | j_pub (5) |
// slot (16), where j_src / j_pub are the indices of the sender's source and of
// the message's publisher in the sender's mesh row (31 = not in the mesh). A
// receiver w at index r = rpos[w][j] of mesh(u) is skipped if r is j_src or
// j_pub, else its position is r + 1 - [j_src < r] - [j_pub < r, j_pub != j_src]
// (mesh rows are sorted by id, so index order is id order).
//
// Exactness is the Delta-stepping argument of the push path: every send adds
// >= D, so after applying window b's candidates all keys below the end of
// window b+1 are final. Candidates are the same keys the push path atomically
// min-reduces, so the result is bit-identical. A chunk that is not live keeps
// its keys and its chunkmin (>= the window end, so still the min beyond it).
//
// Control (device side, no host round trip per pass): ctrl holds three slots
// of {lo, mode, records emitted, min pending}. Pass k decides from slot k-1:
//   records > 0  -> PULL the window whose records were just emitted;
//   else min < INF -> EMIT the window holding the min pending key (a gap);
//   else DONE.

enum : uint64_t { PM_DONE = 0, PM_EMIT = 1, PM_PULL = 2 };
constexpr uint32_t PULL_WAVES = TB / 64;  // rows in flight per block
constexpr uint32_t PULL_LMAX = 1024;       // row lanes held in registers (16 chunks)
constexpr uint32_t PULL_CH = PULL_LMAX / 64;
constexpr uint32_t J_NONE = 31;
static_assert(PULL_CH == MESH_W, "row header lane j carries mesh entry j and chunk j");

struct PullArgs {
  uint64_t* keys;       // [N][L]
  uint64_t* busy;       // [N][B] uplink FIFO end per (peer, message), FP > 1
  uint32_t* chunkmin;   // [N][PULL_CH] hi word of the min pending key per chunk (~0 = none)
  uint64_t* lrec;       // [2][N][L] per-row arrival records
  uint32_t* lcnt;       // [2][N]
  const uint32_t* mesh;
  const uint8_t* rpos;  // [N][MESH_W] index of w in mesh(mesh[w][j])
  const uint32_t* pub;
  const uint8_t* stage;
  const uint32_t* tables;  // lat[S*S] | ser_up[S] | ser_dn[S] (read with scalar loads)
  uint64_t* ctrl;          // [3][4]
  uint64_t* counters;
  uint64_t delta, tmax;
  uint32_t N, B, L, S, sb, tshift, pass;
};

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t umin32(uint32_t x, uint32_t y) { return x < y ? x : y; }

// Lane l receives the wave-wide min of x[l >> 2]: recursive halving over the
// 16 chunk values (17 shuffles instead of 16 full 6-step reductions).
__device__ __forceinline__ uint32_t chunk_min_scatter(const uint32_t (&x)[PULL_CH], int lane) {
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8, b2 = lane & 4;
  uint32_t a8[8], a4[4], a2[2];
#pragma unroll
  for (int i = 0; i < 8; i++) a8[i] = umin32(b5 ? x[i + 8] : x[i], __shfl_xor(b5 ? x[i] : x[i + 8], 32));
#pragma unroll
  for (int i = 0; i < 4; i++) a4[i] = umin32(b4 ? a8[i + 4] : a8[i], __shfl_xor(b4 ? a8[i] : a8[i + 4], 16));
#pragma unroll
  for (int i = 0; i < 2; i++) a2[i] = umin32(b3 ? a4[i + 2] : a4[i], __shfl_xor(b3 ? a4[i] : a4[i + 2], 8));
  uint32_t a1 = umin32(b2 ? a2[1] : a2[0], __shfl_xor(b2 ? a2[0] : a2[1], 4));
  a1 = umin32(a1, __shfl_xor(a1, 2));
  return umin32(a1, __shfl_xor(a1, 1));
}

// Per wave: CW = the row's candidate minima, then (in place) the compacted
// arrivals; LST = their group indices. 10 KB per wave, 4 blocks per CU.
struct PullLds {
  uint64_t cw[PULL_WAVES][PULL_LMAX];
  uint16_t lst[PULL_WAVES][PULL_LMAX];
};

#ifdef GS_PULL_PROF
// Diagnostic build only (scripts/pull_prof.py): per pass, summed over waves,
// the shader clocks spent in each step of the row loop.
__device__ unsigned long long g_pull_prof[32][8];
#define PP_T(v) const uint64_t v = clock64()
#define PP_ADD(k, x) pp[k] += (x)
#else
#define PP_T(v)
#define PP_ADD(k, x)
#endif

template <int FP>
__global__ __launch_bounds__(TB, 4) void k_pull(PullArgs a) {
  __shared__ PullLds Ls;
  // ---- decide this pass from the previous slot (grid-uniform) ----
  const uint64_t* pv = a.ctrl + ((a.pass + 2) % 3) * 4;
  uint64_t lo, mode;
  if (pv[1] != PM_DONE && pv[2]) { mode = PM_PULL; lo = pv[1] == PM_PULL ? pv[0] + a.delta : pv[0]; }
  else if (pv[3] != INF64) { mode = PM_EMIT; lo = ((pv[3] >> a.tshift) / a.delta) * a.delta; }
  else { mode = PM_DONE; lo = pv[0]; }
  uint64_t* me = a.ctrl + (a.pass % 3) * 4;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    me[0] = lo;
    me[1] = mode;
    uint64_t* nx = a.ctrl + ((a.pass + 1) % 3) * 4;
    nx[2] = 0;
    nx[3] = INF64;
    if (mode != PM_DONE) atomicAdd((unsigned long long*)&a.counters[C_PASSES], 1ull);
    if (mode == PM_PULL) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
  }
  if (mode == PM_DONE) return;

  const bool pull = mode == PM_PULL;
  const uint64_t wlo = pull ? lo + a.delta : lo;  // the window this pass emits
  const uint64_t whi = wlo + a.delta;
  // The window in key space. Window bounds are multiples of 2^(32 - tshift) ns
  // (the host rounds D down to that grain), so a key's position relative to
  // them is decided by its high 32 bits alone; keys stay below hi word
  // 0xFFFFFFFF (tmax is lowered by one grain), which is kept for INF.
  const uint64_t lok = wlo > a.tmax ? INF64 : wlo << a.tshift;
  const uint64_t hik = whi > a.tmax ? INF64 : whi << a.tshift;
  const uint32_t hlo = (uint32_t)(lok >> 32), hhi = (uint32_t)(hik >> 32), hspan = hhi - hlo;
  const uint32_t LL = a.L, S = a.S;
  const size_t NL = (size_t)a.N * LL;
  const uint32_t pb = (a.pass + 1) & 1, nb = a.pass & 1;  // records read / written
  const uint64_t* rrec = a.lrec + pb * NL;
  const uint32_t* rcnt = a.lcnt + (size_t)pb * a.N;
  uint64_t* wrec = a.lrec + nb * NL;
  uint32_t* wcnt = a.lcnt + (size_t)nb * a.N;
  const uint32_t* lat = a.tables;
  const uint32_t* sup = a.tables + S * S;
  const uint32_t* sdn = a.tables + S * S + S;

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* CW = Ls.cw[wv];
  uint16_t* LST = Ls.lst[wv];
  const uint64_t smask = (1ull << a.sb) - 1;
  const uint32_t hmask = (1u << HOP_BITS) - 1;
  const uint64_t lanelt = (1ull << lane) - 1;
  uint64_t fd = 0, nr = 0, np = 0, nrec = 0;
  uint32_t nmh = ~0u;  // hi word of the min pending key over this wave's rows
  uint32_t err = 0;
#ifdef GS_PULL_PROF
  uint64_t pp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

  // Row headers are software-pipelined one row ahead: lane j < 16 holds mesh
  // entry j of the row, w's index in that neighbour's row, the length of the
  // neighbour's record list, and chunk j's pending min. The next row's entries
  // are loaded while this row is processed, its list lengths after step 2.
  const uint32_t stride = gridDim.x * PULL_WAVES;
  uint32_t w = blockIdx.x * PULL_WAVES + wv;
  uint32_t ej = EMPTY, cj = 0, rj = 0, cm = ~0u;
  if (w < a.N && lane < (int)MESH_W) {
    ej = a.mesh[(size_t)w * MESH_W + lane];
    rj = a.rpos[(size_t)w * MESH_W + lane];
    if (pull && ej != EMPTY) cj = rcnt[ej & 0xFFFFFFu];
    cm = a.chunkmin[(size_t)w * PULL_CH + lane];
  }
  for (; w < a.N; w += stride) {
    PP_T(tA);
    const uint32_t w2 = w + stride;
    uint32_t ej2 = EMPTY, rj2 = 0, cj2 = 0, cm2 = ~0u;
    if (w2 < a.N && lane < (int)MESH_W) {  // w2 < N is wave-uniform
      ej2 = a.mesh[(size_t)w2 * MESH_W + lane];
      rj2 = a.rpos[(size_t)w2 * MESH_W + lane];
      cm2 = a.chunkmin[(size_t)w2 * PULL_CH + lane];
    }
    const uint64_t cand = __ballot(cj != 0);
    // chunks holding a key due in [wlo, whi) (chunkmin never drops below the
    // emitted windows: keys below wlo are final and were emitted earlier)
    uint32_t live = (uint32_t)__ballot(cm < hhi);
    if (cand == 0 && live == 0) {  // nothing to apply, nothing due
      if (lane == 0) wcnt[w] = 0;
      nmh = umin32(nmh, cm);
      if (pull && lane < (int)MESH_W && ej2 != EMPTY) cj2 = rcnt[ej2 & 0xFFFFFFu];
      ej = ej2; rj = rj2; cj = cj2; cm = cm2;
      PP_T(tS);
      PP_ADD(0, tS - tA);
      continue;
    }
    PP_ADD(5, 1);
    // 1. the due chunks into registers (up to 16 loads in flight per lane)
    const uint64_t* grow = a.keys + (size_t)w * LL;
    uint64_t v[PULL_CH];
#pragma unroll
    for (int q = 0; q < (int)PULL_CH; q++) {
      const uint32_t i = q * 64 + lane;
      v[q] = ((live >> q) & 1u) && i < LL ? grow[i] : INF64;
    }
    const uint32_t sw = a.stage[w];
    if (pull) {
#pragma unroll
      for (int q = 0; q < (int)PULL_CH; q++) CW[q * 64 + lane] = INF64;
      wave_lds_sync();
      // 2. the neighbours' records: lists in groups of 4, two 64-record chunks
      //    each, so up to 8 independent record loads per lane are in flight
      const uint32_t sd = sdn[sw];
      uint64_t cmk = cand;
      uint32_t cb = 0;  // chunks that receive a candidate
      while (cmk) {
        uint32_t U[4], R4[4], NN[4], SER[4];
        uint64_t BASE[4];
        uint32_t maxn = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          U[k] = 0; R4[k] = 0; NN[k] = 0; SER[k] = 0; BASE[k] = 0;
          if (cmk) {  // wave-uniform
            const int j = __builtin_ctzll(cmk);
            cmk &= cmk - 1;
            const uint32_t e = __builtin_amdgcn_readlane(ej, j);
            U[k] = e & 0xFFFFFFu;
            R4[k] = __builtin_amdgcn_readlane(rj, j);
            NN[k] = __builtin_amdgcn_readlane(cj, j);
            const uint32_t su = e >> STAGE_SHIFT;
            SER[k] = sup[su];
            BASE[k] = lo + lat[su * S + sw] + (sd > SER[k] ? sd - SER[k] : 0);
            maxn = NN[k] > maxn ? NN[k] : maxn;
          }
        }
        for (uint32_t i0 = 0; i0 < maxn; i0 += 128) {
          uint64_t rec[4][2];
#pragma unroll
          for (int k = 0; k < 4; k++)
#pragma unroll
            for (int c = 0; c < 2; c++) {
              const uint32_t i = i0 + c * 64 + lane;
              rec[k][c] = i < NN[k] ? rrec[(size_t)U[k] * LL + i] : ~0ull;
            }
#pragma unroll
          for (int k = 0; k < 4; k++)
#pragma unroll
            for (int c = 0; c < 2; c++) {
              const uint64_t rc = rec[k][c];
              if (rc == ~0ull) continue;  // no record (records never have all bits set)
              const uint32_t lo32 = (uint32_t)rc, r = R4[k];
              const uint32_t js = (lo32 >> 21) & 31u, jp = (lo32 >> 16) & 31u;
              if (js == r || jp == r) continue;  // w is the source or the publisher
              const uint32_t pos = r + 1 - (js < r ? 1u : 0u) - ((jp < r && jp != js) ? 1u : 0u);
              const uint64_t arr = BASE[k] + (rc >> 32) + (uint64_t)(pos * SER[k]);
              if (arr > a.tmax) err |= ERR_TIME;
              const uint64_t hp1 = ((lo32 >> 26) & hmask) + 1;
              const uint64_t nk = (arr << a.tshift) | (hp1 << a.sb) | U[k];
              const uint32_t slot = lo32 & 0xFFFFu;
              atomicMin((unsigned long long*)&CW[slot], (unsigned long long)nk);
              cb |= 1u << (slot >> 6);
            }
        }
      }
      for (int off = 32; off > 0; off >>= 1) cb |= __shfl_xor(cb, off);
      cb = __builtin_amdgcn_readfirstlane(cb);
      // 1b. chunks live only through candidates
      const uint32_t extra = cb & ~live;
      live |= cb;
#pragma unroll
      for (int q = 0; q < (int)PULL_CH; q++) {
        const uint32_t i = q * 64 + lane;
        if ((extra >> q) & 1u) v[q] = i < LL ? grow[i] : INF64;
      }
      wave_lds_sync();
    }
    if (pull && lane < (int)MESH_W && ej2 != EMPTY) cj2 = rcnt[ej2 & 0xFFFFFFu];  // next row's lists
    PP_T(tB);
    PP_ADD(1, tB - tA);
    // 3. dense: merge, write back changed lanes, compact the arrivals of
    //    [wlo, whi) in place (groups of FP lanes), per-chunk min beyond it
    const bool chk_pub = wlo == 0;  // only window 0 can hold a publisher's own key
    uint32_t cnt = 0;               // compacted groups
    uint32_t lq[PULL_CH];           // this lane's key beyond the window, per chunk
#pragma unroll
    for (int q = 0; q < (int)PULL_CH; q++) {
      lq[q] = ~0u;
      if (q * 64 < (int)LL && ((live >> q) & 1u)) {  // wave-uniform
        const uint32_t i = q * 64 + lane;
        const bool valid = i < LL;
        uint64_t x = v[q];
        if (pull) {
          const uint64_t c = valid ? CW[i] : INF64;
          const bool chg = c < x;
          if (chg) {
            x = c;
            np++;
          }
          // write back whole 64-B sectors that hold a changed lane: a partial
          // sector store costs a read-modify-write (random single-lane stores
          // into an 8 GB table run at 22 G/s, full sectors at 383 G/s,
          // profiles/r01_v6/ubench_mem.json)
          const uint64_t cm8 = __ballot(chg);
          if (valid && ((cm8 >> (lane & 56)) & 0xFFull)) a.keys[(size_t)w * LL + i] = x;
        }
        const uint32_t hx = (uint32_t)(x >> 32);
        bool act = valid && (hx - hlo) < hspan;
        if (chk_pub && act) act = a.pub[i / FP] != w;
        lq[q] = hx >= hhi ? hx : ~0u;
        const uint64_t am = __ballot(act);
        if (am) {  // wave-uniform
          if constexpr (FP == 1) {
            if (act) {
              const uint32_t k = cnt + (uint32_t)__popcll(am & lanelt);
              CW[k] = x;
              LST[k] = (uint16_t)i;
            }
            cnt += (uint32_t)__popcll(am);
          } else {
            constexpr uint64_t gmask = (FP == 64) ? ~0ull : ((1ull << FP) - 1);
            const int gb = lane & ~(FP - 1);
            const bool gact = ((am >> gb) & gmask) != 0;
            const uint64_t lm = __ballot(gact && (lane & (FP - 1)) == 0);  // group leaders
            const uint32_t k = cnt + (uint32_t)__popcll(lm & ((1ull << gb) - 1));
            if (gact) {
              CW[k * FP + (lane & (FP - 1))] = x;
              if ((lane & (FP - 1)) == 0) LST[k] = (uint16_t)(i / FP);
            }
            cnt += (uint32_t)__popcll(lm);
          }
        }
      }
    }
    wave_lds_sync();
    PP_T(tC);
    PP_ADD(2, tC - tB);
    // 4. sparse: forward targets, uplink FIFO and one record per arrival
    uint32_t ecnt = 0;
    if (cnt) {
      const uint32_t deg = (uint32_t)__popcll(__ballot(ej != EMPTY));  // rows are packed
      const uint32_t serw = sup[sw];
      constexpr uint32_t GPW = 64 / FP;
      for (uint32_t g0 = 0; g0 < cnt; g0 += GPW) {
        const uint32_t gi = g0 + (uint32_t)lane / FP;
        const bool gv = gi < cnt;
        const uint32_t grp = gv ? LST[gi] : 0;
        const uint32_t i = grp * FP + (lane & (FP - 1));
        const uint64_t x = gv ? CW[gi * FP + (lane & (FP - 1))] : INF64;
        const uint32_t pm = gv ? a.pub[grp] : EMPTY;
        const bool act = gv && ((uint32_t)(x >> 32) - hlo) < hspan && w != pm;
        const uint32_t src = (uint32_t)(x & smask);
        uint32_t js = J_NONE, jp = J_NONE;  // indices of src / publisher in mesh(w)
        for (uint32_t k = 0; k < deg; k++) {  // wave-uniform: entry k from lane k
          const uint32_t y = __builtin_amdgcn_readlane(ej, k) & 0xFFFFFFu;
          js = y == src ? k : js;
          jp = y == pm ? k : jp;
        }
        // targets: mesh(w) \ {src, publisher}
        const uint32_t n = act ? deg - (js != J_NONE ? 1u : 0u) - ((jp != J_NONE && jp != js) ? 1u : 0u) : 0u;
        const uint64_t start = uplink_start<FP>(a.busy, (size_t)w * a.B + grp, act, x, n, serw, a.tshift);
        const uint32_t hp = (uint32_t)(x >> a.sb) & hmask;
        if (act) {
          fd++;
          nr += n;
          if (n && hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
          if (start - wlo >= (1ull << 32)) err |= ERR_TIME;
        }
        const bool want = act && n != 0;
        const uint64_t wm = __ballot(want);
        if (want)
          wrec[(size_t)w * LL + ecnt + (uint32_t)__popcll(wm & lanelt)] =
              ((start - wlo) << 32) | ((uint64_t)hp << 26) | ((uint64_t)js << 21) | ((uint64_t)jp << 16) | i;
        ecnt += (uint32_t)__popcll(wm);
      }
    }
    PP_T(tD);
    PP_ADD(3, tD - tC);
    // 5. new chunk minima: lanes 4c..4c+3 hold chunk c's; chunks that were not
    //    live keep theirs (their keys did not change and lie beyond the window)
    {
      const uint32_t red = chunk_min_scatter(lq, lane);
      const uint32_t c = (uint32_t)lane >> 2;
      const uint32_t oldc = (uint32_t)__shfl((int)cm, (int)c);
      const bool lc = (live >> c) & 1u;
      const uint32_t ncm = lc ? red : oldc;
      if ((lane & 3) == 0) a.chunkmin[(size_t)w * PULL_CH + c] = ncm;  // the whole 64-B sector
      nmh = umin32(nmh, ncm);
    }
    if (lane == 0) wcnt[w] = ecnt;
    nrec += ecnt;
    ej = ej2; rj = rj2; cj = cj2; cm = cm2;
    PP_T(tE);
    PP_ADD(4, tE - tD);
  }
#ifdef GS_PULL_PROF
  if (lane == 0 && a.pass < 32)
    for (int k = 0; k < 6; k++) atomicAdd(&g_pull_prof[a.pass][k], (unsigned long long)pp[k]);
#endif
  for (int off = 32; off > 0; off >>= 1) nmh = umin32(nmh, __shfl_xor(nmh, off));
  const uint64_t nmin = nmh == ~0u ? INF64 : (uint64_t)nmh << 32;
  fd = wave_sum(fd);
  nr = wave_sum(nr);
  np = wave_sum(np);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if (lane == 0) {
    if (nrec) atomicAdd((unsigned long long*)&me[2], (unsigned long long)nrec);
    if (nmin != INF64) atomicMin((unsigned long long*)&me[3], (unsigned long long)nmin);
    if (fd) atomicAdd((unsigned long long*)&a.counters[C_FD], (unsigned long long)fd);
    if (nr) atomicAdd((unsigned long long*)&a.counters[C_R_FWD], (unsigned long long)nr);
    if (np) atomicAdd((unsigned long long*)&a.counters[C_PUSH], (unsigned long long)np);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
}

// rpos[w][j] = index of w in mesh(mesh[w][j]) (the mesh is symmetric, so it
// exists); 0 for EMPTY entries. Once per mesh.
__global__ __launch_bounds__(TB) void k_rpos(const uint32_t* __restrict__ mesh, uint8_t* __restrict__ rpos,
                                             uint32_t N, uint64_t* counters) {
  const uint64_t g = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (g >= (uint64_t)N * MESH_W) return;
  const uint32_t w = (uint32_t)(g / MESH_W);
  const uint32_t e = mesh[g];
  uint8_t r = 0;
  if (e != EMPTY) {
    const uint32_t* ur = mesh + (size_t)(e & 0xFFFFFFu) * MESH_W;
    uint32_t k = 0;
    while (k < MESH_W && ur[k] != EMPTY && (ur[k] & 0xFFFFFFu) != w) k++;
    if (k == MESH_W || ur[k] == EMPTY) atomicOr((unsigned*)&counters[C_ERR], ERR_MESH);  // asymmetric
    r = (uint8_t)k;
  }
  rpos[g] = r;
}

// Batch slices (gs_relax.hip run_slices): S copies of the mesh rows, reverse
// positions and stages, copy j's peer ids shifted by j * N. One thread per
// (copy, row, entry).
__global__ __launch_bounds__(TB) void k_srep(uint32_t N, uint32_t S, const uint32_t* __restrict__ mesh,
                                             const uint8_t* __restrict__ rpos, const uint8_t* __restrict__ stage,
                                             uint32_t* __restrict__ smesh, uint8_t* __restrict__ srpos,
                                             uint8_t* __restrict__ sstage) {
  const uint64_t g = (uint64_t)blockIdx.x * TB + threadIdx.x, per = (uint64_t)N * MESH_W;
  if (g >= per * S) return;
  const uint32_t j = (uint32_t)(g / per);
  const uint64_t i = g - (uint64_t)j * per;
  const uint32_t e = mesh[i];
  smesh[g] = e == EMPTY ? EMPTY : e + j * N;  // (stage bits above the id: no carry, S * N < 2^21)
  srpos[g] = rpos[i];
  if (i % MESH_W == 0) sstage[(size_t)j * N + i / MESH_W] = stage[i / MESH_W];
}

// Window grain of the pull path: one unit of the key's high 32-bit word.
inline uint64_t pull_grain(uint32_t tshift) { return tshift >= 32 ? 1ull : 1ull << (32 - tshift); }

void pull_dispatch(uint32_t FP, const PullArgs& a, unsigned grid, hipStream_t s) {
  switch (FP) {
    case 1: k_pull<1><<<grid, TB, 0, s>>>(a); break;
    case 2: k_pull<2><<<grid, TB, 0, s>>>(a); break;
    case 4: k_pull<4><<<grid, TB, 0, s>>>(a); break;
    case 8: k_pull<8><<<grid, TB, 0, s>>>(a); break;
    default: k_pull<16><<<grid, TB, 0, s>>>(a); break;
  }
}
