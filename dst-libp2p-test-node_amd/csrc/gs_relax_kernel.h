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
//   2 SKIP    per-tile {min pending key, scan stamp, push stamp} (fused only)
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

__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t x = __shfl_xor(v, off);
    v = x < v ? x : v;
  }
  return v;
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

// Shared per-bucket constants in LDS.
struct BucketLds {
  uint32_t lat[MAX_STAGES * MAX_STAGES];
  uint32_t su[MAX_STAGES], sd[MAX_STAGES];
};

__device__ __forceinline__ void load_tables(BucketLds& L, const RelaxArgs& a) {
  const uint32_t S = a.S;
  for (uint32_t i = threadIdx.x; i < S * S; i += TB) L.lat[i] = a.tables[i];
  if (threadIdx.x < S) {
    L.su[threadIdx.x] = a.tables[S * S + threadIdx.x];
    L.sd[threadIdx.x] = a.tables[S * S + S + threadIdx.x];
  }
}

// Forward one lane's first arrival (key at lane gid = u*L + slot). `active`
// must be true only for lanes finalised in this bucket; every lane of the wave
// must call this (FP > 1 shuffles across the FP-aligned lane group).
template <int FP, bool FILTER, bool SKIP, bool FB, bool TOUCH = false>
__device__ __forceinline__ void relax_lane(const RelaxArgs& a, const BucketLds& L, bool active,
                                           uint64_t key, uint32_t u, uint32_t slot, uint32_t pm,
                                           uint64_t& nmin, uint64_t& fd, uint64_t& nr, uint64_t& np, uint32_t& err) {
  const uint32_t S = a.S, LL = a.L;
  const int lane = threadIdx.x & 63;
  const uint64_t t = key >> a.tshift;
  const uint64_t smask = (1ull << a.sb) - 1;
  const uint32_t src = (uint32_t)(key & smask);
  const uint32_t hp = (uint32_t)((key >> a.sb) & ((1u << HOP_BITS) - 1));
  const uint32_t su = a.stage[u];
  const uint32_t ser = L.su[su];
  uint32_t row[MESH_W];
  uint32_t skip = 0, n = 0;
  if (active) {
    const uint4* rp = reinterpret_cast<const uint4*>(a.mesh + (size_t)u * MESH_W);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 x = rp[q];
      row[4 * q] = x.x; row[4 * q + 1] = x.y; row[4 * q + 2] = x.z; row[4 * q + 3] = x.w;
    }
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++) {
      const uint32_t e = row[j];
      if (e == EMPTY) { skip |= 1u << j; continue; }  // rows are EMPTY-padded at the tail
      const uint32_t w = e & 0xFFFFFFu;
      bool sk = (w == src) || (w == pm);
      if (!sk && a.idw) {  // IDONTWANT from w already here
        const uint64_t kw = a.keys[(size_t)w * LL + slot];
        sk = kw != INF64 && (kw >> a.tshift) + L.lat[(e >> STAGE_SHIFT) * S + su] <= t;
      }
      if (sk) skip |= 1u << j; else n++;
    }
  }
  uint64_t start = t;
  if constexpr (FP > 1) {
    // Uplink FIFO across this (u, m)'s fragments: the FP lanes of the group
    // fold max(t_f, busy) + n_f * ser in key order (all lanes shuffle).
    const int gb = lane & ~(FP - 1);
    const uint64_t ka = active ? key : INF64;
    const uint32_t m = slot / FP;
    uint64_t kk[FP];
    uint32_t nn[FP];
#pragma unroll
    for (int g = 0; g < FP; g++) { kk[g] = __shfl(ka, gb + g); nn[g] = __shfl(n, gb + g); }
    int first = -1;
#pragma unroll
    for (int g = FP - 1; g >= 0; g--) if (kk[g] != INF64) first = g;
    if (first >= 0) {
      uint64_t cb = a.busy[(size_t)u * a.B + m];
      uint64_t prev = 0;
#pragma unroll
      for (int it = 0; it < FP; it++) {
        uint64_t bk = INF64;
        uint32_t bn = 0;
#pragma unroll
        for (int g = 0; g < FP; g++)
          if (kk[g] > prev && kk[g] < bk) { bk = kk[g]; bn = nn[g]; }
        if (bk == INF64) continue;  // nothing left (kept unrollable: no break)
        const uint64_t tb = bk >> a.tshift;
        const uint64_t s = tb > cb ? tb : cb;
        if (active && bk == key) start = s;
        cb = s + (uint64_t)bn * ser;
        prev = bk;
      }
      if (lane - gb == first) a.busy[(size_t)u * a.B + m] = cb;
    }
  }
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
template <int FP, bool SKIP>
__global__ __launch_bounds__(TB) void k_scan(RelaxArgs a) {
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctrl[(a.launch + 2) % 3] = INF64;
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64) return;  // the frontier kernel exits on the same word
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t LL = a.L;
  const uint64_t ntiles = (a.total + 63) >> 6;
  const uint64_t nwaves = (uint64_t)gridDim.x * (TB / 64);
  const size_t seg = (size_t)wave * a.seg_cap;
  uint64_t nmin = INF64;
  uint32_t cnt = 0;
  for (uint64_t tile = uniform64(wave); tile < ntiles; tile += nwaves) {
    if constexpr (SKIP) {
      // untouched since its last scan and nothing due in this bucket: the
      // tile's keys are unchanged, its min pending key stands for it
      const uint64_t tm = uniform64(a.tmin[tile]);
      const uint32_t tc = __builtin_amdgcn_readfirstlane((uint32_t)a.touched[tile]);
      if (!tc && (tm == INF64 || (tm >> a.tshift) >= hi)) {
        nmin = tm < nmin ? tm : nmin;
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
    const uint64_t fw = __ballot(pending && t < hi);
    if (lane == 0) a.fbits[tile] = fw;
    if constexpr (SKIP) {
      const uint64_t tmn = wave_min(later);
      if (lane == 0) {
        a.tmin[tile] = tmn;
        a.touched[tile] = 0;
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
  if (lane == 0) a.fr_cnt[wave] = cnt;
  nmin = wave_min(nmin);
  if (lane == 0 && nmin != INF64)
    atomicMin((unsigned long long*)&a.ctrl[(a.launch + 1) % 3], (unsigned long long)nmin);
}

// Frontier: every lane carries one compacted arrival (FP lanes per group).
template <int FP, bool FILTER, bool TOUCH>
__global__ __launch_bounds__(TB) void k_frontier(RelaxArgs a) {
  __shared__ BucketLds L;
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64) return;
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
    const uint32_t u = (uint32_t)(gid / LL);
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
    if (variant & 2) k_scan<FP, true><<<grid, TB, 0, s>>>(a);
    else k_scan<FP, false><<<grid, TB, 0, s>>>(a);
    if (mid) (void)hipEventRecord(mid, s);  // splits scan / frontier time when timing
    switch (variant & 3) {
      case 0: k_frontier<FP, false, false><<<grid, TB, 0, s>>>(a); break;
      case 1: k_frontier<FP, true, false><<<grid, TB, 0, s>>>(a); break;
      case 2: k_frontier<FP, false, true><<<grid, TB, 0, s>>>(a); break;
      default: k_frontier<FP, true, true><<<grid, TB, 0, s>>>(a); break;
    }
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
