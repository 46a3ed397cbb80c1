// gs_relax_kernel.h — the hot kernel: one Delta-bucket of eager forwarding.
// Included by gs_relax.hip only (inside namespace gs::{anon}).
//
// A wave owns 64 consecutive lanes ("a tile") of keys[u][m][f]; with 64
// messages per batch and F = 1 a tile is exactly one peer's row, so the
// pushes of a wave into target w hit one 512-B row (coalesced partial writes).
//
// Variants (GS_RELAX_VARIANT bitmask, default 3; both exact):
//   FILTER  read the target key first and issue the 64-bit atomicMin only when
//           the new key is smaller (keys only decrease, so a stale read can only
//           cause an extra atomic, never a missed one)
//   SKIP    per-tile metadata {min pending key, scan stamp, push stamp}: a tile
//           with no push since its last scan and no pending key inside the
//           current bucket is not re-read; its min pending key is folded into
//           the next-bucket reduction from the metadata.

struct TileMeta {
  uint64_t tmin;     // min pending key (>= that launch's bucket end) at last scan
  uint32_t scanned;  // stamp (launch + 1) of the last scan
  uint32_t pushed;   // stamp of the last atomic push into the tile
};

struct RelaxArgs {
  uint64_t* keys;
  uint64_t* busy;
  TileMeta* meta;
  const uint32_t* mesh;
  const uint32_t* pub;
  const uint8_t* stage;
  const uint32_t* tables;  // lat[S*S] | ser_up[S] | ser_dn[S]
  uint64_t* ctrl;
  uint64_t* counters;
  uint64_t total;          // N * L lanes
  uint64_t delta;
  uint64_t tmax;
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

template <int FP, bool FILTER, bool SKIP>
__global__ __launch_bounds__(TB) void k_relax(RelaxArgs a) {
  __shared__ uint32_t s_lat[MAX_STAGES * MAX_STAGES];
  __shared__ uint32_t s_su[MAX_STAGES], s_sd[MAX_STAGES];
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctrl[(a.launch + 2) % 3] = INF64;
  const uint64_t cur = a.ctrl[a.launch % 3];
  if (cur == INF64) return;  // grid-uniform: no pending keys left
  const uint32_t S = a.S;
  for (uint32_t i = threadIdx.x; i < S * S; i += TB) s_lat[i] = a.tables[i];
  if (threadIdx.x < S) {
    s_su[threadIdx.x] = a.tables[S * S + threadIdx.x];
    s_sd[threadIdx.x] = a.tables[S * S + S + threadIdx.x];
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd((unsigned long long*)&a.counters[C_BUCKETS], 1ull);
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint64_t smask = (1ull << a.sb) - 1;
  const uint32_t L = a.L, stamp = a.launch + 1;
  const int lane = threadIdx.x & 63;
  uint64_t nmin = INF64, fd = 0, nr = 0;
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
    const uint32_t u = valid ? (uint32_t)(gid / L) : 0;
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * L);
    const uint32_t m = slot / FP;
    const uint32_t pm = valid ? a.pub[m] : EMPTY;
    const bool pending = key != INF64;
    const bool active = pending && t >= lo && t < hi && u != pm;
    const uint64_t later = (pending && t >= hi) ? key : INF64;
    nmin = later < nmin ? later : nmin;
    const uint32_t src = (uint32_t)(key & smask);
    const uint32_t hp = (uint32_t)((key >> a.sb) & ((1u << HOP_BITS) - 1));
    const uint32_t su = valid ? a.stage[u] : 0;
    const uint32_t ser = s_su[su];
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
          const uint64_t kw = a.keys[(size_t)w * L + slot];
          sk = kw != INF64 && (kw >> a.tshift) + s_lat[(e >> STAGE_SHIFT) * S + su] <= t;
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
    if (active) {
      fd++;
      nr += n;
      if (n && hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
      const uint64_t hbits = ((uint64_t)(hp + 1) << a.sb) | u;
      uint64_t old[MESH_W];
      if constexpr (FILTER) {
#pragma unroll
        for (int j = 0; j < (int)MESH_W; j++)
          old[j] = (skip & (1u << j)) ? 0 : a.keys[(size_t)(row[j] & 0xFFFFFFu) * L + slot];
      }
      uint32_t pos = 0;
#pragma unroll
      for (int j = 0; j < (int)MESH_W; j++) {
        if (skip & (1u << j)) continue;
        const uint32_t e = row[j];
        const uint32_t w = e & 0xFFFFFFu, sw = e >> STAGE_SHIFT;
        pos++;
        const uint32_t sd = s_sd[sw];
        const uint64_t arr = start + (uint64_t)pos * ser + s_lat[su * S + sw] + (sd > ser ? sd - ser : 0);
        if (arr > a.tmax) err |= ERR_TIME;
        const uint64_t nk = (arr << a.tshift) | hbits;
        if (FILTER && !(nk < old[j])) continue;
        const size_t dst = (size_t)w * L + slot;
        atomicMin((unsigned long long*)&a.keys[dst], (unsigned long long)nk);
        if constexpr (SKIP) a.meta[dst >> 6].pushed = stamp;
        nmin = nk < nmin ? nk : nmin;
      }
    }
    if constexpr (SKIP) {
      const uint64_t tm = wave_min(later);
      if (lane == 0) {
        a.meta[tile].tmin = tm;
        a.meta[tile].scanned = stamp;
      }
    }
  }
  nmin = wave_min(nmin);
  fd = wave_sum(fd);
  nr = wave_sum(nr);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if (lane == 0) {
    if (nmin != INF64) atomicMin((unsigned long long*)&a.ctrl[(a.launch + 1) % 3], (unsigned long long)nmin);
    if (fd) atomicAdd((unsigned long long*)&a.counters[C_FD], (unsigned long long)fd);
    if (nr) atomicAdd((unsigned long long*)&a.counters[C_R_FWD], (unsigned long long)nr);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
}

template <int FP>
void relax_fp(uint32_t variant, const RelaxArgs& a, unsigned grid, hipStream_t s) {
  switch (variant & 3) {
    case 0: k_relax<FP, false, false><<<grid, TB, 0, s>>>(a); break;
    case 1: k_relax<FP, true, false><<<grid, TB, 0, s>>>(a); break;
    case 2: k_relax<FP, false, true><<<grid, TB, 0, s>>>(a); break;
    default: k_relax<FP, true, true><<<grid, TB, 0, s>>>(a); break;
  }
}

void relax_dispatch(uint32_t FP, uint32_t variant, const RelaxArgs& a, unsigned grid, hipStream_t s) {
  switch (FP) {
    case 1: relax_fp<1>(variant, a, grid, s); break;
    case 2: relax_fp<2>(variant, a, grid, s); break;
    case 4: relax_fp<4>(variant, a, grid, s); break;
    case 8: relax_fp<8>(variant, a, grid, s); break;
    default: relax_fp<16>(variant, a, grid, s); break;
  }
}
