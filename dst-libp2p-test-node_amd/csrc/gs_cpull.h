// gs_cpull.h — inputs of the churn list pass (k_lpull<FP, CH, false, false,
// GOS, true>; FP fragment lanes per message): config #3 (BASELINE.json: 100k peers,
// heterogeneous links, lazy gossip, churn) on the owner-computes pass.
// Included by gs_relax.hip after gs_lpull_kernel.h (namespace gs::{anon}).
//
// Under churn a forward of a lane first received at t uses
// the sender's mesh of the heartbeat epoch t falls in, and a delivery to a peer
// offline at its arrival is lost. In a lockstep batch (every publish the same
// offset r0 into its epoch; run.sh's schedule, the bench) the relative epoch
// k(t) = floor((r0 + t) / heartbeat) of a time after the publish is the same for
// every message, so lane m at relative time t is in absolute epoch q0[m] + k(t).
// The pass therefore needs, per row, the mesh of every epoch of the batch —
// as a mask over the row's CSR entries, so one 64-bit word per (row, epoch) —
// and, per row and relative epoch, which lanes are offline. A record carries
// the sender's mask of receivers over its CSR row (16 B), and a receiver tests
// its bit at its position in that row (cpos), like the frozen pass's 16-bit
// mesh mask. Built once per batch after the epoch chain:
//  k_cell   (once per topology) CSR rows as 64-wide ELL rows: packed stage | peer
//           and the row's position in each neighbour's row;
//  k_offe   each peer's offline bits over the batch's epochs, from the ring's
//           offline bitsets (a 64 x 64 bit transpose by ballots);
//  k_cprep  per row and epoch: the mesh mask (from the chain's mask ring) and
//           the IHAVE targets (selected among the online connections outside
//           the mesh; none when the row is offline), and per relative epoch k the offline lanes in
//           the final bits' transposed layout (all lanes at k = horizon + 1:
//           past the message's lifetime nothing is delivered).

// CSR -> 64-wide ELL rows, one thread per (row, entry slot).
__global__ __launch_bounds__(TB) void k_cell(uint32_t N, const uint64_t* __restrict__ row,
                                             const uint32_t* __restrict__ col, const uint32_t* __restrict__ rev,
                                             const uint8_t* __restrict__ stage, uint32_t* __restrict__ ccol,
                                             uint8_t* __restrict__ cpos) {
  const uint64_t it = (uint64_t)blockIdx.x * TB + threadIdx.x;
  const uint32_t u = (uint32_t)(it / CELL_W), j = (uint32_t)(it % CELL_W);
  if (u >= N) return;
  const uint64_t b = row[u], deg = row[u + 1] - b;
  uint32_t x = EMPTY;
  uint8_t p = 255;
  if (j < deg) {
    const uint32_t w = col[b + j];
    x = ((uint32_t)stage[w] << STAGE_SHIFT) | w;
    const uint64_t q = rev[b + j] - row[w];
    p = (uint8_t)(q < 255 ? q : 255);
  }
  ccol[it] = x;
  cpos[it] = p;
}

// Offline bits of peers [64 bx, 64 bx + 64) over epochs [E0 + 64 by, +64):
// lane l loads the epoch's bitset word, 64 ballots transpose it. One wave per block.
__global__ __launch_bounds__(64) void k_offe(uint32_t N, const uint64_t* __restrict__ ring_off, uint32_t w64, uint32_t R,
                                             uint64_t E0, uint32_t cE, uint32_t cW, uint64_t* __restrict__ offe) {
  const uint32_t lane = threadIdx.x, cw = blockIdx.y;
  const uint32_t e = cw * 64 + lane;
  const uint64_t word = e < cE ? ring_off[(size_t)((uint32_t)((E0 + e) % R)) * w64 + blockIdx.x] : 0;
  uint64_t mine = 0;
#pragma unroll 8
  for (int p = 0; p < 64; p++) {
    const uint64_t b = __ballot((word >> p) & 1);
    if (lane == p) mine = b;
  }
  const uint32_t x = blockIdx.x * 64 + lane;
  if (x < N) offe[(size_t)x * cW + cw] = mine;
}

struct CPrepArgs {
  const uint32_t* ccol;
  const uint64_t* ring_mm;  // [R][N]
  const uint64_t* offe;     // [N][cW]
  const uint32_t* cq;       // [B]
  uint64_t* cmm;            // [N][cE]
  uint64_t* cgt;            // lazy gossip: IHAVE targets per (row, epoch) (nullptr: no gossip)
  uint32_t* coff;           // [H + 2][N][LP_FW]
  uint64_t E0, seed;
  uint32_t N, R, cE, cW, B, H, d_lazy, gf_milli;
  uint32_t FP;      // fragment lanes per message: lane l is message l / FP's
  uint32_t c0, c1;  // k_cprep: the chunks of 64 epochs [c0, c1) (their epochs are in the ring)
};

// One wave per row w: lane e holds CSR entry e (neighbour x). Per chunk of 64
// epochs, lane j loads the mesh mask of epoch E0 + 64c + j; then for each epoch
// of the chunk the IHAVE-eligible mask is the row's entries outside that mesh
// whose neighbour is online (a ballot of the neighbours' offline bits), and lane
// j selects epoch j's targets. Launched per range of chunks on the side stream
// while the epoch chain fills the ring (gs_relax.hip chn_prepare).
__global__ __launch_bounds__(TB) void k_cprep(CPrepArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t wv = blockIdx.x * (TB / 64) + (threadIdx.x >> 6), nw = gridDim.x * (TB / 64);
  for (uint32_t w = wv; w < a.N; w += nw) {
    const uint32_t xe = a.ccol[(size_t)w * CELL_W + lane];
    const bool valid = xe != EMPTY;
    const uint32_t xc = xe & 0xFFFFFFu;
    const uint64_t cm = __ballot(valid);
    const uint32_t deg = (uint32_t)__popcll(cm);
    const uint64_t pre = rng_pre(a.seed, P_GOSSIP, w);
    const uint64_t* ownp = a.offe + (size_t)w * a.cW;
    for (uint32_t c = a.c0; c < a.c1; c++) {
      const uint32_t e = c * 64 + (uint32_t)lane;
      const uint64_t mml =
          e < a.cE ? a.ring_mm[(size_t)((uint32_t)((a.E0 + e) % a.R)) * a.N + w] & cm : 0;
      const uint64_t offw = valid ? a.offe[(size_t)xc * a.cW + c] : 0;
      const uint64_t own = ownp[c];  // wave-uniform
      uint64_t gel = 0;
      const uint32_t ne = a.cE - c * 64 < 64 ? a.cE - c * 64 : 64;
      for (uint32_t j = 0; j < ne; j++) {
        const uint64_t mmj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(mml >> 32), j) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((uint32_t)mml, j);
        const uint64_t offn = __ballot((offw >> j) & 1);
        const uint64_t ge = ((own >> j) & 1) ? 0 : (cm & ~mmj & ~offn);
        if ((uint32_t)lane == j) gel = ge;
      }
      if (e < a.cE) a.cmm[(size_t)w * a.cE + e] = mml;
      if (a.cgt) {  // lane j: the IHAVE targets of epoch E0 + 64c + j (glp_targets, the oracle's gossip_targets)
        const uint32_t nn = (uint32_t)__popcll(gel);
        uint32_t r = (uint32_t)(((uint64_t)nn * a.gf_milli) / 1000);
        if (r < a.d_lazy) r = a.d_lazy;
        if (r > nn) r = nn;
        const uint64_t tg = glp_targets(pre, (uint32_t)(a.E0 + e), valid ? xc : EMPTY, gel, deg, r);
        if (e < a.cE) a.cgt[(size_t)w * a.cE + e] = tg;
      }
    }
  }
}

// The offline lanes per relative epoch k (lane l of message m = l / FP:
// epoch E0 + cq[m] + k), one wave per row: lane j builds its u16 (bit q = lane
// q*64 + j); the row's own bits are fetched from lane (index >> 6), which
// holds word index >> 6.
__global__ __launch_bounds__(TB) void k_coff(CPrepArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t wv = blockIdx.x * (TB / 64) + (threadIdx.x >> 6), nw = gridDim.x * (TB / 64);
  for (uint32_t w = wv; w < a.N; w += nw) {
    const uint64_t* ownp = a.offe + (size_t)w * a.cW;
    const uint64_t ownl = (uint32_t)lane < a.cW ? ownp[lane] : 0;
    uint32_t cql[PULL_CH];
#pragma unroll
    for (int q = 0; q < (int)PULL_CH; q++) {
      const uint32_t m = ((uint32_t)q * 64 + (uint32_t)lane) / a.FP;
      cql[q] = m < a.B ? a.cq[m] : 0xFFFFFFFFu;
    }
    for (uint32_t k = 0; k <= a.H + 1; k++) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < (int)PULL_CH; q++) {
        const uint32_t idx = cql[q] + k;  // a lane past B reads garbage below, masked by cql
        const int src = (int)((idx >> 6) & 63);
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)ownl, src), hi = (uint32_t)__shfl((int)(uint32_t)(ownl >> 32), src);
        const uint64_t wd = ((uint64_t)hi << 32) | lo;
        const bool off = k > a.H || (cql[q] != 0xFFFFFFFFu && idx < a.cE && ((wd >> (idx & 63)) & 1));
        bits |= off ? 1u << q : 0u;
      }
      reinterpret_cast<uint16_t*>(a.coff + ((size_t)k * a.N + w) * LP_FW)[lane] = (uint16_t)bits;
    }
  }
}
