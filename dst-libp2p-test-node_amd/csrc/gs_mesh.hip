// gs_mesh.hip — GossipSub heartbeat mesh maintenance (GRAFT/PRUNE to
// D / D_lo / D_hi) as synchronous epochs on gfx950.
//
// The reference runs libp2p-gossipsub's heartbeat every 1 s
// (rust-test-node/src/main.rs:228) with mesh_n/low/high 6/4/8, outbound min 3,
// prune back-off 60 s (main.rs:229-236); scoring is inert (main.rs:260-269).
// Each epoch is three row steps over the CSR (a group of lanes per peer):
//   A  heartbeat decisions (graft to D below D_lo, prune to D above D_hi
//      keeping D_out outbound, graft outbound peers when short),
//   B  GRAFT handling at the receiver in (latency, id) order (back-off and
//      D_hi-unless-outbound rejections),
//   C  PRUNEs and rejections applied, both ends back off.
// Random choices use per-(peer, epoch, candidate) keys: take the r smallest.
//
// Churn: each epoch has its offline set (offline_draw), drops
// mesh links of offline peers without back-off, and the heartbeat grafts
// online candidates only. The epochs run event-driven (ev_epochs: a row runs
// a step only when the step can change it). gs_run keeps a ring of per-epoch
// snapshots {mesh ELL, offline bitset, IHAVE targets} (slot = epoch mod R)
// that the relaxation kernels index by the epoch each event falls in.
#include "gs_internal.h"

namespace gs {
namespace {

constexpr int TB = 256;

struct MeshArgs {
  const uint64_t* row;
  const uint32_t* col;
  const uint32_t* rev;
  uint8_t* flags;
  uint8_t* prop;
  uint32_t* until;
  const uint8_t* stage;
  const uint32_t* lat;  // S*S ns
  const uint64_t* off;  // offline bitset of this epoch (churn), nullptr: everyone online
  uint64_t* counters;
  uint64_t seed;
  uint32_t N, S, epoch, bo, d, d_lo, d_hi, d_out;
  uint32_t sub;  // the subscription epoch 0: handshake-ordered grafts; = handshake RTTs (0: a heartbeat)
  // event-driven churn epochs (run_epochs): per-peer state planes, nullptr when
  // every row runs every step
  uint8_t* pst;              // [PS_PLANES][N]
  const uint64_t* off_prev;  // offline bitsets of the previous and the next epoch
  const uint64_t* off_next;  // (nullptr: the last epoch of the run)
  unsigned long long* dbg;   // GS_DEBUG_EV: [3][4] active rows per step (+ for HB: leaving, nbr-off, propd, hungry)
  // churn ring of mesh masks (the churn list pass, gs_lpull_kernel.h): bit e of
  // mm_out[u] = CSR entry e of u is in the epoch's mesh; rows the apply step does
  // not re-extract copy mm_prev (nullptr: no mask ring)
  uint64_t* mm_out;
  const uint64_t* mm_prev;
  // event-driven epochs: iprop[rev[e]] mirrors the PR_GRAFT / PR_PRUNE bit of a
  // proposal prop[e], so the receiver reads its own row contiguously instead of
  // gathering prop[rev[.]]; cleared by the step that consumes it (GRAFT / apply)
  uint8_t* iprop;
};

// Planes of MeshArgs::pst. A row runs the heavy per-row code of an epoch step
// only when one of its flags says the step can change it; the flags are set by
// the rows (or the offline draw) that cause the change.
enum : uint32_t {
  PS_PROPD = 0,   // the row wrote GRAFT/PRUNE proposals this epoch (cleared by its next heartbeat step)
  PS_INBOX = 1,   // a neighbour proposed a GRAFT to the row
  PS_PRUNED = 2,  // a neighbour PRUNEd the row
  PS_NBROFF = 3,  // a mesh neighbour went offline this epoch
  PS_DIRTY = 4,   // the row's mesh flags changed this epoch (recount, re-extract its ELL row)
  PS_MC = 5,      // mesh count after the last epoch
  PS_OC = 6,      // outbound mesh count after the last epoch
  PS_PLANES = 7
};

__device__ __forceinline__ bool is_off(const uint64_t* off, uint32_t u) {
  return off && ((off[u >> 6] >> (u & 63)) & 1);
}

// the calling lane's group bits of a wave ballot
template <int G>
__device__ __forceinline__ uint64_t gballot(bool p) {
  const uint64_t m = __ballot(p);
  if constexpr (G == 64) {
    return m;
  } else {
    const int gbase = (threadIdx.x & 63) & ~(G - 1);
    return (m >> gbase) & ((1ull << G) - 1);
  }
}

// Links to offline peers leave the mesh (a disconnect, not a PRUNE: no back-off).
// One peer per wave, lane per CSR entry.
// Returns (group-uniform) whether a mesh link was dropped.
template <int G>
__device__ __forceinline__ bool row_disconnect(const MeshArgs& a, uint32_t u) {
  const bool ou = is_off(a.off, u);
  const uint64_t b = a.row[u], en = a.row[u + 1];
  bool ch = false;
  for (uint64_t e = b + (threadIdx.x & (G - 1)); e < en; e += G) {
    const uint8_t f = a.flags[e];
    if ((f & F_MESH) && (ou || is_off(a.off, a.col[e]))) {
      a.flags[e] = (uint8_t)(f & ~F_MESH);
      ch = true;
    }
  }
  return gballot<G>(ch) != 0;
}
template <int G>
__global__ __launch_bounds__(TB) void k_disconnect(MeshArgs a) {
  const uint32_t u = (blockIdx.x * TB + threadIdx.x) / G;
  if (u < a.N) row_disconnect<G>(a, u);  // group-uniform
}

// Heartbeat decisions of one peer per wave (lane l holds CSR entries l, l+64,
// l+128, l+192 of the row; MAX_DEG = 256). Every choice is a wave-wide argmin
// of (rng key, entry index), so the graft picks, the prune walk and the
// outbound grafts are exactly the sequential rules of DESIGN.md §2.3: the r
// smallest pairs, and the mesh visited in ascending pair order. (Thread per
// peer left 1.5 waves per SIMD at 100k peers and walked the row serially.)
constexpr int HB_PER_LANE = (int)(MAX_DEG / 64);
static_assert(MAX_DEG % 64 == 0 && HB_PER_LANE <= 4, "k_heartbeat covers MAX_DEG entries with 64 lanes");

// Row kernels run one peer per group of G lanes (G = 64, or 16 when every
// row has at most 4*16 entries: four rows per wave, four times the memory
// requests in flight of the latency-bound one-row-per-wave form). Lane l of a
// group holds entries k*G + l, k < HB_PER_LANE.

// One step of a 16-lane (key, idx) min through a DPP lane permutation inside
// the 16-lane row: an ALU operand modifier, not an LDS-pipe ds_bpermute round
// trip — the selection loops of the heartbeat and of GRAFT handling run one
// group_argmin per choice, back to back.
template <int CTRL>
__device__ __forceinline__ void dpp_min_step(uint64_t& key, uint32_t& idx) {
  const uint32_t kl = (uint32_t)key, kh = (uint32_t)(key >> 32);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)kl, (int)kl, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)kh, (int)kh, CTRL, 0xF, 0xF, false);
  const uint32_t i2 = (uint32_t)__builtin_amdgcn_update_dpp((int)idx, (int)idx, CTRL, 0xF, 0xF, false);
  const uint64_t k2 = ((uint64_t)hi << 32) | lo;
  if (k2 < key || (k2 == key && i2 < idx)) { key = k2; idx = i2; }
}

// group argmin over (key, idx); ~0u if every key is INF64. (key, idx) is a
// total order, so the reduction order does not change the result.
template <int G>
__device__ __forceinline__ uint32_t group_argmin(uint64_t key, uint32_t idx) {
  if constexpr (G == 16) {  // lane ^ 1, lane ^ 2 (quad_perm), then the 8- and 16-lane row mirrors
    dpp_min_step<0xB1>(key, idx);
    dpp_min_step<0x4E>(key, idx);
    dpp_min_step<0x141>(key, idx);
    dpp_min_step<0x140>(key, idx);
    return key == INF64 ? ~0u : idx;
  }
  for (int off = G / 2; off > 0; off >>= 1) {
    const uint64_t k2 = __shfl_xor(key, off);
    const uint32_t i2 = (uint32_t)__shfl_xor((int)idx, off);
    if (k2 < key || (k2 == key && i2 < idx)) { key = k2; idx = i2; }
  }
  return key == INF64 ? ~0u : idx;
}

// This lane's smallest (key, entry) among its entries k*G + lane.
template <int G>
__device__ __forceinline__ void lane_min(const uint64_t (&key)[HB_PER_LANE], int lane, uint64_t& bk, uint32_t& bi) {
  bk = INF64;
  bi = ~0u;
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++)  // ascending k: a tie keeps the lower entry
    if (key[k] < bk) { bk = key[k]; bi = (uint32_t)(k * G + lane); }
}

template <int G>
__device__ __forceinline__ void drop_key(uint64_t (&key)[HB_PER_LANE], uint32_t sel) {
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++)
    if ((uint32_t)k == (sel / G)) key[k] = INF64;
}

// The decisions of row_heartbeat on the row's loaded entries (f, w, elig) and
// its mesh / outbound counts m, o.
template <int G>
__device__ __forceinline__ void row_heartbeat_rest(const MeshArgs& a, uint32_t u, uint64_t b, uint32_t deg,
                                                   const uint32_t (&f)[HB_PER_LANE], const uint32_t (&w)[HB_PER_LANE],
                                                   const bool (&elig)[HB_PER_LANE], uint32_t m, uint32_t o) {
  const int lane = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  (void)gbase;
  auto out_of = [&](uint32_t sel) {  // entry sel is outbound: the holding lane's flag, by ballot
    bool ob = false;
    if ((int)(sel % G) == lane)
#pragma unroll
      for (int k = 0; k < HB_PER_LANE; k++)
        if ((uint32_t)k == (sel / G)) ob = (f[k] & F_OUT) != 0;
    return gballot<G>(ob) != 0;
  };
  uint64_t key[HB_PER_LANE];
  if (a.sub) {  // subscription epoch: the first D_lo connections in subscription-arrival order
    const uint32_t su = a.stage[u];
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++) {
      key[k] = INF64;
      if (k * G < (int)deg && (uint32_t)(k * G + lane) < deg && !(f[k] & F_MESH)) {
        const uint32_t sw = a.stage[w[k]];
        const uint64_t lwu = a.lat[sw * a.S + su];
        key[k] = (uint64_t)a.sub * (a.lat[su * a.S + sw] + lwu) + lwu;
      }
    }
    for (uint32_t q = 0; q < a.d_lo; q++) {
      uint64_t bk;
      uint32_t bi;
      lane_min<G>(key, lane, bk, bi);
      const uint32_t sel = group_argmin<G>(bk, bi);
      if (sel == ~0u) break;
      if ((int)(sel % G) == lane) {
        drop_key<G>(key, sel);
        a.prop[b + sel] = PR_GRAFT;  // (prop is clear at the heartbeat: plain stores, no load in the loop)
      }
    }
    return;
  }
  // event-driven epochs: the receivers of this row's proposals are flagged
  // for GRAFT handling / apply (the lane holding the chosen entry stores)
  auto mark = [&](uint32_t sel, uint32_t plane) {
    if (!a.pst) return;
    uint32_t ws = 0;
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++)
      if ((uint32_t)k == (sel / G)) ws = w[k];
    a.pst[(size_t)plane * a.N + ws] = 1;
  };
  bool proposed = false;
  uint32_t mm = m, oo = o;
  uint32_t graft = 0;  // bit k: entry k*G + lane grafted this epoch
  uint32_t pruned = 0;  // bit k: entry k*G + lane pruned this epoch
  // (prop is clear at the heartbeat — last epoch's proposals were cleared by the
  // caller — so each proposal is one plain store, no load inside the loops)
  if (m < a.d_lo) {  // graft mesh_n - |mesh| random eligible peers
    const uint64_t pre = rng_pre(a.seed, P_GRAFT, u);
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++) {
      key[k] = INF64;
      if (k * G < (int)deg && elig[k]) key[k] = rng_fin(pre, a.epoch, w[k]);
    }
    for (uint32_t q = 0; q < a.d - m; q++) {
      uint64_t bk;
      uint32_t bi;
      lane_min<G>(key, lane, bk, bi);
      const uint32_t sel = group_argmin<G>(bk, bi);
      if (sel == ~0u) break;
      if ((int)(sel % G) == lane) {
        drop_key<G>(key, sel);
        graft |= 1u << (sel / G);
        a.prop[b + sel] = PR_GRAFT;
        mark(sel, PS_INBOX);
      }
      proposed = true;
      mm++;
      oo += out_of(sel) ? 1u : 0u;
    }
  }
  if (mm > a.d_hi) {  // prune down to mesh_n, keep mesh_outbound_min outbound
    // walk the (start-of-epoch) mesh in ascending (key, entry) order
    const uint32_t excess = mm - a.d;
    uint32_t removed = 0;
    const uint64_t pre = rng_pre(a.seed, P_PRUNE, u);
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++) {
      key[k] = INF64;
      if (k * G < (int)deg && (f[k] & F_MESH)) key[k] = rng_fin(pre, a.epoch, w[k]);
    }
    for (uint32_t q = 0; q < m && removed < excess; q++) {
      uint64_t bk;
      uint32_t bi;
      lane_min<G>(key, lane, bk, bi);
      const uint32_t sel = group_argmin<G>(bk, bi);
      if (sel == ~0u) break;
      if ((int)(sel % G) == lane) drop_key<G>(key, sel);
      if (out_of(sel)) {
        if (oo <= a.d_out) continue;
        oo--;
      }
      if ((int)(sel % G) == lane) {
        pruned |= 1u << (sel / G);
        a.prop[b + sel] = PR_PRUNE;
        mark(sel, PS_PRUNED);
      }
      proposed = true;
      removed++;
      mm--;
    }
  }
  if (mm >= a.d_lo && oo < a.d_out) {  // graft outbound peers
    const uint64_t pre = rng_pre(a.seed, P_OUT_GRAFT, u);
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++)
    {
      key[k] = INF64;
      if (k * G < (int)deg && elig[k] && (f[k] & F_OUT) && !((graft >> k) & 1u))
        key[k] = rng_fin(pre, a.epoch, w[k]);
    }
    for (uint32_t q = 0; q < a.d_out - oo; q++) {
      uint64_t bk;
      uint32_t bi;
      lane_min<G>(key, lane, bk, bi);
      const uint32_t sel = group_argmin<G>(bk, bi);
      if (sel == ~0u) break;
      if ((int)(sel % G) == lane) {
        drop_key<G>(key, sel);
        graft |= 1u << (sel / G);
        a.prop[b + sel] = PR_GRAFT;
        mark(sel, PS_INBOX);
      }
      proposed = true;
    }
  }
  if (a.iprop && (graft | pruned)) {  // mirror the proposals at the receivers' entries (reverse ids loaded together)
    uint32_t rv[HB_PER_LANE];
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++)
      if (((graft | pruned) >> k) & 1u) rv[k] = a.rev[b + k * G + lane];
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++)
      if (((graft | pruned) >> k) & 1u) a.iprop[rv[k]] = ((graft >> k) & 1u) ? PR_GRAFT : PR_PRUNE;
  }
  if (a.pst && proposed && lane == 0) {
    a.pst[(size_t)PS_PROPD * a.N + u] = 1;
    a.pst[(size_t)PS_DIRTY * a.N + u] = 1;
  }
}


template <int G>
__device__ __forceinline__ void row_heartbeat(const MeshArgs& a, uint32_t u) {
  const int lane = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  (void)gbase;
  if (is_off(a.off, u)) return;  // wave-uniform
  const uint64_t b = a.row[u], en = a.row[u + 1];
  const uint32_t deg = (uint32_t)(en - b);
  uint32_t f[HB_PER_LANE], w[HB_PER_LANE];
  bool elig[HB_PER_LANE];  // not in mesh, back-off over, neighbour online
  uint32_t m = 0, o = 0;
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    f[k] = 0;
    w[k] = 0;
    elig[k] = false;
    if (k * G >= (int)deg) continue;  // wave-uniform
    if (i < deg) {
      f[k] = a.flags[b + i];
      w[k] = a.col[b + i];
      elig[k] = !(f[k] & F_MESH) && a.epoch > a.until[b + i] && !is_off(a.off, w[k]);
    }
    m += (uint32_t)__popcll(gballot<G>(f[k] & F_MESH));
    o += (uint32_t)__popcll(gballot<G>((f[k] & F_MESH) && (f[k] & F_OUT)));
  }
  row_heartbeat_rest<G>(a, u, b, deg, f, w, elig, m, o);
}

// Heartbeat step of an event-driven epoch for one row (row base b, degree deg
// from the block's activity scan), every load issued once: last epoch's
// proposals cleared (propd), links to offline peers dropped (the disconnect),
// then the heartbeat decisions on the same registers — the results of the
// prop clear + row_disconnect + row_heartbeat sequence. Returns (group-uniform)
// whether the disconnect dropped a mesh link.
template <int G>
__device__ __forceinline__ bool row_hb_ev(const MeshArgs& a, uint32_t u, uint64_t b, uint32_t deg, bool propd,
                                          bool ou) {
  const int lane = threadIdx.x & (G - 1);
  uint32_t f[HB_PER_LANE], w[HB_PER_LANE], un[HB_PER_LANE];
  bool elig[HB_PER_LANE];
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    const bool v = i < deg;
    f[k] = v ? a.flags[b + i] : 0u;
    w[k] = v ? a.col[b + i] : 0u;
    un[k] = v ? a.until[b + i] : 0u;
  }
  if (propd)  // last epoch's proposals (read by the neighbours until its apply step)
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++)
      if ((uint32_t)(k * G + lane) < deg) a.prop[b + k * G + lane] = 0;
  bool ch = false;
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    const bool offw = i < deg && is_off(a.off, w[k]);
    if (i < deg && (f[k] & F_MESH) && (ou || offw)) {  // disconnect: no back-off
      f[k] &= ~(uint32_t)F_MESH;
      a.flags[b + i] = (uint8_t)f[k];
      ch = true;
    }
    elig[k] = i < deg && !(f[k] & F_MESH) && a.epoch > un[k] && !offw;
  }
  const bool dirty = gballot<G>(ch) != 0;
  if (ou) return dirty;  // offline: the heartbeat decides nothing
  uint32_t m = 0, o = 0;
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    m += (uint32_t)__popcll(gballot<G>(f[k] & F_MESH));
    o += (uint32_t)__popcll(gballot<G>((f[k] & F_MESH) && (f[k] & F_OUT)));
  }
  row_heartbeat_rest<G>(a, u, b, deg, f, w, elig, m, o);
  return dirty;
}

template <int G>
__global__ __launch_bounds__(TB) void k_heartbeat(MeshArgs a) {
  const uint32_t u = (blockIdx.x * TB + threadIdx.x) / G;
  if (u < a.N) row_heartbeat<G>(a, u);  // group-uniform
}

// GRAFT handling at receiver w, one peer per wave: the proposals of w's
// neighbours are found in parallel (lane per entry), then taken in arrival
// order — (latency u->w, id), by wave argmin — with the running mesh size c.
// Returns (group-uniform) whether a GRAFT was accepted (w's mesh changed).
template <int G>
__device__ __forceinline__ bool row_handle_graft(const MeshArgs& a, uint32_t w, uint64_t b, uint32_t deg) {
  const int lane = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  (void)gbase;
  const uint32_t sw = a.stage[w];
  uint32_t f[HB_PER_LANE], p[HB_PER_LANE], r[HB_PER_LANE], un[HB_PER_LANE], cl[HB_PER_LANE], ip[HB_PER_LANE];
  uint64_t lvl[HB_PER_LANE];  // latency u->w of a proposing neighbour u, else INF64
  uint32_t c = 0;
  // the row's entries first (ids too), then the neighbours' proposals and stages
  // together: two dependent round trips instead of three (rev -> prop -> col -> stage)
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    f[k] = 0;
    p[k] = 0;
    r[k] = 0;
    un[k] = 0;
    cl[k] = 0;
    ip[k] = 0;
    if (i < deg) {
      f[k] = a.flags[b + i];
      p[k] = a.prop[b + i];
      r[k] = a.rev[b + i];
      un[k] = a.until[b + i];  // loaded with the row: the GRAFT loop below is serial
      cl[k] = a.col[b + i];
      if (a.iprop) ip[k] = a.iprop[b + i];
    }
  }
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    lvl[k] = INF64;
    if (i < deg) {
      // event-driven epochs: the mirrored bit (row-contiguous), the proposer's stage only when it proposed
      const bool g = a.iprop ? (ip[k] & PR_GRAFT) != 0 : (a.prop[r[k]] & PR_GRAFT) != 0;
      if (g) {  // arrival order: latency u->w (heartbeat), handshake (subscription)
        const uint32_t su = a.stage[cl[k]];
        lvl[k] = a.sub ? (uint64_t)(a.sub + 1) * (a.lat[su * a.S + sw] + a.lat[sw * a.S + su])
                       : a.lat[su * a.S + sw];
        if (a.iprop) a.iprop[b + i] = (uint8_t)(ip[k] & ~PR_GRAFT);  // consumed
      }
    }
    c += (uint32_t)__popcll(gballot<G>(((f[k] & F_MESH) && !(p[k] & PR_PRUNE)) || (p[k] & PR_GRAFT)));
  }
  bool acc = false;
  for (;;) {
    uint64_t bk;
    uint32_t bi;
    lane_min<G>(lvl, lane, bk, bi);
    const uint32_t sel = group_argmin<G>(bk, bi);  // entry (w -> u) of the next GRAFT to arrive
    if (sel == ~0u) break;
    // the lane holding entry sel decides from its own registers; the group
    // learns the outcome by a ballot (no cross-lane shuffle in this serial loop)
    bool took = false;
    if ((int)(sel % G) == lane) {
      uint32_t fs = 0, ps = 0, us = 0, rs = 0;
#pragma unroll
      for (int k = 0; k < HB_PER_LANE; k++)
        if ((uint32_t)k == (sel / G)) { fs = f[k]; ps = p[k]; us = un[k]; rs = r[k]; }
      const bool in_mesh = ((fs & F_MESH) && !(ps & PR_PRUNE)) || (ps & PR_GRAFT);
      const bool rej = !in_mesh && (a.epoch < us || (c >= a.d_hi && !(fs & F_OUT)));
      const uint64_t e = b + sel;
      drop_key<G>(lvl, sel);
      if (rej) a.until[e] = a.epoch + a.bo;  // PRUNE back, both ends back off
      else a.prop[rs] = PR_GRAFT | PR_ACCEPT;  // (the entry holds exactly the GRAFT: a store, no load)
      if (!in_mesh && !rej) a.flags[e] = (uint8_t)(fs | F_MESH);
      took = !in_mesh && !rej;
    }
    if (gballot<G>(took) != 0) {
      c++;
      acc = true;
    }
  }
  return acc;
}
template <int G>
__global__ __launch_bounds__(TB) void k_handle_graft(MeshArgs a) {
  const uint32_t w = (blockIdx.x * TB + threadIdx.x) / G;
  if (w < a.N) row_handle_graft<G>(a, w, a.row[w], (uint32_t)(a.row[w + 1] - a.row[w]));  // group-uniform
}

// Apply the epoch's decisions, one peer per wave (lane per entry). The change
// flag only has to be non-zero when anything changed (run_mesh's fixed-point
// test), so every wave with a change stores 1: no atomics.
template <int G>
__device__ __forceinline__ bool row_apply(const MeshArgs& a, uint32_t u) {
  const int lane = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  (void)gbase;
  const uint64_t b = a.row[u];
  const uint32_t deg = (uint32_t)(a.row[u + 1] - b);
  bool changed = false;
  for (uint32_t i = (uint32_t)lane; i < deg; i += G) {
    const uint64_t e = b + i;
    const uint8_t p = a.prop[e];
    uint8_t f = a.flags[e];
    if (p & PR_GRAFT) {
      changed = true;
      if (p & PR_ACCEPT) f |= F_MESH;
      else { f &= (uint8_t)~F_MESH; a.until[e] = a.epoch + a.bo; }
    }
    if (p & PR_PRUNE) { changed = true; f &= (uint8_t)~F_MESH; a.until[e] = a.epoch + a.bo; }
    if (a.prop[a.rev[e]] & PR_PRUNE) { f &= (uint8_t)~F_MESH; a.until[e] = a.epoch + a.bo; }
    a.flags[e] = f;
  }
  return gballot<G>(changed) != 0;
}
template <int G>
__global__ __launch_bounds__(TB) void k_apply(MeshArgs a) {
  const uint32_t u = (blockIdx.x * TB + threadIdx.x) / G;
  if (u >= a.N) return;  // group-uniform
  if (row_apply<G>(a, u) && (threadIdx.x & (G - 1)) == 0) a.counters[C_MESH_CHANGES] = 1;
}

// Quiescent epoch: earliest back-off expiry that can wake a hungry peer.
__global__ __launch_bounds__(TB) void k_wake(MeshArgs a) {
  const uint32_t u = blockIdx.x * TB + threadIdx.x;
  uint64_t wake = INF64;
  if (u < a.N) {
    const uint64_t b = a.row[u], en = a.row[u + 1];
    uint32_t m = 0, o = 0;
    for (uint64_t e = b; e < en; e++)
      if (a.flags[e] & F_MESH) { m++; o += a.flags[e] & F_OUT; }
    const bool need_any = m < a.d_lo;
    const bool need_out = !need_any && m <= a.d_hi && o < a.d_out;
    if (need_any || need_out)
      for (uint64_t e = b; e < en; e++) {
        const uint8_t f = a.flags[e];
        if ((f & F_MESH) || (need_out && !(f & F_OUT))) continue;
        if (a.until[e] >= a.epoch + 1 && (uint64_t)a.until[e] + 1 < wake) wake = (uint64_t)a.until[e] + 1;
      }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t x = __shfl_xor(wake, off);
    wake = x < wake ? x : wake;
  }
  if ((threadIdx.x & 63) == 0 && wake != INF64)
    atomicMin((unsigned long long*)&a.counters[C_MESH_WAKE], (unsigned long long)wake);
}

__global__ __launch_bounds__(TB) void k_clear_mesh(uint64_t nnz, uint8_t* flags, uint32_t* until) {
  const uint64_t e = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (e >= nnz) return;
  flags[e] &= (uint8_t)~F_MESH;
  until[e] = 0;
}

// ELL extraction: packed stage<<24 | peer in ascending id, EMPTY padded.
__global__ __launch_bounds__(TB) void k_extract(MeshArgs a, uint32_t* mesh, uint8_t* mcnt) {
  const uint32_t u = blockIdx.x * TB + threadIdx.x;
  if (u >= a.N) return;
  uint32_t c = 0;
  if (a.mm_out) {  // the mask ring's slot (rows of <= 64 entries)
    uint64_t mm = 0;
    for (uint64_t e = a.row[u]; e < a.row[u + 1] && e - a.row[u] < 64; e++)
      if (a.flags[e] & F_MESH) mm |= 1ull << (e - a.row[u]);
    a.mm_out[u] = mm;
  }
  for (uint64_t e = a.row[u]; e < a.row[u + 1]; e++)
    if (a.flags[e] & F_MESH) {
      if (c == MESH_W) { atomicOr((unsigned*)&a.counters[C_ERR], ERR_MESH); break; }
      const uint32_t w = a.col[e];
      mesh[(size_t)u * MESH_W + c++] = ((uint32_t)a.stage[w] << STAGE_SHIFT) | w;
    }
  if (mcnt) mcnt[u] = (uint8_t)c;
  for (uint32_t q = c; q < MESH_W; q++) mesh[(size_t)u * MESH_W + q] = EMPTY;
}

// Lazy gossip under churn: who sends IHAVEs to whom at epoch h. Peer u's
// targets are the r smallest (rng(GOSSIP, u, h, w), w) among its online
// connections outside its epoch-h mesh, r = max(D_lazy, factor·|non-mesh|)
// capped at |non-mesh|. The receiver side of lazy gossip
// (k_gossip, receiver-centric under churn) reads them inverted, per target:
// in[w] lists the senders v whose epoch-h IHAVEs reach w (packed stage << 24
// | v, at most GT_IN, EMPTY after the last; GT_REDO in entry 0 tells k_gossip
// to recompute). Built in two passes per chunk of epochs, without atomics:
//  1. k_gossip_out_range: one thread per (sender, epoch) makes the selection
//     (one rng per connection, an 8-deep sorted insert in registers with
//     static indices; the rare fan-outs above 8 rescan for the next pair) and
//     stores it as a bit mask over the sender's CSR row, coalesced;
//  2. k_gossip_in_gather: one thread per (receiver, epoch) walks its CSR row
//     and tests its own bit in each neighbour's mask (the position of w in
//     v's row, csrpos); the masks of one epoch (8 B per peer) stay in L2/MALL.
// Rows wider than 63 entries have no mask (GT_WIDE): their receivers get a
// count above GT_IN, and k_gossip selects for them itself.
constexpr uint64_t GT_WIDE = ~0ull;
__global__ __launch_bounds__(TB) void k_gossip_out_range(const uint64_t* __restrict__ row,
                                                         const uint32_t* __restrict__ col,
                                                         const uint32_t* __restrict__ ring_mesh,
                                                         const uint64_t* __restrict__ ring_off, uint32_t N, uint32_t w64,
                                                         uint32_t R, uint64_t seed, uint64_t h0, uint32_t d_lazy,
                                                         uint32_t gf_milli, uint64_t* __restrict__ outm,
                                                         uint32_t ny) {
  // grid-stride over (sender, epoch): the side stream may run on a capped grid
  for (uint64_t it = (uint64_t)blockIdx.x * TB + threadIdx.x; it < (uint64_t)N * ny; it += (uint64_t)gridDim.x * TB) {
  const uint32_t u = (uint32_t)(it % N), y = (uint32_t)(it / N);
  const uint64_t h = h0 + y;
  const size_t slot = (size_t)(h % R);
  const uint64_t* off = ring_off + slot * w64;
  const uint64_t e0 = row[u], e1 = row[u + 1];
  uint64_t mask = 0;
  if (e1 - e0 > 63) {
    mask = GT_WIDE;
  } else if (!is_off(off, u)) {  // offline peers gossip nothing
    uint32_t mrow[MESH_W];
    const uint4* rp = reinterpret_cast<const uint4*>(ring_mesh + (slot * N + u) * MESH_W);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 x = rp[q];
      mrow[4 * q] = x.x & 0xFFFFFFu; mrow[4 * q + 1] = x.y & 0xFFFFFFu;
      mrow[4 * q + 2] = x.z & 0xFFFFFFu; mrow[4 * q + 3] = x.w & 0xFFFFFFu;
    }
    auto eligible = [&](uint32_t w) {
      bool inm = false;
#pragma unroll
      for (int q = 0; q < (int)MESH_W; q++) inm |= mrow[q] == w;
      return !inm && !is_off(off, w);
    };
    auto lt = [](uint64_t k1, uint32_t w1, uint64_t k2, uint32_t w2) { return k1 < k2 || (k1 == k2 && w1 < w2); };
    uint64_t kk[GT_W];
    uint32_t ww[GT_W], pp[GT_W];
#pragma unroll
    for (int q = 0; q < (int)GT_W; q++) { kk[q] = INF64; ww[q] = ~0u; pp[q] = 0; }
    uint32_t nonmesh = 0;
    const uint64_t pre = rng_pre(seed, P_GOSSIP, u);
    for (uint64_t e = e0; e < e1; e++) {
      const uint32_t w = col[e];
      if (!eligible(w)) continue;
      nonmesh++;
      const uint64_t rk = rng_fin(pre, (uint32_t)h, w);
      const uint32_t pe = (uint32_t)(e - e0);
      if (!lt(rk, w, kk[GT_W - 1], ww[GT_W - 1])) continue;
#pragma unroll
      for (int q = (int)GT_W - 1; q > 0; q--) {  // insert, shifting the larger pairs up
        if (lt(rk, w, kk[q - 1], ww[q - 1])) { kk[q] = kk[q - 1]; ww[q] = ww[q - 1]; pp[q] = pp[q - 1]; }
        else if (lt(rk, w, kk[q], ww[q])) { kk[q] = rk; ww[q] = w; pp[q] = pe; }
      }
      if (lt(rk, w, kk[0], ww[0])) { kk[0] = rk; ww[0] = w; pp[0] = pe; }
    }
    uint32_t r = (uint32_t)(((uint64_t)nonmesh * gf_milli) / 1000);
    if (r < d_lazy) r = d_lazy;
    if (r > nonmesh) r = nonmesh;
#pragma unroll
    for (int q = 0; q < (int)GT_W; q++)
      if ((uint32_t)q < r) mask |= 1ull << pp[q];
    uint64_t pk = kk[GT_W - 1];
    uint32_t pw = ww[GT_W - 1];
    for (uint32_t q = GT_W; q < r; q++) {  // rare: more than GT_W targets
      uint64_t bk = ~0ull;
      uint32_t bw = ~0u, bp = 0;
      for (uint64_t e = e0; e < e1; e++) {
        const uint32_t w = col[e];
        if (!eligible(w)) continue;
        const uint64_t rk = rng_fin(pre, (uint32_t)h, w);
        if (lt(pk, pw, rk, w) && lt(rk, w, bk, bw)) { bk = rk; bw = w; bp = (uint32_t)(e - e0); }
      }
      mask |= 1ull << bp;
      pk = bk;
      pw = bw;
    }
  }
  outm[(size_t)y * N + u] = mask;
  }
}

// 16 lanes per (receiver, epoch): the group loads 16 neighbours' masks at
// once (independent loads), ballots the hits and appends them in CSR order.
constexpr uint32_t GIN_G = 16;
static_assert(GIN_G == GT_IN, "k_gossip_in_gather: one lane per list entry");
__global__ __launch_bounds__(TB) void k_gossip_in_gather(const uint64_t* __restrict__ row,
                                                         const uint32_t* __restrict__ col,
                                                         const uint8_t* __restrict__ csrpos,
                                                         const uint64_t* __restrict__ ring_off,
                                                         const uint8_t* __restrict__ stage, uint32_t N, uint32_t w64,
                                                         uint32_t R, uint64_t h0, const uint64_t* __restrict__ outm,
                                                         uint32_t* __restrict__ ring_in,
                                                         uint32_t ny) {
  const uint32_t lane = threadIdx.x & (GIN_G - 1);
  // grid-stride over (receiver, epoch) groups (group-uniform)
  for (uint64_t it = ((uint64_t)blockIdx.x * TB + threadIdx.x) / GIN_G; it < (uint64_t)N * ny;
       it += (uint64_t)gridDim.x * (TB / GIN_G)) {
  const uint32_t w = (uint32_t)(it % N), y = (uint32_t)(it / N);
  const uint64_t h = h0 + y;
  const size_t slot = (size_t)(h % R);
  const uint64_t* m = outm + (size_t)y * N;
  uint32_t* lst = ring_in + (slot * N + w) * GT_IN;
  uint32_t cnt = 0;
  bool wide = false;
  if (!is_off(ring_off + slot * w64, w)) {  // an offline peer is nobody's target (group-uniform)
    const uint64_t b = row[w], en = row[w + 1];
    for (uint64_t e0 = b; e0 < en; e0 += GIN_G) {  // group-uniform
      const uint64_t e = e0 + lane;
      bool hit = false, wd = false;
      uint32_t v = 0;
      if (e < en) {
        v = col[e];
        const uint64_t mv = m[v];
        const uint32_t p = csrpos[e];
        wd = mv == GT_WIDE || p > 63;
        hit = !wd && ((mv >> p) & 1);
      }
      wide |= gballot<GIN_G>(wd) != 0;
      const uint64_t hm = gballot<GIN_G>(hit);
      const uint32_t pos = cnt + (uint32_t)__popcll(hm & ((1ull << lane) - 1));
      if (hit && pos < GT_IN) lst[pos] = ((uint32_t)stage[v] << STAGE_SHIFT) | v;
      cnt += (uint32_t)__popcll(hm);
    }
  }
  // EMPTY after the senders; GT_REDO in entry 0 when k_gossip must select itself
  if (lane >= cnt && lane < GT_IN) lst[lane] = EMPTY;
  if (lane == 0 && (wide || cnt > GT_IN)) lst[0] = GT_REDO;
  }
}

// Position of u in the row of w = col[e], per CSR entry e (255 past 254).
__global__ __launch_bounds__(TB) void k_csrpos(uint32_t N, const uint64_t* __restrict__ row,
                                               const uint32_t* __restrict__ col, const uint32_t* __restrict__ rev,
                                               uint8_t* __restrict__ pos) {
  const uint32_t u = blockIdx.x * TB + threadIdx.x;
  if (u >= N) return;
  for (uint64_t e = row[u]; e < row[u + 1]; e++) {
    const uint64_t p = rev[e] - row[col[e]];
    pos[e] = (uint8_t)(p < 255 ? p : 255);
  }
}

// ---- event-driven churn epochs (the default run_epochs path) ----
// Under churn most rows do nothing in a given epoch (1 % departures per epoch:
// ~18 % of the rows change, most of them by one dropped link). Each step of an
// epoch therefore tests a few per-peer flags (MeshArgs::pst) and runs the
// row code only where the step can change the row; every rule is the one of
// the per-row kernels above, so the result is the same mesh:
//  heartbeat step: rows going offline, rows with a mesh neighbour going
//    offline (flagged by that neighbour), rows outside [D_lo, D_hi] or below
//    D_out (the only ones a heartbeat can change), rows whose last proposals
//    must be cleared;
//  GRAFT handling: rows a neighbour proposed to;
//  apply: proposers and PRUNEd rows; rows whose mesh changed are recounted
//    and re-extracted into the ring slot, the others copy their previous row.
// Offline bitsets and IHAVE targets do not depend on the epoch sequence and
// run batched over the whole range (k_offline_range; the IHAVE lists per
// chunk of epochs on the side stream, ring_in_lists).

// ELL row of u from its CSR flags (packed stage<<24 | peer, ascending ids).
template <int G>
__device__ __forceinline__ void row_extract(const MeshArgs& a, uint32_t u, uint32_t* mesh) {
  const int lane = threadIdx.x & (G - 1);
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  (void)gbase;
  const uint64_t b = a.row[u];
  const uint32_t deg = (uint32_t)(a.row[u + 1] - b);
  uint32_t cnt = 0;
  for (uint32_t i0 = 0; i0 < deg; i0 += G) {
    const uint32_t i = i0 + (uint32_t)lane;
    const bool in = i < deg && (a.flags[b + i] & F_MESH);
    const uint64_t m = gballot<G>(in);
    const uint32_t pos = cnt + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (in && pos < MESH_W) {
      const uint32_t w = a.col[b + i];
      mesh[(size_t)u * MESH_W + pos] = ((uint32_t)a.stage[w] << STAGE_SHIFT) | w;
    }
    cnt += (uint32_t)__popcll(m);
  }
  if (cnt > MESH_W && lane == 0) atomicOr((unsigned*)&a.counters[C_ERR], ERR_MESH);
  if ((uint32_t)lane >= cnt && lane < (int)MESH_W) mesh[(size_t)u * MESH_W + lane] = EMPTY;
}

// Mesh links of u (all, outbound) from its CSR flags.
template <int G>
__device__ __forceinline__ void row_counts(const MeshArgs& a, uint32_t u, uint32_t& m, uint32_t& o) {
  const uint64_t b = a.row[u], en = a.row[u + 1];
  m = 0;
  o = 0;
  for (uint64_t e0 = b; e0 < en; e0 += G) {  // group-uniform
    const uint64_t e = e0 + (threadIdx.x & (G - 1));
    const uint8_t f = e < en ? a.flags[e] : 0;
    m += (uint32_t)__popcll(gballot<G>(f & F_MESH));
    o += (uint32_t)__popcll(gballot<G>((f & F_MESH) && (f & F_OUT)));
  }
}

// u goes offline at the next epoch: flag its mesh neighbours (their links to
// u leave the mesh there).
template <int G>
__device__ __forceinline__ void mark_departure(const MeshArgs& a, uint32_t u) {
  const uint64_t b = a.row[u], en = a.row[u + 1];
  for (uint64_t e = b + (threadIdx.x & (G - 1)); e < en; e += G)
    if (a.flags[e] & F_MESH) a.pst[(size_t)PS_NBROFF * a.N + a.col[e]] = 1;
}

// Offline bitsets of epochs h0 + y, y < gridDim.y, into lin[y] (w64 words
// each) and, for epochs >= ring_h0 and a ring, into ring slot h % R.
__global__ __launch_bounds__(TB) void k_offline_range(uint32_t N, uint64_t seed, uint32_t ppm, uint32_t down,
                                                      uint64_t h0, uint64_t* lin, uint32_t w64, uint64_t* ring,
                                                      uint32_t R, uint64_t ring_h0) {
  const uint32_t u = blockIdx.x * TB + threadIdx.x;
  const uint64_t h = h0 + blockIdx.y;
  const uint64_t m = __ballot(u < N && offline_draw(seed, ppm, down, u, h));
  if ((threadIdx.x & 63) == 0 && u < N) {
    lin[(size_t)blockIdx.y * w64 + (u >> 6)] = m;
    if (ring && h >= ring_h0) ring[(size_t)(h % R) * w64 + (u >> 6)] = m;
  }
}

// Start of a run of epochs: mesh counts, and the departures of its first
// epoch. Grid-stride, one row per group of G lanes (group-uniform loop).
template <int G>
__global__ __launch_bounds__(TB) void k_ev_init(MeshArgs a) {
  const int lane = threadIdx.x & (G - 1);
  for (uint32_t u = (blockIdx.x * TB + threadIdx.x) / G; u < a.N; u += gridDim.x * (TB / G)) {
    uint32_t m, o;
    row_counts<G>(a, u, m, o);
    if (lane == 0) {
      a.pst[(size_t)PS_MC * a.N + u] = (uint8_t)(m < 255 ? m : 255);
      a.pst[(size_t)PS_OC * a.N + u] = (uint8_t)(o < 255 ? o : 255);
    }
    if (is_off(a.off, u) && !is_off(a.off_prev, u)) mark_departure<G>(a, u);
  }
}

// The apply step of an event-driven epoch for one row, in one pass over it:
// row_apply (when the row proposed or was pruned), then, when its mesh may
// have changed, the recount, the ELL re-extraction and (departing next epoch)
// the neighbour flags — every load of the row issued together (flags, props,
// reverse entries, ids, then the neighbours' props and stages), the new flags
// kept in registers instead of re-read. Same results as row_apply +
// row_counts + row_extract + mark_departure.
template <int G>
__device__ __forceinline__ void row_apply_ev(const MeshArgs& a, uint32_t u, uint64_t b, uint32_t deg, bool need,
                                             bool dirty, bool depart, uint32_t* mesh) {
  uint64_t mmask = 0;  // the new mesh as a mask over the CSR row (entries < 64)
  const int lane = threadIdx.x & (G - 1);
  uint8_t* P = a.pst;
  const uint32_t N = a.N;
  uint32_t f[HB_PER_LANE], pp[HB_PER_LANE], cw[HB_PER_LANE], pr[HB_PER_LANE], sg[HB_PER_LANE];
  // (a neighbour's PRUNE arrives as the mirrored bit a.iprop, on the row itself)
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    const bool v = i < deg;
    f[k] = v ? a.flags[b + i] : 0u;
    pp[k] = v && need ? a.prop[b + i] : 0u;
    pr[k] = v && need ? a.iprop[b + i] : 0u;
    cw[k] = v && (dirty || depart) ? a.col[b + i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < HB_PER_LANE; k++) {
    const uint32_t i = (uint32_t)(k * G + lane);
    const bool v = i < deg;
    sg[k] = v && dirty && mesh ? a.stage[cw[k]] : 0u;
  }
  if (need) {  // row_apply
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++) {
      const uint32_t i = (uint32_t)(k * G + lane);
      if (i >= deg) continue;
      const uint64_t e = b + i;
      const uint32_t p = pp[k];
      uint32_t fk = f[k];
      bool bo = false;
      if (p & PR_GRAFT) {
        if (p & PR_ACCEPT) fk |= F_MESH;
        else { fk &= ~(uint32_t)F_MESH; bo = true; }
      }
      if (p & PR_PRUNE) { fk &= ~(uint32_t)F_MESH; bo = true; }
      if (pr[k] & PR_PRUNE) {
        fk &= ~(uint32_t)F_MESH;
        bo = true;
        a.iprop[e] = 0;  // consumed
      }
      if (bo) a.until[e] = a.epoch + a.bo;
      a.flags[e] = (uint8_t)fk;
      f[k] = fk;
    }
  }
  if (dirty) {  // row_counts + row_extract on the new flags
    uint32_t m = 0, o = 0;
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++) {
      const bool in = (f[k] & F_MESH) != 0;
      const uint64_t bm = gballot<G>(in);
      if (mesh && in) {
        const uint32_t pos = m + (uint32_t)__popcll(bm & ((1ull << lane) - 1));
        if (pos < MESH_W) mesh[(size_t)u * MESH_W + pos] = (sg[k] << STAGE_SHIFT) | cw[k];
      }
      if (k * G < 64) mmask |= bm << (k * G);
      m += (uint32_t)__popcll(bm);
      o += (uint32_t)__popcll(gballot<G>(in && (f[k] & F_OUT)));
    }
    if (a.mm_out && lane == 0) a.mm_out[u] = mmask;
    if (mesh) {
      if (m > MESH_W && lane == 0) atomicOr((unsigned*)&a.counters[C_ERR], ERR_MESH);
      if ((uint32_t)lane >= m && lane < (int)MESH_W) mesh[(size_t)u * MESH_W + lane] = EMPTY;
    }
    if (lane == 0) {
      P[(size_t)PS_MC * N + u] = (uint8_t)(m < 255 ? m : 255);
      P[(size_t)PS_OC * N + u] = (uint8_t)(o < 255 ? o : 255);
      P[(size_t)PS_DIRTY * N + u] = 0;
      P[(size_t)PS_PRUNED * N + u] = 0;
    }
  }
  if (depart)  // u goes offline at the next epoch: flag its mesh neighbours
#pragma unroll
    for (int k = 0; k < HB_PER_LANE; k++)
      if ((uint32_t)(k * G + lane) < deg && (f[k] & F_MESH)) P[(size_t)PS_NBROFF * N + cw[k]] = 1;
}

// One step of an event-driven epoch. A block owns 64 * SW consecutive rows:
// its first wave tests them one thread per row and compacts the rows the step
// can change into LDS; then every group of G lanes takes active rows (most
// blocks have a handful, so one round). Steps:
enum : int { EV_HB = 0, EV_GRAFT = 1, EV_APPLY = 2 };
// SW scanning waves per block: a block owns 64 * SW rows (GS_EV_SW; the steps
// are short, so the number of workgroups per launch matters, not only the rows)
template <int G, int STEP, int SW>
__global__ __launch_bounds__(TB) void k_ev_step(MeshArgs a, uint32_t* mesh, const uint32_t* mesh_prev) {
  constexpr uint32_t RW = 64u * SW;
  static_assert(SW >= 1 && 64 * SW <= TB, "scanning waves of the block");
  // per active row: id, CSR base, degree, the step's flags (loaded by the scan,
  // so a row's own work starts with its entries)
  __shared__ uint32_t act[RW], actd[RW];
  __shared__ uint64_t actb[RW];
  __shared__ uint8_t actf[RW];
  __shared__ uint32_t nact;
  uint8_t* P = a.pst;
  const uint32_t N = a.N;
  const uint32_t base = blockIdx.x * RW;
  if (STEP == EV_APPLY) {  // unchanged rows keep their ELL row / mesh mask: copy the block's rows
    const uint32_t nrow = base + RW <= N ? RW : N - base;
    if (mesh && mesh_prev) {
      const uint4* src = reinterpret_cast<const uint4*>(mesh_prev + (size_t)base * MESH_W);
      uint4* dst = reinterpret_cast<uint4*>(mesh + (size_t)base * MESH_W);
      for (uint32_t i = threadIdx.x; i < nrow * (MESH_W / 4); i += TB) dst[i] = src[i];
    }
    if (a.mm_out && a.mm_prev)
      for (uint32_t i = threadIdx.x; i < nrow; i += TB) a.mm_out[base + i] = a.mm_prev[base + i];
  }
  if (SW > 1) {
    if (threadIdx.x == 0) nact = 0;
    __syncthreads();
  }
  if (threadIdx.x < 64 * SW) {
    const uint32_t l = threadIdx.x & 63;
    const uint32_t u = base + threadIdx.x;
    bool on = false;
    uint32_t fl = 0;
    uint64_t rb = 0, re = 0;
    if (u < N) {
      rb = a.row[u];
      re = a.row[u + 1];
      if (STEP == EV_HB) {
        const bool off = is_off(a.off, u), leaving = off && !is_off(a.off_prev, u);
        const uint32_t mc = P[(size_t)PS_MC * N + u], oc = P[(size_t)PS_OC * N + u];
        const bool propd = P[(size_t)PS_PROPD * N + u] != 0;
        on = leaving || P[(size_t)PS_NBROFF * N + u] || propd || (!off && (mc < a.d_lo || mc > a.d_hi || oc < a.d_out));
        fl = (propd ? 1u : 0u) | (off ? 2u : 0u);
      } else if (STEP == EV_GRAFT) {
        on = P[(size_t)PS_INBOX * N + u];
      } else {
        const bool need = P[(size_t)PS_PROPD * N + u] || P[(size_t)PS_PRUNED * N + u];
        // (the first epoch of a run writes every row: no previous snapshot to copy)
        const bool dirty = need || P[(size_t)PS_DIRTY * N + u] || (mesh && !mesh_prev) || (a.mm_out && !a.mm_prev);
        const bool depart = a.off_next && !is_off(a.off, u) && is_off(a.off_next, u);
        on = dirty || depart;
        fl = (need ? 1u : 0u) | (dirty ? 2u : 0u) | (depart ? 4u : 0u);
      }
    }
    const uint64_t bm = __ballot(on);
    uint32_t q0 = 0;  // this wave's first slot (one wave: 0; else claimed in LDS, any order)
    if (SW > 1) {
      if (l == 0 && bm) q0 = atomicAdd(&nact, (uint32_t)__popcll(bm));
      q0 = (uint32_t)__shfl((int)q0, 0);
    }
    if (on) {
      const uint32_t q = q0 + (uint32_t)__popcll(bm & ((1ull << l) - 1));
      act[q] = u;
      actb[q] = rb;
      actd[q] = (uint32_t)(re - rb);
      actf[q] = (uint8_t)fl;
    }
    if (SW == 1 && threadIdx.x == 0) nact = (uint32_t)__popcll(bm);
    if (a.dbg) {  // diagnostic counts (GS_DEBUG_EV)
      uint32_t c[4] = {(uint32_t)__popcll(bm), 0, 0, 0};
      if (STEP == EV_HB && u < N) {
        const bool off = is_off(a.off, u);
        const uint32_t mc = P[(size_t)PS_MC * N + u], oc = P[(size_t)PS_OC * N + u];
        c[1] = (uint32_t)__popcll(__ballot(off && !is_off(a.off_prev, u)));
        c[2] = (uint32_t)__popcll(__ballot(P[(size_t)PS_NBROFF * N + u] != 0));
        c[3] = (uint32_t)__popcll(__ballot(!off && (mc < a.d_lo || mc > a.d_hi || oc < a.d_out)));
      } else if (STEP == EV_HB) {
        c[1] = (uint32_t)__popcll(__ballot(false));
        c[2] = (uint32_t)__popcll(__ballot(false));
        c[3] = (uint32_t)__popcll(__ballot(false));
      }
      if (l == 0)
        for (int q = 0; q < 4; q++)
          if (c[q]) atomicAdd(&a.dbg[STEP * 4 + q], (unsigned long long)c[q]);
    }
  }
  __syncthreads();  // also orders the ELL copy before the re-extracted rows
  const int lane = threadIdx.x & (G - 1);
  const uint32_t n = nact;
  for (uint32_t i = threadIdx.x / G; i < n; i += TB / G) {  // group-uniform
    const uint32_t u = act[i], deg = actd[i], fl = actf[i];
    const uint64_t b = actb[i];
    if (STEP == EV_HB) {
      if (lane == 0) {
        P[(size_t)PS_PROPD * N + u] = 0;
        P[(size_t)PS_NBROFF * N + u] = 0;
      }
      if (row_hb_ev<G>(a, u, b, deg, (fl & 1u) != 0, (fl & 2u) != 0) && lane == 0) P[(size_t)PS_DIRTY * N + u] = 1;
    } else if (STEP == EV_GRAFT) {
      const bool acc = row_handle_graft<G>(a, u, b, deg);
      if (lane == 0) {
        P[(size_t)PS_INBOX * N + u] = 0;
        if (acc) P[(size_t)PS_DIRTY * N + u] = 1;
      }
    } else {
      // (depart: the departures of the next epoch flag their mesh neighbours)
      row_apply_ev<G>(a, u, b, deg, (fl & 1u) != 0, (fl & 2u) != 0, (fl & 4u) != 0, mesh);
    }
  }
}


inline unsigned blocks(uint64_t n) { return (unsigned)((n + TB - 1) / TB); }

// Lanes per peer of the row kernels: 16 (four peers per wave) when every row
// fits 4 x 16 entries, else 64 (GS_ROW_GROUP=64 forces one peer per wave).
inline uint32_t row_group(const Ctx& c) {
  static const char* e = getenv("GS_ROW_GROUP");
  if (e && atoi(e) == 64) return 64u;
  return c.max_degree <= 4 * 16 ? 16u : 64u;
}
inline unsigned row_blocks(uint32_t N, uint32_t G) { return (unsigned)(((uint64_t)N * G + TB - 1) / TB); }
#define GS_ROWS(kernel, G, N, s, ...)                                                   \
  do {                                                                                   \
    if ((G) == 16) kernel<16><<<row_blocks(N, 16), TB, 0, s>>>(__VA_ARGS__);            \
    else kernel<64><<<row_blocks(N, 64), TB, 0, s>>>(__VA_ARGS__);                      \
  } while (0)

// Inverse IHAVE lists of the ring snapshots: epochs per chunk (the masks of a
// chunk take <= 256 MB of d_gout), one chunk [h0, h0 + ny) on stream s.
static uint64_t ring_in_chunk_epochs(uint32_t N) {
  return std::max<uint64_t>(1, std::min<uint64_t>(64, (256ull << 20) / ((uint64_t)N * 8)));
}
static void ring_in_prepare(Ctx& c, uint64_t E, hipStream_t s) {
  const uint32_t N = c.cfg.peers;
  c.d_csrpos.alloc(c.nnz ? c.nnz : 1);
  c.d_gout.alloc((size_t)std::min<uint64_t>(ring_in_chunk_epochs(N), E) * N);
  k_csrpos<<<blocks(N), TB, 0, s>>>(N, c.d_row.p, c.d_col.p, c.d_rev.p, c.d_csrpos.p);
}
// bpc = blocks per CU (0: one thread / group per item): beside the epoch steps
// the lists run on a capped grid, so the steps' blocks find free slots
static void ring_in_chunk(Ctx& c, uint64_t h0, uint32_t ny, hipStream_t s, uint32_t bpc = 0) {
  const uint32_t N = c.cfg.peers, R = c.ring_R, w64 = (N + 63) / 64;
  if (c.ring_in_tag.size() != R) c.ring_in_tag.assign(R, ~0ull);
  for (uint64_t h = h0; h < h0 + ny; h++) c.ring_in_tag[h % R] = h;
  const uint64_t cap = bpc ? (uint64_t)std::max(c.num_cus, 1) * bpc : ~0ull;
  const unsigned g1 = (unsigned)std::min<uint64_t>(cap, ((uint64_t)N * ny + TB - 1) / TB);
  const unsigned g2 = (unsigned)std::min<uint64_t>(cap, ((uint64_t)N * ny * GIN_G + TB - 1) / TB);
  k_gossip_out_range<<<g1, TB, 0, s>>>(c.d_row.p, c.d_col.p, c.d_ring_mesh.p, c.d_ring_off.p, N, w64, R, c.cfg.seed,
                                       h0, c.cfg.d_lazy, c.cfg.gossip_factor_milli, c.d_gout.p, ny);
  k_gossip_in_gather<<<g2, TB, 0, s>>>(c.d_row.p, c.d_col.p, c.d_csrpos.p, c.d_ring_off.p, c.d_stage.p, N, w64, R, h0,
                                       c.d_gout.p, c.d_ring_in.p, ny);
}
// (deferred while the churn list pass takes the batches: it decides IHAVEs from
// the mask ring; ensure_in_lists builds them when a batch falls back to the push path)
static bool ring_in_wanted(const Ctx& c) { return c.cfg.lazy_gossip && c.d_ring_in.p && !c.ring_in_defer; }

// Epochs [h0, h1] (h1 - h0 < ring_R) on the context's stream: per chunk of
// epochs, the senders' target masks, then every receiver's list
// (k_gossip_out_range, k_gossip_in_gather).
void ring_in_lists(Ctx& c, uint64_t h0, uint64_t h1) {
  if (!ring_in_wanted(c)) return;
  const uint64_t E = h1 - h0 + 1, CE = ring_in_chunk_epochs(c.cfg.peers);
  ring_in_prepare(c, E, c.stream);
  for (uint64_t y0 = 0; y0 < E; y0 += CE) ring_in_chunk(c, h0 + y0, (uint32_t)std::min<uint64_t>(CE, E - y0), c.stream);
  GS_HIP(hipGetLastError());
}

// Side stream + its i-th event (created on first use).
static hipEvent_t side_event(Ctx& c, size_t i) {
  if (!c.side) {  // lowest priority: the epoch steps' dependent chain is dispatched first
    int lo = 0, hi = 0;
    GS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    const char* sp = getenv("GS_SIDE_PRIORITY");  // A/B knob: 0 = default priority
    if (const uint32_t x = xcd_env("GS_SIDE_XCDS")) c.side = xcd_stream(c, x);  // (experiment: its XCDs)
    else if (sp && *sp && atoi(sp) == 0) GS_HIP(hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking));
    else GS_HIP(hipStreamCreateWithPriority(&c.side, hipStreamNonBlocking, lo));
  }
  while (c.side_ev.size() <= i) {
    hipEvent_t e;
    GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c.side_ev.push_back(e);
  }
  return c.side_ev[i];
}

MeshArgs mesh_args(Ctx& c, hipStream_t s = nullptr) {
  const uint32_t N = c.cfg.peers;
  c.d_until.alloc(c.nnz ? c.nnz : 1);
  c.d_prop.alloc(c.nnz ? c.nnz : 1);
  if (!c.lat32_ok) {  // (once per link set: gs_set_links clears it)
    if (!s) s = c.stream;
    c.d_lat32.alloc((size_t)c.S * c.S);
    std::vector<uint32_t> lat32(c.lat_ns.begin(), c.lat_ns.end());
    GS_HIP(hipMemcpyAsync(c.d_lat32.p, lat32.data(), lat32.size() * 4, hipMemcpyHostToDevice, s));
    GS_HIP(hipStreamSynchronize(s));  // lat32 dies here
    c.lat32_ok = true;
  }
  MeshArgs a{};
  a.row = c.d_row.p; a.col = c.d_col.p; a.rev = c.d_rev.p; a.flags = c.d_flags.p;
  a.prop = c.d_prop.p; a.until = c.d_until.p; a.stage = c.d_stage.p; a.lat = c.d_lat32.p;
  a.counters = c.d_counters.p; a.seed = c.cfg.seed; a.N = N; a.S = c.S;
  a.bo = (uint32_t)((c.cfg.backoff_ns + c.cfg.heartbeat_ns - 1) / c.cfg.heartbeat_ns);
  a.d = c.cfg.d; a.d_lo = c.cfg.d_lo; a.d_hi = c.cfg.d_hi; a.d_out = c.cfg.d_out;
  return a;
}

// The subscription epoch 0 from the cleared mesh (everyone online; DESIGN.md
// §2.3): handshake-ordered grafts, GRAFT handling, apply.
void sub_epoch(Ctx& c, MeshArgs a) {
  if (!c.cfg.sub_graft) return;
  const uint32_t N = c.cfg.peers;
  hipStream_t s = c.stream;
  a.sub = c.cfg.hs_rtts ? c.cfg.hs_rtts : HS_RTTS;
  a.epoch = 0;
  a.off = nullptr;
  GS_HIP(hipMemsetAsync(c.d_prop.p, 0, c.nnz ? c.nnz : 1, s));
  const uint32_t G = row_group(c);
  GS_ROWS(k_heartbeat, G, N, s, a);
  GS_ROWS(k_handle_graft, G, N, s, a);
  GS_ROWS(k_apply, G, N, s, a);
  GS_HIP(hipGetLastError());
}

// Epoch h of a run [h0, h1] of event-driven epochs (three steps on stream s):
// lin[y] = offline bitset of epoch h0 - 1 + y; `ring`: the slot h % ring_R gets
// the mask ring row (and, `ell`, the ELL snapshot).
static void ev_epoch(Ctx& c, MeshArgs& a, uint64_t h, uint64_t h0, uint64_t h1, const uint64_t* lin, uint32_t w64,
                     bool ring, bool ell, uint32_t G, hipStream_t s) {
  const uint32_t N = c.cfg.peers;
  static const uint32_t ev_sw = [] {  // GS_EV_SW: scanning waves (rows / 64) per block of the steps
    const char* e = getenv("GS_EV_SW");
    const int v = e && *e ? atoi(e) : 1;
    return (uint32_t)(v >= 4 ? 4 : v >= 2 ? 2 : 1);
  }();
  const unsigned sgrid = (unsigned)((N + 64 * ev_sw - 1) / (64 * ev_sw));
#define GS_EVS1(SW, STEP, ...)                                                     \
  do {                                                                             \
    if (G == 16) k_ev_step<16, STEP, SW><<<sgrid, TB, 0, s>>>(__VA_ARGS__);        \
    else k_ev_step<64, STEP, SW><<<sgrid, TB, 0, s>>>(__VA_ARGS__);                \
  } while (0)
#define GS_EVS(STEP, ...)                                                          \
  do {                                                                             \
    if (ev_sw == 4) GS_EVS1(4, STEP, __VA_ARGS__);                                 \
    else if (ev_sw == 2) GS_EVS1(2, STEP, __VA_ARGS__);                            \
    else GS_EVS1(1, STEP, __VA_ARGS__);                                            \
  } while (0)
  const uint64_t y = h - h0 + 1;
  a.epoch = (uint32_t)h;
  a.off = lin + y * w64;
  a.off_prev = lin + (y - 1) * w64;
  a.off_next = h < h1 ? lin + (y + 1) * w64 : nullptr;
  uint32_t* mesh = ell ? c.d_ring_mesh.p + (size_t)(h % c.ring_R) * N * MESH_W : nullptr;
  const uint32_t* prev = ell && h > h0 ? c.d_ring_mesh.p + (size_t)((h - 1) % c.ring_R) * N * MESH_W : nullptr;
  if (ring) {
    if (c.ring_ell_tag.size() != c.ring_R) c.ring_ell_tag.assign(c.ring_R, ~0ull);
    c.ring_ell_tag[h % c.ring_R] = ell ? h : ~0ull;
  }
  const bool mmr = ring && c.d_ring_mm.p;
  a.mm_out = mmr ? c.d_ring_mm.p + (size_t)(h % c.ring_R) * N : nullptr;
  a.mm_prev = mmr && h > h0 ? c.d_ring_mm.p + (size_t)((h - 1) % c.ring_R) * N : nullptr;
  MeshArgs an = a;  // the mask ring is written by the apply step only
  an.mm_out = nullptr;
  an.mm_prev = nullptr;
  GS_EVS(EV_HB, an, nullptr, nullptr);
  GS_EVS(EV_GRAFT, an, nullptr, nullptr);
  GS_EVS(EV_APPLY, a, mesh, prev);
#undef GS_EVS
#undef GS_EVS1
}

// Event-driven churn epochs [h0, h1] (see k_ev_step): offline bitsets
// of [h0-1, h1] in one launch (and into the ring), three row steps per epoch,
// then the IHAVE targets of every ring slot written.
void ev_epochs(Ctx& c, MeshArgs a, uint64_t h0, uint64_t h1, bool ring) {
  const uint32_t N = c.cfg.peers;
  const uint32_t w64 = (N + 63) / 64;
  hipStream_t s = c.stream;
  const uint64_t E = h1 - h0 + 1;
  // the range may be longer than the ring: only its last ring_R epochs keep
  // their slots (offline bits and targets are written in parallel over epochs)
  const uint64_t hr = ring && E > c.ring_R ? h1 + 1 - c.ring_R : h0;
  c.d_offlin.alloc((size_t)(E + 1) * w64);
  for (uint64_t y0 = 0; y0 < E + 1; y0 += 32768) {  // grid.y limit
    const uint32_t ny = (uint32_t)std::min<uint64_t>(32768, E + 1 - y0);
    k_offline_range<<<dim3(blocks(N), ny), TB, 0, s>>>(N, c.cfg.seed, c.cfg.churn_ppm, c.cfg.churn_down,
                                                       h0 - 1 + y0, c.d_offlin.p + y0 * w64, w64,
                                                       ring ? c.d_ring_off.p : nullptr, c.ring_R, hr);
  }
  c.d_pst.alloc((size_t)PS_PLANES * N);
  GS_HIP(hipMemsetAsync(c.d_pst.p, 0, (size_t)PS_MC * N, s));         // flags clear
  GS_HIP(hipMemsetAsync(c.d_pst.p + (size_t)PS_DIRTY * N, 1, N, s));  // first epoch: extract every row
  GS_HIP(hipMemsetAsync(c.d_prop.p, 0, c.nnz ? c.nnz : 1, s));
  c.d_iprop.alloc(c.nnz ? c.nnz : 1);
  GS_HIP(hipMemsetAsync(c.d_iprop.p, 0, c.nnz ? c.nnz : 1, s));
  const uint64_t* lin = c.d_offlin.p;  // lin[y] = epoch h0 - 1 + y
  a.pst = c.d_pst.p;
  a.iprop = c.d_iprop.p;
  static const bool dbg_ev = getenv("GS_DEBUG_EV") != nullptr;
  DevBuf<uint64_t> dbg;
  if (dbg_ev) {
    dbg.alloc(12);
    GS_HIP(hipMemsetAsync(dbg.p, 0, 12 * 8, s));
    a.dbg = (unsigned long long*)dbg.p;
  }
  a.off = lin + w64;
  a.off_prev = lin;
  a.off_next = nullptr;
  const uint32_t G = row_group(c);
  if (c.num_cus == 0) {
    hipDeviceProp_t prop;
    c.num_cus = hipGetDeviceProperties(&prop, c.cfg.device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(row_blocks(N, G), (uint64_t)c.num_cus * 8));
  if (G == 16) k_ev_init<16><<<grid, TB, 0, s>>>(a);
  else k_ev_init<64><<<grid, TB, 0, s>>>(a);
  if (c.epoch_hook && ring) c.epoch_hook(h0 - 1);
  // the IHAVE lists of the ring epochs [hr, h1] run on the side stream, a
  // chunk as soon as its epochs are stepped (compute-bound list kernels beside
  // the latency-bound epoch steps)
  const bool lists = ring && ring_in_wanted(c);
  const char* sb = getenv("GS_SIDE_BPC");  // list blocks per CU beside the steps (0: full grid)
  const uint32_t side_bpc = sb && *sb ? (uint32_t)atoi(sb) : 2u;
  const uint64_t CE = ring_in_chunk_epochs(N);
  uint64_t chunk0 = hr;
  size_t nev = 0;
  if (lists) {
    const hipEvent_t e = side_event(c, nev++);
    ring_in_prepare(c, h1 - hr + 1, c.side);  // (hipMalloc before the side stream waits)
    GS_HIP(hipEventRecord(e, s));
    GS_HIP(hipStreamWaitEvent(c.side, e, 0));
  }
  for (uint64_t h = h0; h <= h1; h++) {
    ev_epoch(c, a, h, h0, h1, lin, w64, ring, ring && !(c.ring_ell_defer && c.d_ring_mm.p), G, s);
    if (c.epoch_hook && ring) c.epoch_hook(h);
    if (lists && h >= hr && (h + 1 - chunk0 == CE || h == h1)) {
      const hipEvent_t e = side_event(c, nev++);
      GS_HIP(hipEventRecord(e, s));
      GS_HIP(hipStreamWaitEvent(c.side, e, 0));
      ring_in_chunk(c, chunk0, (uint32_t)(h + 1 - chunk0), c.side, side_bpc);
      chunk0 = h + 1;
    }
  }
  GS_HIP(hipGetLastError());
  if (lists) {  // the context's stream continues once every list is written
    const hipEvent_t e = side_event(c, nev++);
    GS_HIP(hipEventRecord(e, c.side));
    GS_HIP(hipStreamWaitEvent(s, e, 0));
  }
  if (dbg_ev) {
    uint64_t h[12];
    GS_HIP(hipMemcpyAsync(h, dbg.p, sizeof h, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    fprintf(stderr, "[gs] epochs %llu: active rows hb %llu (leaving %llu nbr-off %llu hungry %llu) graft %llu apply %llu\n",
            (unsigned long long)E, (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2],
            (unsigned long long)h[3], (unsigned long long)h[4], (unsigned long long)h[8]);
  }
}

// Churn epochs [h0, h1] from the current mesh state (ev_epochs); `ring`:
// also the ELL snapshots (+ inverse IHAVE lists) into the ring slots h % ring_R.
void run_epochs(Ctx& c, MeshArgs a, uint64_t h0, uint64_t h1, bool ring) { ev_epochs(c, a, h0, h1, ring); }

}  // namespace

hipStream_t side_stream(Ctx& c) {
  (void)side_event(c, 0);
  return c.side;
}

// The inverse IHAVE lists of ring epochs [h0, h1] that were deferred (the push
// path's receiver-centric gossip reads them), on the context's stream.
void ensure_in_lists(Ctx& c, uint64_t h0, uint64_t h1) {
  if (!c.cfg.lazy_gossip || !c.d_ring_in.p) return;
  const uint32_t R = c.ring_R;
  if (c.ring_in_tag.size() != R) c.ring_in_tag.assign(R, ~0ull);
  const uint64_t CE = ring_in_chunk_epochs(c.cfg.peers);
  bool prepared = false;
  for (uint64_t h = h0; h <= h1;) {
    if (c.ring_in_tag[h % R] == h) { h++; continue; }
    uint64_t e = h;  // a run of epochs without lists, at most one chunk
    while (e + 1 <= h1 && e + 1 - h < CE && c.ring_in_tag[(e + 1) % R] != e + 1) e++;
    if (!prepared) ring_in_prepare(c, std::min<uint64_t>(CE, h1 - h0 + 1), c.stream);
    prepared = true;
    ring_in_chunk(c, h, (uint32_t)(e - h + 1), c.stream);
    h = e + 1;
  }
  GS_HIP(hipGetLastError());
}

// Make the churn ring hold the snapshots of epochs [h_lo, h_hi] (h_hi - h_lo
// < ring_R): replay from the empty mesh when h_lo has left the ring, else run
// the epochs after the current mesh state. Snapshot h = mesh after heartbeat h
// with the offline bits of epoch h; epoch 0 is the empty mesh, all online.
// A stream restricted to n compute units (bits [c0, c0 + n) of
// hipExtStreamCreateWithCUMask's mask; GS_CU_STRIDE=s takes every s-th bit).
hipStream_t cu_stream(Ctx& c, uint32_t c0, uint32_t n) {
  ensure_cus(c);
  const uint32_t total = (uint32_t)std::max(c.num_cus, 1);
  const char* st = getenv("GS_CU_STRIDE");
  const uint32_t stride = st && *st ? (uint32_t)std::max(1, atoi(st)) : 1u;
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t b = (c0 + i * stride) % total;
    mask[b / 32] |= 1u << (b % 32);
  }
  hipStream_t s = nullptr;
  GS_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  return s;
}

// A stream on every CU except the bits c0, c0 + stride, ... (the complement of
// cu_stream(c, c0, total / stride) with GS_CU_STRIDE = stride).
hipStream_t cu_stream_except(Ctx& c, uint32_t c0, uint32_t stride) {
  ensure_cus(c);
  const uint32_t total = (uint32_t)std::max(c.num_cus, 1);
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (uint32_t b = 0; b < total; b++)
    if (stride == 0 || b < c0 || (b - c0) % stride != 0) mask[b / 32] |= 1u << (b % 32);
  hipStream_t s = nullptr;
  GS_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  return s;
}

// A stream on the CUs of the XCDs in `xcds` (bit x: XCD x). The CU mask's bit b
// is CU b / XCDS of XCD b % XCDS (measured: bits 0, 8, 16, ... run the epoch
// chain as fast as all 256 CUs, bits 0..31 take twice as long).
constexpr uint32_t XCDS = 8;
hipStream_t xcd_stream(Ctx& c, uint32_t xcds) {
  ensure_cus(c);
  const uint32_t total = (uint32_t)std::max(c.num_cus, 1);
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (uint32_t b = 0; b < total; b++)
    if ((xcds >> (b % XCDS)) & 1u) mask[b / 32] |= 1u << (b % 32);
  hipStream_t s = nullptr;
  GS_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  return s;
}
// "0", "1,2", "3-7" -> XCD bits (0: unset or empty)
uint32_t xcd_env(const char* name) {
  const char* e = getenv(name);
  if (!e || !*e) return 0;
  uint32_t m = 0;
  for (const char* p = e; *p;) {
    char* q = nullptr;
    const long a = strtol(p, &q, 10);
    if (q == p) break;
    long b = a;
    if (*q == '-') {
      p = q + 1;
      b = strtol(p, &q, 10);
    }
    for (long x = a; x <= b && x < (long)XCDS; x++)
      if (x >= 0) m |= 1u << x;
    p = *q ? q + 1 : q;
  }
  return m;
}

// GS_CHAIN_CUS=n (experiment): the epoch chain of churn_ring on a stream of n CUs.
static uint32_t chain_cus() {
  const char* e = getenv("GS_CHAIN_CUS");
  if (const uint32_t x = xcd_env("GS_CHAIN_XCDS")) return 0x10000u | x;  // (GS_CHAIN_XCDS wins)
  return e && *e ? (uint32_t)std::max(0, atoi(e)) : 0u;
}

static void churn_ring_on(Ctx& c, uint64_t h_lo, uint64_t h_hi);
void churn_ring(Ctx& c, uint64_t h_lo, uint64_t h_hi) {
  const uint32_t n = c.chain_pipe ? 0u : chain_cus();
  if (!n && !c.chain_pipe) return churn_ring_on(c, h_lo, h_hi);
  static uint32_t made = 0;  // (experiment: one mask per process)
  if (!c.chain_pipe && (!c.chain || made != n)) {
    if (c.chain) GS_HIP(hipStreamDestroy(c.chain));
    c.chain = n & 0x10000u ? xcd_stream(c, n & 0xFFu) : cu_stream(c, 0, n);
    made = n;
    for (auto& e : c.chain_ev)
      if (e) GS_HIP(hipEventDestroy(e));
    for (auto& e : c.chain_ev) GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipStream_t main = c.stream, cs = c.chain_pipe ? c.chain_pipe : c.chain;
  for (auto& e : c.chain_ev)
    if (!e) GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  GS_HIP(hipEventRecord(c.chain_ev[0], main));
  GS_HIP(hipStreamWaitEvent(cs, c.chain_ev[0], 0));
  c.stream = cs;  // every launch of the chain (and the hook's events) on the chain's CUs
  try {
    churn_ring_on(c, h_lo, h_hi);
  } catch (...) {
    c.stream = main;
    throw;
  }
  c.stream = main;
  GS_HIP(hipEventRecord(c.chain_ev[1], cs));
  GS_HIP(hipStreamWaitEvent(main, c.chain_ev[1], 0));
}

static void churn_ring_on(Ctx& c, uint64_t h_lo, uint64_t h_hi) {
  const uint32_t N = c.cfg.peers, R = c.ring_R;
  const size_t w64 = ((size_t)N + 63) / 64;
  hipStream_t s = c.stream;
  if (h_hi - h_lo >= R) c.fail(GS_EINVAL, "internal: batch spans more epochs than the churn ring");
  MeshArgs a = mesh_args(c);
  if (h_lo < c.ring_lo) {  // replay from epoch 0
    if (c.nnz) k_clear_mesh<<<blocks(c.nnz), TB, 0, s>>>(c.nnz, c.d_flags.p, c.d_until.p);
    sub_epoch(c, a);
    c.churn_state = 0;
    c.ring_hi = 0;
    c.ring_lo = 1;
    if (h_lo == 0) {  // slot 0: the mesh after the subscription exchange (empty without it); a
      // row may be wider than the ELL before heartbeat 1 prunes it (GS_ERANGE below)
      MeshArgs a0 = a;
      a0.mm_out = c.d_ring_mm.p;  // slot 0 (nullptr: no mask ring)
      k_extract<<<blocks(N), TB, 0, s>>>(a0, c.d_ring_mesh.p, nullptr);
      if (c.ring_ell_tag.size() != R) c.ring_ell_tag.assign(R, ~0ull);
      c.ring_ell_tag[0] = 0;
      GS_HIP(hipMemsetAsync(c.d_ring_off.p, 0, w64 * 8, s));
      ring_in_lists(c, 0, 0);
      c.ring_lo = 0;
    }
  }
  if (c.churn_state + 1 <= h_hi)
    run_epochs(c, a, c.churn_state + 1, h_hi, true);
  GS_HIP(hipGetLastError());
  if (h_hi > c.churn_state) {
    c.churn_state = h_hi;
    c.ring_hi = h_hi;
    c.ring_lo = std::max<uint64_t>(c.ring_lo, h_hi + 1 >= R ? h_hi + 1 - R : 0);
  }
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_counters.p + C_ERR, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  if (c.h_pinned[0] & ERR_MESH) c.fail(GS_ERANGE, "mesh row exceeds GS_MESH_W entries");
}

// The epoch chain of a churn list-pass batch enqueued in slices (the batch
// after the current one runs its chain beside the current batch's passes,
// gs_relax.hip ChnAhead): epochs churn_state + 1 .. h1 on stream s, the mask
// ring only (no ELL snapshots, no inverse IHAVE lists: the list pass reads
// neither), the hook after every epoch (the batch tables' chunks). The ring
// bookkeeping (churn_state, ring_lo / hi) moves when the last epoch is enqueued.
struct EvRun {
  MeshArgs a{};
  uint64_t h0 = 0, h1 = 0, h = 0;
  uint32_t w64 = 0, G = 16;
  hipStream_t s = nullptr;
  std::function<void(uint64_t)> hook;
};
void chain_free(EvRun* r) { delete r; }
EvRun* chain_begin(Ctx& c, uint64_t h1, hipStream_t s, std::function<void(uint64_t)> hook) {
  const uint32_t N = c.cfg.peers;
  if (c.churn_state + 1 > h1 || c.churn_state + 1 < c.ring_lo || h1 - c.churn_state > c.ring_R || !c.d_ring_mm.p)
    return nullptr;  // (nothing to run, or not a plain continuation: the caller runs churn_ring)
  EvRun* r = new EvRun();
  r->a = mesh_args(c, s);
  r->h0 = r->h = c.churn_state + 1;
  r->h1 = h1;
  r->w64 = (N + 63) / 64;
  r->G = row_group(c);
  r->s = s;
  r->hook = std::move(hook);
  const uint64_t E = h1 - r->h0 + 1;
  c.d_offlin.alloc((size_t)(E + 1) * r->w64);
  for (uint64_t y0 = 0; y0 < E + 1; y0 += 32768) {  // grid.y limit
    const uint32_t ny = (uint32_t)std::min<uint64_t>(32768, E + 1 - y0);
    k_offline_range<<<dim3(blocks(N), ny), TB, 0, s>>>(N, c.cfg.seed, c.cfg.churn_ppm, c.cfg.churn_down,
                                                       r->h0 - 1 + y0, c.d_offlin.p + y0 * r->w64, r->w64,
                                                       c.d_ring_off.p, c.ring_R, r->h0);
  }
  c.d_pst.alloc((size_t)PS_PLANES * N);
  GS_HIP(hipMemsetAsync(c.d_pst.p, 0, (size_t)PS_MC * N, s));
  GS_HIP(hipMemsetAsync(c.d_pst.p + (size_t)PS_DIRTY * N, 1, N, s));
  GS_HIP(hipMemsetAsync(c.d_prop.p, 0, c.nnz ? c.nnz : 1, s));
  c.d_iprop.alloc(c.nnz ? c.nnz : 1);
  GS_HIP(hipMemsetAsync(c.d_iprop.p, 0, c.nnz ? c.nnz : 1, s));
  r->a.pst = c.d_pst.p;
  r->a.iprop = c.d_iprop.p;
  r->a.dbg = nullptr;
  r->a.off = c.d_offlin.p + r->w64;
  r->a.off_prev = c.d_offlin.p;
  r->a.off_next = nullptr;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(row_blocks(N, r->G), (uint64_t)c.num_cus * 8));
  if (r->G == 16) k_ev_init<16><<<grid, TB, 0, s>>>(r->a);
  else k_ev_init<64><<<grid, TB, 0, s>>>(r->a);
  GS_HIP(hipGetLastError());
  if (r->hook) r->hook(r->h0 - 1);
  return r;
}
bool chain_advance(Ctx& c, EvRun& r, uint64_t max_epochs) {
  for (uint64_t k = 0; k < max_epochs && r.h <= r.h1; k++, r.h++) {
    ev_epoch(c, r.a, r.h, r.h0, r.h1, c.d_offlin.p, r.w64, true, false, r.G, r.s);
    if (r.hook) r.hook(r.h);
  }
  GS_HIP(hipGetLastError());
  if (r.h <= r.h1) return false;
  if (r.h1 > c.churn_state) {  // (as churn_ring: the state and the ring's valid range)
    c.churn_state = r.h1;
    c.ring_hi = r.h1;
    c.ring_lo = std::max<uint64_t>(c.ring_lo, r.h1 + 1 >= c.ring_R ? r.h1 + 1 - c.ring_R : 0);
  }
  return true;
}

// ELL snapshots of ring epochs [h0, h0 + gridDim.y) rebuilt from the mask ring:
// row u's mesh = its CSR entries (ccol: stage << 24 | peer, ascending, the ELL
// order) whose bit is set. One wave per row.
__global__ __launch_bounds__(TB) void k_mm2ell(const uint32_t* __restrict__ ccol, const uint64_t* __restrict__ ring_mm,
                                               uint32_t* __restrict__ ring_mesh, uint32_t N, uint32_t R, uint64_t h0,
                                               uint64_t* counters) {
  const uint32_t lane = threadIdx.x & 63, u = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  if (u >= N) return;
  const size_t slot = (size_t)((h0 + blockIdx.y) % R);
  const uint64_t m = ring_mm[slot * N + u];
  const uint32_t x = ccol[(size_t)u * 64 + lane];
  const bool in = (m >> lane) & 1ull;
  const uint64_t bm = __ballot(in);
  const uint32_t pos = (uint32_t)__popcll(bm & ((1ull << lane) - 1)), cnt = (uint32_t)__popcll(bm);
  uint32_t* row = ring_mesh + (slot * N + u) * MESH_W;
  if (in && pos < MESH_W) row[pos] = x;
  if (lane >= cnt && lane < MESH_W) row[lane] = EMPTY;
  if (cnt > MESH_W && lane == 0) atomicOr((unsigned*)&counters[C_ERR], ERR_MESH);
}

// The ELL snapshots of ring epochs [h0, h1] the epochs skipped (ring_ell_defer),
// on the context's stream (the mask ring and the 64-wide CSR rows hold them).
void ensure_ring_ell(Ctx& c, uint64_t h0, uint64_t h1) {
  if (!c.d_ring_mm.p || !c.cell_valid) return;  // (no mask ring: every epoch wrote its ELL)
  const uint32_t R = c.ring_R, N = c.cfg.peers;
  if (c.ring_ell_tag.size() != R) c.ring_ell_tag.assign(R, ~0ull);
  for (uint64_t h = h0; h <= h1;) {
    if (c.ring_ell_tag[h % R] == h) { h++; continue; }
    uint64_t e = h;
    while (e + 1 <= h1 && e + 1 - h < 32768 && c.ring_ell_tag[(e + 1) % R] != e + 1) e++;
    k_mm2ell<<<dim3((N + TB / 64 - 1) / (TB / 64), (unsigned)(e - h + 1)), TB, 0, c.stream>>>(
        c.d_ccol.p, c.d_ring_mm.p, c.d_ring_mesh.p, N, R, h, c.d_counters.p);
    for (uint64_t k = h; k <= e; k++) c.ring_ell_tag[k % R] = k;
    h = e + 1;
  }
  GS_HIP(hipGetLastError());
}

// Position of each row's peer in its neighbour's row (k_csrpos), once per CSR:
// the IHAVE receivers of the list pass test their bit in the sender's target mask.
void ensure_csrpos(Ctx& c) {
  if (c.csrpos_valid) return;
  c.d_csrpos.alloc(c.nnz ? c.nnz : 1);
  k_csrpos<<<blocks(c.cfg.peers), TB, 0, c.stream>>>(c.cfg.peers, c.d_row.p, c.d_col.p, c.d_rev.p, c.d_csrpos.p);
  GS_HIP(hipGetLastError());
  c.csrpos_valid = true;
}

uint32_t run_mesh(Ctx& c, uint32_t max_hb) {
  const uint32_t N = c.cfg.peers;
  hipStream_t s = c.stream;
  MeshArgs a = mesh_args(c);
  if (c.nnz) k_clear_mesh<<<blocks(c.nnz), TB, 0, s>>>(c.nnz, c.d_flags.p, c.d_until.p);
  GS_HIP(hipMemsetAsync(c.d_counters.p + C_ERR, 0, 8, s));
  c.ring_in_tag.assign(c.ring_in_tag.size(), ~0ull);  // a new mesh: the churn ring restarts
  c.ring_ell_tag.assign(c.ring_ell_tag.size(), ~0ull);
  c.glp_prefer = false;  // and gossip batches try the eager pass + no-op proof first again
  sub_epoch(c, a);
  uint32_t epoch = 1, last = 0;
  uint64_t* h = c.h_pinned;
  if (c.cfg.churn_ppm) {  // no fixed point under churn: exactly max_hb epochs
    if (max_hb >= 1) run_epochs(c, a, 1, max_hb, false);
    last = max_hb;
    c.churn_state = max_hb;  // the ring restarts after this state
    c.ring_lo = (uint64_t)max_hb + 1;
    c.ring_hi = max_hb;
    epoch = max_hb + 1;
  }
  while (epoch <= max_hb) {
    a.epoch = epoch;
    GS_HIP(hipMemsetAsync(c.d_prop.p, 0, c.nnz ? c.nnz : 1, s));
    GS_HIP(hipMemsetAsync(c.d_counters.p + C_MESH_CHANGES, 0, 8, s));
    const uint32_t G = row_group(c);
    GS_ROWS(k_heartbeat, G, N, s, a);
    GS_ROWS(k_handle_graft, G, N, s, a);
    GS_ROWS(k_apply, G, N, s, a);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(h, c.d_counters.p + C_MESH_CHANGES, 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    last = epoch;
    if (h[0]) { epoch++; continue; }
    GS_HIP(hipMemsetAsync(c.d_counters.p + C_MESH_WAKE, 0xFF, 8, s));
    k_wake<<<blocks(N), TB, 0, s>>>(a);
    GS_HIP(hipMemcpyAsync(h, c.d_counters.p + C_MESH_WAKE, 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    if (h[0] == INF64 || h[0] > max_hb) break;
    epoch = (uint32_t)h[0];
  }
  c.d_mesh.alloc((size_t)N * MESH_W);
  c.rpos_valid = false;
  c.mesh_dmax = 0;
  c.d_mcnt.alloc(N);
  k_extract<<<blocks(N), TB, 0, s>>>(a, c.d_mesh.p, c.d_mcnt.p);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(h, c.d_counters.p + C_ERR, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  if (h[0] & ERR_MESH) c.fail(GS_ERANGE, "mesh row exceeds GS_MESH_W entries");
  return last;
}

}  // namespace gs
