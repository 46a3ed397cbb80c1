// gs_relax.hip — eager forwarding + seen-cache + uplink FIFO + reassembly as
// Delta-stepping frontier relaxation over a batch of concurrent messages.
//
// Reference behaviour replaced: publish_new_message
// (rust-test-node/src/main.rs:101-143) flood-publishes F fragments; each peer's
// first receipt of a fragment is forwarded to mesh \ {src, publisher}
// (libp2p-gossipsub forward_msg, upstream) through the peer's uplink FIFO;
// create_message_handler (main.rs:79-99) completes on the F-th fragment.
//
// Layout (HBM): keys[u][m][f] (u64, peer-major, f padded to FP = 2^k) holds
// key = t_rel_ns << (6+sb) | hops << sb | src; min key wins, so the seen-cache
// IS the key array and ties break on (time, hops, src) deterministically.
// Every relaxation adds >= Delta = min latency + min serialisation, so all
// keys inside the current bucket [lo, lo+Delta) are final: one launch per
// non-empty bucket scans the keys (coalesced), forwards the bucket's arrivals
// with 64-bit atomicMin pushes into the same (m,f) slot of the targets, and
// reduces the next pending key to pick the next bucket on the device
// (triple-buffered ctrl words; no host round trip per bucket).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <exception>

#include "gs_internal.h"
#include "gs_layout.h"

namespace gs {
namespace {

constexpr int TB = 256;

#include "gs_relax_kernel.h"
#include "gs_pull_kernel.h"
#include "gs_traffic.h"


struct SeedArgs {
  uint64_t* keys;
  const uint64_t* row;
  const uint32_t* col;
  const uint32_t* mesh;
  const uint32_t* pub;
  const uint8_t* stage;
  const uint32_t* tables;
  uint64_t* ctrl;      // min seeded key (push: the first bucket; pull: slot 2's min)
  uint32_t* chunkmin;  // pull path: [N][16] min pending key hi-word per 64-lane chunk (push path: nullptr)
  // list pull path: seeds appended to a list instead of the dense keys (k_lseed
  // files them into the candidate lists); the publishers' own lanes go to k_lpub
  uint64_t* skey;
  uint32_t* slane;     // (row << 11) | lane
  uint32_t* scnt;
  uint64_t* counters;
  uint64_t tmax;
  uint32_t L, FP, Fe, S, sb, tshift, flood;
  uint32_t u0, un;  // keys held for peers [u0, u0 + un) (the whole graph unless partitioned)
  uint32_t soff;    // batch slice (run_slices): its rows are soff + peer (list seeds and key sources)
  // churn: see RelaxArgs
  const uint32_t* ring_mesh;
  const uint64_t* ring_off;
  const uint64_t* q0;
  const uint64_t* r0;
  uint64_t hb_ns;
  uint32_t churn, ring_R, w64, horizon, N;
};

// publish_new_message (main.rs:101-143): self key at the publisher and the
// flood (or mesh) sends of every fragment through its uplink FIFO. Only
// targets inside [u0, u0 + un) are written; the publisher's owner counts R.
__global__ __launch_bounds__(TB) void k_seed(SeedArgs a) {
  __shared__ uint32_t live[MAX_DEG];  // churn: the connections online at t_pub, ascending
  __shared__ uint32_t wcnt[TB / 64];
  const uint32_t m = blockIdx.x, p = a.pub[m], sp = a.stage[p], S = a.S;
  const uint64_t ser = a.tables[S * S + sp];
  // churn: an offline publisher publishes nothing (the injector's POST finds no node)
  if (a.churn && ep_off(a, a.q0[m], p)) return;
  const bool own_pub = p - a.u0 < a.un;
  if (own_pub && threadIdx.x < a.Fe && !a.skey) a.keys[(size_t)(p - a.u0) * a.L + (size_t)m * a.FP + threadIdx.x] = (uint64_t)p;
  uint32_t deg;
  const uint32_t* tg;
  bool packed;
  if (a.flood) { deg = (uint32_t)(a.row[p + 1] - a.row[p]); tg = a.col + a.row[p]; packed = false; }
  else {
    tg = a.churn ? ep_mesh(a, a.q0[m], p) : a.mesh + (size_t)p * MESH_W;
    deg = 0;
    while (deg < MESH_W && tg[deg] != EMPTY) deg++;
    packed = true;
  }
  if (a.churn && a.flood) {  // compact the online connections in id order (deg <= MAX_DEG = TB)
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
  uint64_t nmin = INF64;
  uint32_t err = 0;
  const uint32_t total = a.Fe * deg;
  for (uint32_t i = threadIdx.x; i < total; i += TB) {
    const uint32_t f = i / deg, j = i % deg;
    const uint32_t w = packed ? (tg[j] & 0xFFFFFFu) : tg[j];
    const uint32_t sw = a.stage[w];
    const uint64_t sd = a.tables[S * S + S + sw];
    const uint64_t arr = ((uint64_t)f * deg + j + 1) * ser + a.tables[sp * S + sw] + (sd > ser ? sd - ser : 0);
    if (arr > a.tmax) err |= ERR_TIME;
    const uint64_t nk = (arr << a.tshift) | (1ull << a.sb) | (p + a.soff);
    if (w - a.u0 >= a.un) continue;
    if (a.churn && ev_lost(a, m, arr, w)) continue;
    if (a.skey) {  // one send per (target, fragment): no duplicates to reduce
      const uint32_t q = atomicAdd(a.scnt, 1u);
      a.skey[q] = nk;
      a.slane[q] = ((w - a.u0 + a.soff) << 11) | (m * a.FP + f);
      nmin = nk < nmin ? nk : nmin;
      continue;
    }
    atomicMin((unsigned long long*)&a.keys[(size_t)(w - a.u0) * a.L + (size_t)m * a.FP + f], (unsigned long long)nk);
    if (a.chunkmin)
      atomicMin(&a.chunkmin[(size_t)(w - a.u0) * PULL_CH + ((m * a.FP + f) >> 6)], (uint32_t)(nk >> 32));
    nmin = nk < nmin ? nk : nmin;
  }
  nmin = wave_min(nmin);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if ((threadIdx.x & 63) == 0) {
    if (nmin != INF64) atomicMin((unsigned long long*)a.ctrl, (unsigned long long)nmin);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
  if (threadIdx.x == 0 && own_pub) atomicAdd((unsigned long long*)&a.counters[C_R], (unsigned long long)total);
}

struct CompArgs {
  const uint64_t* keys;
  const uint32_t* pub;
  const uint64_t* tpub;
  uint64_t* tc;     // [N][B] peer-major, like the keys
  uint8_t* hops;    // [N][B]
  uint16_t* lat;    // [N][B] logged latency in ms (GS_WANT_LAT_MS), else nullptr
  uint64_t* counters;
  uint64_t* mstat;  // [B][MS_COLS] per-message reductions (k_complete / k_pct)
  uint32_t* hist;   // [B][GS_HIST_BINS] 100 ms latency bins (summary requested), else nullptr
  const uint32_t* pbin;  // k_pct: [B][2] the 100 ms bins holding p50 / p95
  uint32_t* fine;   // k_pct: [B][2][GS_HIST_MS] 1 ms counts inside those bins
  uint32_t N, B, F, FP, L, sb, tshift, collide, self_log, MT;
  uint32_t u0;  // global id of keys row 0
};

// per-message columns of mstat
enum : uint32_t { MS_TMAX = 0, MS_UNDEL = 1, MS_LOGGED = 2, MS_LSUM = 3, MS_LMAX = 4, MS_COLS = 8 };

// Lane -> (message, row offset) of the message-tiled completion kernels: a
// wave covers MT consecutive messages of 64/MT consecutive rows (MT = 64 for
// batches of >= 64 messages), so every load is a contiguous piece of a row
// and every lane keeps one message for the whole kernel (per-message
// reductions stay in registers). grid = (row chunks, message tiles).
struct MsgTile {
  uint32_t m, uoff, rstep;
  bool mv;
  __device__ MsgTile(uint32_t MT, uint32_t B) {
    const uint32_t lane = threadIdx.x & 63;
    m = blockIdx.y * MT + lane % MT;
    uoff = (threadIdx.x >> 6) * (64 / MT) + lane / MT;
    rstep = gridDim.x * (TB / 64) * (64 / MT);
    mv = m < B;
  }
};

// Sum per-lane values of the block's lanes that hold the same message and add
// them to the message's global counter (LDS staging, one atomic per message).
template <bool MAX>
__device__ __forceinline__ void msg_flush(uint64_t v, uint64_t* lds, uint32_t MT, uint32_t m0, uint32_t B,
                                          uint64_t* dst, uint32_t col) {
  __syncthreads();
  lds[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x < MT && m0 + threadIdx.x < B) {
    uint64_t t = 0;
    for (uint32_t i = threadIdx.x; i < TB; i += MT) t = MAX ? (lds[i] > t ? lds[i] : t) : t + lds[i];
    if (t) {
      unsigned long long* p = (unsigned long long*)&dst[(size_t)(m0 + threadIdx.x) * MS_COLS + col];
      if (MAX) atomicMax(p, (unsigned long long)t); else atomicAdd(p, (unsigned long long)t);
    }
  }
}

// Reassembly (main.rs:79-99): completion = max over fragments of the first
// arrival. keys[(u*B + m)*FP + f] -> tc[u*B + m] (peer-major; the transpose to
// the caller's message-major sink runs only when results are copied out).
// Per message it also reduces: the latest relative completion and the number
// of non-publishers that never complete (the lazy-gossip no-op proof of
// DESIGN.md §2.7), and with HIST the log lines, their latency sum / max and a
// 100 ms histogram (gs_msg_summary).
template <int FP, bool HIST>
__global__ __launch_bounds__(TB) void k_complete(CompArgs a) {
  __shared__ uint64_t red[TB];
  __shared__ uint32_t sh[HIST ? 64 * GS_HIST_BINS : 1];
  const MsgTile mt(a.MT, a.B);
  if (HIST)
    for (uint32_t i = threadIdx.x; i < 64 * GS_HIST_BINS; i += TB) sh[i] = 0;
  if (HIST) __syncthreads();
  uint64_t deliv = 0, lsum = 0, lmax = 0, tmax = 0, undel = 0, logged = 0, lgsum = 0, lgmax = 0;
  const uint32_t pm = mt.mv ? a.pub[mt.m] : EMPTY;
  const uint64_t tp = mt.mv ? a.tpub[mt.m] : 0;
  for (uint32_t u = blockIdx.x * (TB / 64) * (64 / a.MT) + mt.uoff; mt.mv && u < a.N; u += mt.rstep) {
    const size_t i = (size_t)u * a.B + mt.m;
    const uint64_t* kp = a.keys + i * FP;
    uint64_t mk = 0;
    bool ok = true;
#pragma unroll
    for (int f = 0; f < FP; f++) {  // padded fragments are INF: only f < F count
      const uint64_t x = f < (int)a.F ? kp[f] : 0;
      ok &= x != INF64;
      mk = x > mk ? x : mk;
    }
    uint64_t tc = INF64;
    uint8_t h = 0xFF;
    int64_t lms = -1;  // logged latency in ms
    if (u + a.u0 == pm) {  // its own key is set unless it published nothing (churn)
      if (kp[0] != INF64) {
        tc = tp;
        h = 0;
        if (a.self_log) lms = 0;
      }
    } else if (!a.collide && ok) {
      const uint64_t trel = mk >> a.tshift;
      tc = tp + trel;
      h = (uint8_t)((mk >> a.sb) & ((1u << HOP_BITS) - 1));
      const uint64_t ms = trel / 1000000ull;
      deliv++;
      lsum += ms;
      lmax = ms > lmax ? ms : lmax;
      tmax = trel > tmax ? trel : tmax;
      lms = (int64_t)ms;
    } else {
      undel++;
    }
    if (HIST && lms >= 0) {
      logged++;
      lgsum += (uint64_t)lms;
      lgmax = (uint64_t)lms > lgmax ? (uint64_t)lms : lgmax;
      const uint32_t bin = (uint64_t)lms / GS_HIST_MS < GS_HIST_BINS ? (uint32_t)((uint64_t)lms / GS_HIST_MS)
                                                                       : GS_HIST_BINS - 1;
      atomicAdd(&sh[((threadIdx.x & 63) % a.MT) * GS_HIST_BINS + bin], 1u);
    }
    if (a.tc) {  // results kept only when a sink will read them
      a.tc[i] = tc;
      a.hops[i] = h;
    }
    if (a.lat) {  // the log line's value (main.rs:93), GS_LAT_NONE where nothing is logged
      if (lms >= 0xFFFF) atomicOr((unsigned*)&a.counters[C_ERR], ERR_LAT16);
      a.lat[i] = lms < 0 ? (uint16_t)GS_LAT_NONE : (uint16_t)(lms < 0xFFFF ? lms : 0xFFFE);
    }
  }
  {
    const uint64_t d = wave_sum(deliv), s = wave_sum(lsum);
    uint64_t mx = lmax;
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t x = __shfl_xor(mx, off);
      mx = x > mx ? x : mx;
    }
    if ((threadIdx.x & 63) == 0 && d) {
      atomicAdd((unsigned long long*)&a.counters[C_DELIV], (unsigned long long)d);
      atomicAdd((unsigned long long*)&a.counters[C_LAT_SUM], (unsigned long long)s);
      atomicMax((unsigned long long*)&a.counters[C_LAT_MAX], (unsigned long long)mx);
    }
  }
  if (!a.mstat) return;  // block-uniform
  const uint32_t m0 = blockIdx.y * a.MT;
  msg_flush<true>(tmax, red, a.MT, m0, a.B, a.mstat, MS_TMAX);
  msg_flush<false>(undel, red, a.MT, m0, a.B, a.mstat, MS_UNDEL);
  if constexpr (HIST) {
    msg_flush<false>(logged, red, a.MT, m0, a.B, a.mstat, MS_LOGGED);
    msg_flush<false>(lgsum, red, a.MT, m0, a.B, a.mstat, MS_LSUM);
    msg_flush<true>(lgmax, red, a.MT, m0, a.B, a.mstat, MS_LMAX);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.MT * GS_HIST_BINS; i += TB) {
      const uint32_t mm = m0 + i / GS_HIST_BINS;
      if (sh[i] && mm < a.B) atomicAdd(&a.hist[(size_t)mm * GS_HIST_BINS + i % GS_HIST_BINS], sh[i]);
    }
  }
}

// Exact percentiles, second pass: 1 ms counts inside the two 100 ms bins that
// hold each message's p50 / p95 rank (the host picked them from the histogram).
__global__ __launch_bounds__(TB) void k_pct(CompArgs a) {
  __shared__ uint32_t sf[64 * 2 * GS_HIST_MS];
  const MsgTile mt(a.MT, a.B);
  for (uint32_t i = threadIdx.x; i < 64 * 2 * GS_HIST_MS; i += TB) sf[i] = 0;
  __syncthreads();
  const uint32_t pm = mt.mv ? a.pub[mt.m] : EMPTY;
  const uint64_t tp = mt.mv ? a.tpub[mt.m] : 0;
  const uint32_t b50 = mt.mv ? a.pbin[mt.m * 2] : ~0u, b95 = mt.mv ? a.pbin[mt.m * 2 + 1] : ~0u;
  const uint32_t ml = (threadIdx.x & 63) % a.MT;
  for (uint32_t u = blockIdx.x * (TB / 64) * (64 / a.MT) + mt.uoff; mt.mv && u < a.N; u += mt.rstep) {
    const uint64_t t = a.tc[(size_t)u * a.B + mt.m];
    if (t == INF64 || (u + a.u0 == pm && !a.self_log)) continue;
    const uint64_t ms = (t - tp) / 1000000ull;
    const uint32_t bin = ms / GS_HIST_MS < GS_HIST_BINS ? (uint32_t)(ms / GS_HIST_MS) : GS_HIST_BINS - 1;
    const uint32_t r = bin == GS_HIST_BINS - 1 ? GS_HIST_MS - 1 : (uint32_t)(ms % GS_HIST_MS);
    if (bin == b50) atomicAdd(&sf[(ml * 2) * GS_HIST_MS + r], 1u);
    if (bin == b95) atomicAdd(&sf[(ml * 2 + 1) * GS_HIST_MS + r], 1u);
  }
  __syncthreads();
  const uint32_t m0 = blockIdx.y * a.MT;
  for (uint32_t i = threadIdx.x; i < a.MT * 2 * GS_HIST_MS; i += TB) {
    const uint32_t mm = m0 + i / (2 * GS_HIST_MS);
    if (sf[i] && mm < a.B) atomicAdd(&a.fine[(size_t)mm * 2 * GS_HIST_MS + i % (2 * GS_HIST_MS)], sf[i]);
  }
}

// The logged latency [N][B] u16 -> [B][N] through a 64x64 LDS tile (the
// message-major GS_WANT_LAT_MS stream).
__global__ __launch_bounds__(TB) void k_transpose16(const uint16_t* __restrict__ lat, uint16_t* __restrict__ lat_t,
                                                    uint32_t N, uint32_t B) {
  __shared__ uint16_t s[64][66];
  const uint32_t u0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
  const uint32_t nu = min(64u, N - u0), nm = min(64u, B - m0);
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += TB) {
    const uint32_t pu = i >> 6, qm = i & 63;
    if (pu < nu && qm < nm) s[qm][pu] = lat[(size_t)(u0 + pu) * B + m0 + qm];
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += TB) {
    const uint32_t qm = i >> 6, pu = i & 63;
    if (pu < nu && qm < nm) lat_t[(size_t)(m0 + qm) * N + u0 + pu] = s[qm][pu];
  }
}

// [N][B] -> [B][N] through a 64x64 LDS tile, for the caller's message-major
// sink (include/gossipsim.h); not on the device-resident path.
__global__ __launch_bounds__(TB) void k_transpose(const uint64_t* __restrict__ tc, const uint8_t* __restrict__ hp,
                                                  uint64_t* __restrict__ tc_t, uint8_t* __restrict__ hp_t,
                                                  uint32_t N, uint32_t B) {
  __shared__ uint64_t s_tc[64][65];
  __shared__ uint8_t s_h[64][68];
  const uint32_t u0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
  const uint32_t nu = min(64u, N - u0), nm = min(64u, B - m0);
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += TB) {
    const uint32_t pu = i >> 6, qm = i & 63;
    if (pu < nu && qm < nm) {
      const size_t src = (size_t)(u0 + pu) * B + m0 + qm;
      s_tc[qm][pu] = tc[src];
      s_h[qm][pu] = hp[src];
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 64 * 64; i += TB) {
    const uint32_t qm = i >> 6, pu = i & 63;
    if (pu < nu && qm < nm) {
      const size_t dst = (size_t)(m0 + qm) * N + u0 + pu;
      tc_t[dst] = s_tc[qm][pu];
      hp_t[dst] = s_h[qm][pu];
    }
  }
}

#include "gs_lpull_kernel.h"
#include "gs_cpull.h"

uint32_t pow2_at_least(uint32_t x) { uint32_t p = 1; while (p < x) p <<= 1; return p; }

}  // namespace

// Chunks of one publish (PublishCommand.chunks, main.rs:65-71,163-168): the
// row's own count, 0 = FRAGMENTS of the node (env.rs:64-67).
static uint32_t frags_of(const Ctx& c, const gs_publish& p) { return p.frags ? p.frags : c.cfg.fragments; }

static void check_schedule(Ctx& c, const gs_publish* sched, uint64_t n_msgs) {
  for (uint64_t i = 0; i < n_msgs; i++) {
    if (sched[i].publisher >= c.cfg.peers) c.fail(GS_EINVAL, "publisher id out of range");
    if (sched[i].frags > MAX_FRAGS) c.fail(GS_EINVAL, "frags must be in 0..16 (0 = cfg.fragments)");
    if (frag_invalid(c.cfg.node, sched[i].msg_size, frags_of(c, sched[i])))  // the node's publish fails
      c.fail(GS_EINVAL, c.cfg.node == NODE_RUST ? "fragment payload shorter than the 8-byte tx_time stamp"
                        : c.cfg.node == NODE_GO ? "fragment too short for its chunk byte (payload[10])"
                                                : "fragment shorter than the 16-byte nim header + chunk byte");
  }
}

// Upload pub/tpub/link tables for messages [i0, i1) (equal msg_size) and
// compute the bucket width Delta = min latency + min serialisation.
// upload = false: only the host fields (a batch slice after the first: same shape and tables)
static Batch setup_batch(Ctx& c, const gs_publish* sched, uint64_t i0, uint64_t i1, bool upload = true) {
  Batch b;
  const uint32_t N = c.cfg.peers, S = c.S;
  b.F = frags_of(c, sched[i0]);
  b.FP = pow2_at_least(b.F);
  b.B = (uint32_t)(i1 - i0);
  b.L = b.B * b.FP;
  b.sb = bits_for(N);
  b.tshift = b.sb + HOP_BITS;
  b.tmax = b.tshift >= 64 ? 0 : (INF64 >> b.tshift);
  b.payload = frag_payload(c.cfg.node, sched[i0].msg_size, b.F);
  b.collide = frag_collide(c.cfg.node, sched[i0].msg_size, b.F);  // defect D8 (rust layout)
  b.Fe = b.collide ? 1 : b.F;
  hipStream_t s = c.stream;
  const uint64_t wire = gs_wire_bytes(b.payload, c.cfg.muxer, c.cfg.signed_msgs);
  std::vector<uint32_t> tab((size_t)S * S + 2 * S), pub(b.B);
  uint64_t min_lat = INF64, min_ser = INF64;
  // Delta from the link classes peers actually sit on (a Shadow graph may
  // carry nodes no peer uses, e.g. topogen's 1 ms injector hub)
  for (uint32_t x = 0; x < S; x++)
    for (uint32_t y = 0; y < S; y++) {
      if (c.lat_ns[(size_t)x * S + y] >= (1ull << 32)) c.fail(GS_ERANGE, "latency >= 2^32 ns");
      tab[(size_t)x * S + y] = (uint32_t)c.lat_ns[(size_t)x * S + y];
      if (c.stage_used[x] && c.stage_used[y]) min_lat = std::min<uint64_t>(min_lat, c.lat_ns[(size_t)x * S + y]);
    }
  for (uint32_t x = 0; x < S; x++) {
    const uint64_t up = ser_ns(wire, c.bw_up[x]), dn = ser_ns(wire, c.bw_dn[x]);
    if (up >= (1ull << 32) || dn >= (1ull << 32)) c.fail(GS_ERANGE, "serialisation >= 2^32 ns");
    tab[(size_t)S * S + x] = (uint32_t)up;
    tab[(size_t)S * S + S + x] = (uint32_t)dn;
    if (c.stage_used[x]) min_ser = std::min(min_ser, up);
  }
  b.delta = std::max<uint64_t>(1, min_lat + min_ser);
  for (uint32_t x = 0; x < S; x++) {
    if (!c.stage_used[x]) continue;
    b.ser_max = std::max<uint64_t>(b.ser_max, tab[(size_t)S * S + x]);
    for (uint32_t y = 0; y < S; y++) {
      if (!c.stage_used[y]) continue;
      const uint64_t up = tab[(size_t)S * S + x], dn = tab[(size_t)S * S + S + y];
      b.lat_adj_max = std::max<uint64_t>(b.lat_adj_max, tab[(size_t)x * S + y] + (dn > up ? dn - up : 0));
    }
  }
  b.lat_min = min_lat;
  for (uint32_t x = 0; x < S; x++)  // IHAVE x -> y, IWANT y -> x, answer x -> y (uplink of x, downlink of y)
    for (uint32_t y = 0; y < S; y++) {
      if (!c.stage_used[x] || !c.stage_used[y]) continue;
      const uint64_t up = tab[(size_t)S * S + x], dn = tab[(size_t)S * S + S + y];
      b.lat_max = std::max<uint64_t>(b.lat_max, tab[(size_t)x * S + y]);
      b.ans_max = std::max<uint64_t>(b.ans_max, (uint64_t)tab[(size_t)y * S + x] + up + tab[(size_t)x * S + y] +
                                                    (dn > up ? dn - up : 0));
    }
  b.tpub.resize(b.B);
  for (uint32_t q = 0; q < b.B; q++) { pub[q] = sched[i0 + q].publisher; b.tpub[q] = sched[i0 + q].t_pub_ns; }
  if (!upload) return b;
  c.d_pub.alloc(c.cfg.batch);
  c.d_tpub.alloc(c.cfg.batch);
  c.d_tables.alloc((size_t)S * S + 2 * S);
  GS_HIP(hipMemcpyAsync(c.d_pub.p, pub.data(), b.B * 4, hipMemcpyHostToDevice, s));
  GS_HIP(hipMemcpyAsync(c.d_tpub.p, b.tpub.data(), b.B * 8, hipMemcpyHostToDevice, s));
  GS_HIP(hipMemcpyAsync(c.d_tables.p, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, s));
  // the host vectors die here: make the copies complete first
  GS_HIP(hipStreamSynchronize(s));
  return b;
}

// churn fields shared by SeedArgs and RelaxArgs (the ring and per-message epochs of gs_run)
template <class A>
static void set_churn_args(Ctx& c, A& a) {
  if (!c.cfg.churn_ppm) return;
  a.churn = 1;
  a.ring_mesh = c.d_ring_mesh.p;
  a.ring_off = c.d_ring_off.p;
  a.q0 = c.d_q0.p;
  a.r0 = c.d_r0.p;
  a.hb_ns = c.cfg.heartbeat_ns;
  a.ring_R = c.ring_R;
  a.w64 = (c.cfg.peers + 63) / 64;
  a.horizon = c.cfg.churn_horizon;
  a.N = c.cfg.peers;
}

static void launch_seed(Ctx& c, const Batch& b, uint32_t u0, uint32_t un, uint64_t* seed_min = nullptr,
                        uint32_t* chunkmin = nullptr, bool to_list = false, const uint32_t* pub = nullptr,
                        uint32_t soff = 0) {
  SeedArgs sa{};
  if (to_list) {
    sa.skey = c.d_skey.p;
    sa.slane = c.d_slane.p;
    sa.scnt = c.d_scnt.p;
  }
  set_churn_args(c, sa);
  sa.keys = c.d_keys.p; sa.row = c.d_row.p; sa.col = c.d_col.p; sa.mesh = c.d_mesh.p;
  sa.pub = pub ? pub : c.d_pub.p; sa.stage = c.d_stage.p; sa.tables = c.d_tables.p;
  sa.soff = soff;
  sa.ctrl = seed_min ? seed_min : c.d_ctrl.p; sa.chunkmin = chunkmin;
  sa.counters = c.d_counters.p; sa.tmax = b.tmax; sa.L = b.L; sa.FP = b.FP; sa.Fe = b.Fe;
  sa.S = c.S; sa.sb = b.sb; sa.tshift = b.tshift; sa.flood = c.cfg.flood_publish;
  sa.u0 = u0; sa.un = un;
  k_seed<<<b.B, TB, 0, c.stream>>>(sa);
  GS_HIP(hipGetLastError());
}

// k_complete over the keys rows [0, un) (global ids u0 + row) into d_tc /
// d_hops; with `mstat` also the per-message reductions, with `hist` the
// 100 ms histograms of gs_msg_summary.
// store: write d_tc / d_hops (results go to a sink); without it only the
// counters and reductions are produced (a device-resident run).
// lat: also the logged latencies [un][B] u16 into d_lat (GS_WANT_LAT_MS).
// r0: the batch's rows start at row r0 of the key / log buffers (a batch slice, run_slices)
// pub / tpub: the batch's publishers and publish times (default d_pub / d_tpub)
static void run_complete(Ctx& c, const Batch& b, uint32_t u0, uint32_t un, bool mstat, bool hist,
                         bool store = true, bool lat = false, size_t r0 = 0, const uint32_t* pub = nullptr,
                         const uint64_t* tpub = nullptr, uint32_t nsl = 1) {
  if (!pub) pub = c.d_pub.p;
  if (!tpub) tpub = c.d_tpub.p;
  hipStream_t s = c.stream;
  if (lat) c.d_lat.alloc((size_t)un * c.cfg.batch);
  if (c.keys_log) {  // list pull path, results on the device: reduce the final logs
    // (nsl batch slices of un rows each, one launch: block row y = slice y, run_slices)
    if (hist || store || (lat && nsl > 1)) c.fail(GS_EINVAL, "internal: final logs need k_lfinal");
    LPullArgs la{};
    la.u0 = u0;  // rows [0, un) are global peers u0 + row (a part of gs_run_partitioned)
    la.keys = c.d_keys.p + r0 * b.L; la.flane = c.d_flane.p + r0 * b.L; la.st = c.d_lst.p + r0 * LP_SW;
    la.pub = pub;
    la.counters = c.d_counters.p; la.N = un; la.B = b.B; la.L = b.L; la.tshift = b.tshift;
    la.F = b.F; la.collide = b.collide ? 1u : 0u;
    la.self_log = c.cfg.self_log;
    if (mstat) {
      c.d_mstat.alloc((size_t)std::max(c.cfg.batch, nsl * b.B) * MS_COLS);
      GS_HIP(hipMemsetAsync(c.d_mstat.p, 0, (size_t)nsl * b.B * MS_COLS * 8, s));
    }
    const unsigned grid = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>(((uint64_t)un + LC_WAVES - 1) / LC_WAVES,
                              std::max<uint64_t>(1, (uint64_t)std::max(1, c.num_cus) / nsl)));
    k_lcomplete<<<dim3(grid, nsl), LC_WAVES * 64, 0, s>>>(la, mstat ? c.d_mstat.p : nullptr, lat ? c.d_lat.p : nullptr);
    GS_HIP(hipGetLastError());
    return;
  }
  CompArgs ca{};
  ca.keys = c.d_keys.p + r0 * b.L; ca.pub = pub; ca.tpub = tpub; ca.tc = store ? c.d_tc.p : nullptr;
  ca.hops = c.d_hops.p; ca.counters = c.d_counters.p; ca.N = un; ca.B = b.B; ca.F = b.F;
  ca.lat = lat ? c.d_lat.p : nullptr;
  ca.FP = b.FP; ca.L = b.L; ca.sb = b.sb; ca.tshift = b.tshift; ca.collide = b.collide ? 1 : 0;
  ca.u0 = u0;
  ca.self_log = c.cfg.self_log;
  ca.MT = std::min<uint32_t>(64, pow2_at_least(b.B));
  if (mstat || hist) {
    c.d_mstat.alloc((size_t)c.cfg.batch * MS_COLS);
    GS_HIP(hipMemsetAsync(c.d_mstat.p, 0, (size_t)b.B * MS_COLS * 8, s));
    ca.mstat = c.d_mstat.p;
  }
  if (hist) {
    c.d_hist.alloc((size_t)c.cfg.batch * GS_HIST_BINS);
    GS_HIP(hipMemsetAsync(c.d_hist.p, 0, (size_t)b.B * GS_HIST_BINS * 4, s));
    ca.hist = c.d_hist.p;
  }
  const uint32_t tiles = (b.B + ca.MT - 1) / ca.MT;
  const uint64_t rows_per_block = (TB / 64) * (64 / ca.MT);
  const uint64_t want = std::max<uint64_t>(1, (uint64_t)c.num_cus * 16 / tiles);
  // >= 16 rows per lane: every block ends in one atomic per message and column,
  // and a grid of thin blocks serialises on them (config #2, 10k rows x 2 message
  // tiles: 2048 blocks per tile, 595 us per batch, profiles/r04_v3)
  const uint64_t thick = (un + rows_per_block * 16 - 1) / (rows_per_block * 16);
  dim3 grid((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(thick, want)), tiles);
#define GS_COMPLETE(FPV)                                                      \
  if (hist) k_complete<FPV, true><<<grid, TB, 0, s>>>(ca);                    \
  else k_complete<FPV, false><<<grid, TB, 0, s>>>(ca);
  switch (b.FP) {
    case 1: GS_COMPLETE(1) break;
    case 2: GS_COMPLETE(2) break;
    case 4: GS_COMPLETE(4) break;
    case 8: GS_COMPLETE(8) break;
    default: GS_COMPLETE(16) break;
  }
#undef GS_COMPLETE
  GS_HIP(hipGetLastError());
}

// Nearest-rank percentile (rank ceil(q*n)) resolved from the 100 ms histogram:
// the bin holding the rank, and the rank left inside that bin.
static void pct_bin(const uint32_t* h, uint64_t n, uint32_t q100, uint32_t* bin, uint64_t* rest) {
  const uint64_t rank = (n * q100 + 99) / 100;
  uint64_t acc = 0;
  for (uint32_t k = 0; k < GS_HIST_BINS; k++) {
    if (acc + h[k] >= rank) { *bin = k; *rest = rank - acc; return; }
    acc += h[k];
  }
  *bin = GS_HIST_BINS - 1;
  *rest = 0;
}

// gs_msg_summary of the batch's messages (rows [0, un) of d_tc): counts and
// histograms from k_complete, exact p50 / p95 from k_pct's 1 ms counts inside
// the two bins (a rank in the open last bin is read from the message's column).
static void fill_summary(Ctx& c, const Batch& b, uint32_t u0, uint32_t un, gs_msg_summary* out) {
  hipStream_t s = c.stream;
  const uint32_t B = b.B;
  std::vector<uint64_t> ms((size_t)B * MS_COLS);
  std::vector<uint32_t> hist((size_t)B * GS_HIST_BINS), pbin((size_t)B * 2, ~0u), rest((size_t)B * 2, 0);
  GS_HIP(hipMemcpyAsync(ms.data(), c.d_mstat.p, ms.size() * 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipMemcpyAsync(hist.data(), c.d_hist.p, hist.size() * 4, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  std::vector<uint32_t> slow;  // messages whose p50 or p95 lies in the open last bin
  for (uint32_t q = 0; q < B; q++) {
    gs_msg_summary& r = out[q];
    memset(&r, 0, sizeof r);
    r.delivered = ms[(size_t)q * MS_COLS + MS_LOGGED];
    r.lat_sum_ms = ms[(size_t)q * MS_COLS + MS_LSUM];
    r.max_ms = (uint32_t)ms[(size_t)q * MS_COLS + MS_LMAX];
    memcpy(r.hist, &hist[(size_t)q * GS_HIST_BINS], sizeof r.hist);
    if (!r.delivered) continue;
    uint64_t rs[2];
    uint32_t bn[2];
    pct_bin(r.hist, r.delivered, 50, &bn[0], &rs[0]);
    pct_bin(r.hist, r.delivered, 95, &bn[1], &rs[1]);
    if (bn[0] == GS_HIST_BINS - 1 || bn[1] == GS_HIST_BINS - 1) { slow.push_back(q); continue; }
    for (int k = 0; k < 2; k++) { pbin[q * 2 + k] = bn[k]; rest[q * 2 + k] = (uint32_t)rs[k]; }
  }
  c.d_pbin.alloc((size_t)c.cfg.batch * 2);
  c.d_fine.alloc((size_t)c.cfg.batch * 2 * GS_HIST_MS);
  GS_HIP(hipMemcpyAsync(c.d_pbin.p, pbin.data(), pbin.size() * 4, hipMemcpyHostToDevice, s));
  GS_HIP(hipMemsetAsync(c.d_fine.p, 0, (size_t)B * 2 * GS_HIST_MS * 4, s));
  CompArgs ca{};
  ca.pub = c.d_pub.p; ca.tpub = c.d_tpub.p; ca.tc = c.d_tc.p; ca.N = un; ca.B = B; ca.u0 = u0;
  ca.self_log = c.cfg.self_log; ca.pbin = c.d_pbin.p; ca.fine = c.d_fine.p;
  ca.MT = std::min<uint32_t>(64, pow2_at_least(B));
  const uint32_t tiles = (B + ca.MT - 1) / ca.MT;
  const uint64_t rows_per_block = (TB / 64) * (64 / ca.MT);
  dim3 grid((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((un + rows_per_block - 1) / rows_per_block,
                                                               std::max<uint64_t>(1, (uint64_t)c.num_cus * 8 / tiles))),
            tiles);
  k_pct<<<grid, TB, 0, s>>>(ca);
  GS_HIP(hipGetLastError());
  std::vector<uint32_t> fine((size_t)B * 2 * GS_HIST_MS);
  GS_HIP(hipMemcpyAsync(fine.data(), c.d_fine.p, fine.size() * 4, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  for (uint32_t q = 0; q < B; q++) {
    if (pbin[q * 2] == ~0u) continue;
    for (int k = 0; k < 2; k++) {
      const uint32_t* f = &fine[((size_t)q * 2 + k) * GS_HIST_MS];
      uint64_t acc = 0;
      uint32_t r = 0;
      while (r < GS_HIST_MS - 1 && acc + f[r] < rest[q * 2 + k]) acc += f[r++];
      (k ? out[q].p95_ms : out[q].p50_ms) = pbin[q * 2 + k] * GS_HIST_MS + r;
    }
  }
  for (uint32_t q : slow) {  // rare (heavy churn tails): the column, sorted on the host
    std::vector<uint64_t> col(un);
    GS_HIP(hipMemcpy2DAsync(col.data(), 8, c.d_tc.p + q, (size_t)B * 8, 8, un, hipMemcpyDeviceToHost, s));
    std::vector<uint32_t> pub(1);
    GS_HIP(hipMemcpyAsync(pub.data(), c.d_pub.p + q, 4, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> v;
    for (uint32_t u = 0; u < un; u++)
      if (col[u] != INF64 && (u + u0 != pub[0] || c.cfg.self_log)) v.push_back((col[u] - b.tpub[q]) / 1000000ull);
    std::sort(v.begin(), v.end());
    const uint64_t n = v.size();
    out[q].p50_ms = (uint32_t)v[(n * 50 + 99) / 100 - 1];
    out[q].p95_ms = (uint32_t)v[(n * 95 + 99) / 100 - 1];
  }
}

// What a sink takes from a batch (include/gossipsim.h gs_result_sink): with
// on_block the want bits select t_complete / hops (neither = both), without
// it the non-NULL arrays do; on_lat takes the logged latency (GS_WANT_LAT_MS).
struct SinkWants {
  bool tc = false, h = false, lat = false, summary = false;
  bool rows() const { return tc || h; }
};
static SinkWants sink_wants(const gs_result_sink* sink) {
  SinkWants w;
  if (!sink) return w;
  if (sink->on_block) {
    uint32_t th = sink->want & (GS_WANT_T_COMPLETE | GS_WANT_HOPS);
    if (!th) th = GS_WANT_T_COMPLETE | GS_WANT_HOPS;
    w.tc = (th & GS_WANT_T_COMPLETE) != 0;
    w.h = (th & GS_WANT_HOPS) != 0;
  } else {
    w.tc = sink->t_complete_ns != nullptr;
    w.h = sink->hops != nullptr;
  }
  w.lat = sink->on_lat != nullptr;
  w.summary = sink->summary != nullptr;
  return w;
}

// Message-major rows of the batch — [B][un] in d_tc_t / d_hops_t, and the
// latency in d_lat_t — into a sink's rows [row0, row0 + B): its arrays (host
// memory; device memory when c.sink_dev, the message-sharded partitioned
// batches of gs_comm.hip), and the on_block / on_lat streams in blocks of
// block_msgs messages through two pinned staging halves (the copy of block k
// runs while the caller's callbacks consume block k - 1).
void deliver_rows(Ctx& c, uint32_t B, uint32_t un, const gs_result_sink* sink, uint64_t sink_row0) {
  hipStream_t s = c.stream;
  const SinkWants w = sink_wants(sink);
  if (!sink->on_block && w.rows()) {
    const hipMemcpyKind kind = c.sink_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (w.tc) GS_HIP(hipMemcpyAsync(sink->t_complete_ns + sink_row0 * un, c.d_tc_t.p, (size_t)B * un * 8, kind, s));
    if (w.h) GS_HIP(hipMemcpyAsync(sink->hops + sink_row0 * un, c.d_hops_t.p, (size_t)B * un, kind, s));
  }
  const bool st_rows = sink->on_block != nullptr, st_lat = w.lat;
  if (!st_rows && !st_lat) return;
  const uint32_t bm = std::max<uint32_t>(1, std::min<uint32_t>(sink->block_msgs ? sink->block_msgs : 64, B));
  const size_t cell = (st_rows && w.tc ? 8 : 0) + (st_lat ? 2 : 0) + (st_rows && w.h ? 1 : 0);
  const size_t half = ((size_t)bm * un * cell + 255) & ~(size_t)255;
  if (c.h_block_bytes < 2 * half) {
    if (c.h_block) GS_HIP(hipHostFree(c.h_block));
    c.h_block = nullptr;
    c.h_block_bytes = 0;
    GS_HIP(hipHostMalloc(&c.h_block, 2 * half, hipHostMallocDefault));
    c.h_block_bytes = 2 * half;
  }
  for (int k = 0; k < 2; k++)
    if (!c.blk_ev[k]) GS_HIP(hipEventCreateWithFlags(&c.blk_ev[k], hipEventDisableTiming));
  struct Part { uint64_t* tc; uint16_t* lat; uint8_t* h; };
  auto part = [&](int k) {  // [t_complete u64][latency u16][hops u8] of one half
    uint8_t* p = (uint8_t*)c.h_block + (size_t)k * half;
    Part q{nullptr, nullptr, nullptr};
    if (st_rows && w.tc) { q.tc = (uint64_t*)p; p += (size_t)bm * un * 8; }
    if (st_lat) { q.lat = (uint16_t*)p; p += (size_t)bm * un * 2; }
    if (st_rows && w.h) q.h = p;
    return q;
  };
  auto hand_over = [&](int k, uint32_t q0, uint32_t n) {
    GS_HIP(hipEventSynchronize(c.blk_ev[k]));
    const Part q = part(k);
    if (st_rows) sink->on_block(sink->user, sink_row0 + q0, n, un, q.tc, q.h);
    if (st_lat) sink->on_lat(sink->user, sink_row0 + q0, n, un, q.lat);
  };
  int prev = -1;
  uint32_t pq0 = 0, pn = 0;
  for (uint32_t q0 = 0, k = 0; q0 < B; q0 += bm, k ^= 1) {
    const uint32_t n = std::min(bm, B - q0);
    const Part q = part((int)k);
    if (q.tc) GS_HIP(hipMemcpyAsync(q.tc, c.d_tc_t.p + (size_t)q0 * un, (size_t)n * un * 8, hipMemcpyDeviceToHost, s));
    if (q.lat)
      GS_HIP(hipMemcpyAsync(q.lat, c.d_lat_t.p + (size_t)q0 * un, (size_t)n * un * 2, hipMemcpyDeviceToHost, s));
    if (q.h) GS_HIP(hipMemcpyAsync(q.h, c.d_hops_t.p + (size_t)q0 * un, (size_t)n * un, hipMemcpyDeviceToHost, s));
    GS_HIP(hipEventRecord(c.blk_ev[k], s));
    if (prev >= 0) hand_over(prev, pq0, pn);  // block k - 1 while block k is copied
    prev = (int)k;
    pq0 = q0;
    pn = n;
  }
  hand_over(prev, pq0, pn);
}

// The pending latency-only delivery of the previous batch (deliver_lat_async):
// wait for its copy, check the error word it carried (a latency the u16 stream
// cannot hold fails the run before any of that batch's lines are handed out),
// then its callbacks block by block.
static void lat_flush(Ctx& c) {
  Ctx::LatPending& p = c.lat_pend;
  if (!p.on) return;
  p.on = false;
  GS_HIP(hipEventSynchronize(c.lat_done[p.par]));
  if (c.h_laterr[p.par] & ERR_LAT16)
    c.fail(GS_ERANGE, "a logged latency of 65535 ms or more does not fit the u16 stream (GS_WANT_LAT_MS)");
  for (uint32_t q0 = 0; q0 < p.B; q0 += p.bm) {
    const uint32_t n = std::min(p.bm, p.B - q0);
    p.sink->on_lat(p.sink->user, p.row0 + q0, n, p.un, c.h_lat[p.par] + (size_t)q0 * p.un);
  }
}

// A latency-only sink inside gs_run (on_lat, no rows, no summary): the batch's
// transposed u16 latencies leave on the copy stream into a whole-batch pinned
// buffer of this batch's parity while the next batch's passes run; the
// previous batch's callbacks run now (its copy had this batch's passes to
// finish), this batch's at the next delivery or at the end of the run.
static void deliver_lat_async(Ctx& c, const Batch& b, uint32_t un, const gs_result_sink* sink, uint64_t sink_row0) {
  hipStream_t s = c.stream;
  const uint32_t par = c.lat_par;
  c.lat_par ^= 1u;
  DevBuf<uint16_t>& lt = par ? c.d_lat_t2 : c.d_lat_t;
  lt.alloc((size_t)un * c.cfg.batch);
  dim3 tg((un + 63) / 64, (b.B + 63) / 64);
  k_transpose16<<<tg, TB, 0, s>>>(c.d_lat.p, lt.p, un, b.B);
  GS_HIP(hipGetLastError());
  const size_t bytes = (size_t)b.B * un * 2;
  if (c.h_lat_bytes[par] < bytes) {
    if (c.h_lat[par]) GS_HIP(hipHostFree(c.h_lat[par]));
    c.h_lat[par] = nullptr;
    c.h_lat_bytes[par] = 0;
    GS_HIP(hipHostMalloc((void**)&c.h_lat[par], bytes, hipHostMallocDefault));
    c.h_lat_bytes[par] = bytes;
  }
  if (!c.h_laterr) GS_HIP(hipHostMalloc((void**)&c.h_laterr, 2 * 8, hipHostMallocDefault));
  if (!c.copy) GS_HIP(hipStreamCreateWithFlags(&c.copy, hipStreamNonBlocking));
  for (int k = 0; k < 2; k++) {
    if (!c.lat_src[k]) GS_HIP(hipEventCreateWithFlags(&c.lat_src[k], hipEventDisableTiming));
    if (!c.lat_done[k]) GS_HIP(hipEventCreateWithFlags(&c.lat_done[k], hipEventDisableTiming));
  }
  GS_HIP(hipEventRecord(c.lat_src[par], s));
  GS_HIP(hipStreamWaitEvent(c.copy, c.lat_src[par], 0));
  GS_HIP(hipMemcpyAsync(c.h_lat[par], lt.p, bytes, hipMemcpyDeviceToHost, c.copy));
  GS_HIP(hipMemcpyAsync(c.h_laterr + par, c.d_counters.p + C_ERR, 8, hipMemcpyDeviceToHost, c.copy));
  GS_HIP(hipEventRecord(c.lat_done[par], c.copy));
  lat_flush(c);  // the previous batch, in message order
  Ctx::LatPending& p = c.lat_pend;
  p.on = true;
  p.par = par;
  p.B = b.B;
  p.un = un;
  p.bm = std::max<uint32_t>(1, std::min<uint32_t>(sink->block_msgs ? sink->block_msgs : 64, b.B));
  p.row0 = sink_row0;
  p.sink = sink;
}

// Results of a completed batch (peer-major d_tc / d_hops / d_lat of peers
// [u0, u0 + un)) into the sink: transposed to message-major, copied out,
// summaries.
static void deliver(Ctx& c, const Batch& b, uint32_t u0, uint32_t un, const gs_result_sink* sink,
                    uint64_t sink_row0) {
  if (!sink) return;
  hipStream_t s = c.stream;
  const SinkWants w = sink_wants(sink);
  if (c.lat_async && w.lat && !w.rows() && !w.summary && sink->on_lat) {
    deliver_lat_async(c, b, un, sink, sink_row0);
    return;
  }
  lat_flush(c);  // (a pending batch is delivered before this one)
  if (w.rows()) {
    c.d_tc_t.alloc((size_t)un * c.cfg.batch);
    c.d_hops_t.alloc((size_t)un * c.cfg.batch);
    dim3 tg((un + 63) / 64, (b.B + 63) / 64);
    k_transpose<<<tg, TB, 0, s>>>(c.d_tc.p, c.d_hops.p, c.d_tc_t.p, c.d_hops_t.p, un, b.B);
    GS_HIP(hipGetLastError());
  }
  if (w.lat) {
    c.d_lat_t.alloc((size_t)un * c.cfg.batch);
    dim3 tg((un + 63) / 64, (b.B + 63) / 64);
    k_transpose16<<<tg, TB, 0, s>>>(c.d_lat.p, c.d_lat_t.p, un, b.B);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_counters.p + C_ERR, 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    if (c.h_pinned[0] & ERR_LAT16) c.fail(GS_ERANGE, "a logged latency of 65535 ms or more does not fit the u16 "
                                                     "stream (GS_WANT_LAT_MS)");
  }
  if (w.rows() || w.lat) deliver_rows(c, b.B, un, sink, sink_row0);
  if (w.summary) fill_summary(c, b, u0, un, sink->summary + sink_row0);
}

// Completion + delivery of a finished batch.
static void launch_complete(Ctx& c, const Batch& b, uint32_t u0, uint32_t un, const gs_result_sink* sink,
                            uint64_t sink_row0, size_t r0 = 0) {
  const bool hist = sink && sink->summary;
  const SinkWants w = sink_wants(sink);
  run_complete(c, b, u0, un, hist, hist, w.rows() || w.summary, w.lat, r0);  // k_pct reads d_tc
  deliver(c, b, u0, un, sink, sink_row0);
}

// The batch's fields of RelaxArgs shared by the bucket launches and the
// traffic passes: keys, graph, link tables, churn ring, and with `gossip` the
// lazy-gossip inputs (heartbeats per message, CSR, IHAVE target ring).
// Bucket launches one churn + gossip batch may take (the holder list's
// per-launch marks, RelaxArgs::hl_lo / hl_end).
constexpr uint32_t HL_LAUNCHES = 1u << 16;

static RelaxArgs relax_args(Ctx& c, const Batch& b, bool gossip) {
  RelaxArgs ra{};
  set_churn_args(c, ra);
  ra.keys = c.d_keys.p; ra.mesh = c.d_mesh.p; ra.pub = c.d_pub.p;
  ra.stage = c.d_stage.p; ra.tables = c.d_tables.p;
  ra.total = (uint64_t)c.cfg.peers * b.L; ra.tmax = b.tmax;
  ra.N = c.cfg.peers; ra.B = b.B; ra.F = b.F; ra.L = b.L; ra.S = c.S; ra.sb = b.sb; ra.tshift = b.tshift;
  ra.idw = (c.cfg.idontwant && b.payload >= c.cfg.idontwant) ? 1 : 0;
  ra.row = c.d_row.p;
  ra.col = c.d_col.p;
  if (gossip) {
    ra.rel0 = c.d_rel0.p;
    ra.habs0 = c.d_habs0.p;
    ra.hb_ns = c.cfg.heartbeat_ns;
    ra.seed = c.cfg.seed;
    ra.gossip = 1;
    if (c.cfg.churn_ppm) {
      ra.ring_in = c.d_ring_in.p;
      // heartbeats of a message from index gs_switch on are decided
      // sender-centric (exact for any value; GS_GOSSIP_SWITCH for tests / A/B)
      const char* gsw = getenv("GS_GOSSIP_SWITCH");
      ra.gs_switch = gsw && *gsw ? (uint32_t)atoi(gsw) : 4u;
      // the per-lane first gossip heartbeat (RelaxArgs::hwin) saturates at 254:
      // the receiver-centric test k < j0 needs gs_switch <= 254 to stay exact
      // (a larger switch puts every heartbeat of a 16-epoch lifetime on that side anyway)
      if (ra.gs_switch > 254) ra.gs_switch = 254;
    }
    ra.hist = c.cfg.history_gossip;
    ra.d_lazy = c.cfg.d_lazy;
    ra.gf_milli = c.cfg.gossip_factor_milli;
  }
  return ra;
}

// Per-peer traffic of the batch just finished (keys final, before the next
// reset; gs_traffic.h).
static void launch_traffic(Ctx& c, const Batch& b) {
  const bool gossip = c.cfg.lazy_gossip != 0;
  const RelaxArgs ra = relax_args(c, b, gossip);
  TrafficArgs ta{};
  ta.traffic = c.d_traffic.p;
  ta.W = gs_wire_bytes(b.payload, c.cfg.muxer, c.cfg.signed_msgs);
  gs_wire_packets(b.payload, c.cfg.muxer, c.cfg.signed_msgs, &ta.pk, &ta.hdr);
  gs_control_packets(GS_CTRL_IHAVE, c.cfg.node, c.cfg.muxer, &ta.ihw, &ta.ihpk, &ta.ihhd);
  gs_control_packets(GS_CTRL_IWANT, c.cfg.node, c.cfg.muxer, &ta.iww, &ta.iwpk, &ta.iwhd);
  gs_control_packets(GS_CTRL_ACK, c.cfg.node, c.cfg.muxer, &ta.ack, nullptr, nullptr);
  ta.Fe = b.Fe;
  ta.flood = c.cfg.flood_publish;
  ta.collide = b.collide ? 1 : 0;
  hipStream_t s = c.stream;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((ra.total + TB - 1) / TB,
                                                                           (uint64_t)c.num_cus * 8));
  k_traffic_pub<<<b.B, TB, 0, s>>>(ra, ta);
#define GS_TRAFFIC(FPV)                                                    \
  k_traffic_fwd<FPV><<<grid, TB, 0, s>>>(ra, ta);                          \
  if (gossip && c.cfg.history_gossip) k_traffic_gossip<FPV><<<grid, TB, 0, s>>>(ra, ta);
  switch (b.FP) {
    case 1: GS_TRAFFIC(1) break;
    case 2: GS_TRAFFIC(2) break;
    case 4: GS_TRAFFIC(4) break;
    case 8: GS_TRAFFIC(8) break;
    default: GS_TRAFFIC(16) break;
  }
#undef GS_TRAFFIC
  GS_HIP(hipGetLastError());
}

// Read the device counters into ctx->stats (and raise the device error word).
static void collect_stats(Ctx& c) {
  hipStream_t s = c.stream;
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  const uint64_t* h = c.h_pinned;
  if (h[C_ERR] & ERR_TIME) c.fail(GS_ERANGE, "relative arrival time overflowed the key's time field");
  if (h[C_ERR] & ERR_HOPS) c.fail(GS_ERANGE, "hop count overflowed the key's 6-bit hop field");
  c.stats.frag_deliveries = h[C_FD];
  c.stats.relaxations = h[C_R] + h[C_R_FWD] + h[C_GOSSIP];
  c.stats.gossip_iwant = h[C_GOSSIP];
  c.stats.deliveries = h[C_DELIV];
  c.stats.latency_sum_ms = h[C_LAT_SUM];
  c.stats.latency_max_ms = h[C_LAT_MAX];
  c.stats.buckets = h[C_BUCKETS];
  c.stats.bytes_alg = 16 * h[C_FD] + 12 * c.stats.relaxations + 8 * h[C_DELIV];
  c.stats.relax_bytes_alg = 16 * h[C_FD] + 12 * h[C_R_FWD];
  c.stats.pushes = h[C_PUSH];
  static const bool dbg = getenv("GS_DEBUG_COUNTS") != nullptr;
  if (dbg)
    fprintf(stderr, "[gs] buckets %llu gossip-listed lanes %llu tiles scanned %llu (for gossip only %llu) iwant %llu\n",
            (unsigned long long)h[C_BUCKETS], (unsigned long long)h[C_GLISTED], (unsigned long long)h[C_TSCANNED],
            (unsigned long long)h[C_TSCANNED_G], (unsigned long long)h[C_GOSSIP]);
}


// One batch on the owner-computes path (gs_pull_kernel.h): seed, then passes in
// chunks of 8 until a pass decides DONE (one host read of the ctrl slots per chunk).
template <class EvFn>
static void run_pull_batch(Ctx& c, const Batch& b, EvFn& ev, size_t& n_ev, int dev_cus) {
  const uint32_t N = c.cfg.peers, L = b.L;
  hipStream_t s = c.stream;
  const size_t NL = (size_t)N * L;
  c.d_chunkmin.alloc((size_t)N * PULL_CH);
  c.d_lrec.alloc(2 * NL);
  c.d_lcnt.alloc(2 * (size_t)N);
  c.d_pctrl.alloc(12);
  if (!c.rpos_valid) {
    c.d_rpos.alloc((size_t)N * MESH_W);
    GS_HIP(hipMemsetAsync(c.d_counters.p + C_ERR, 0, 8, s));
    k_rpos<<<(unsigned)(((uint64_t)N * MESH_W + TB - 1) / TB), TB, 0, s>>>(c.d_mesh.p, c.d_rpos.p, N, c.d_counters.p);
    GS_HIP(hipGetLastError());
    if (read_counter(c, C_ERR) & ERR_MESH) c.fail(GS_ERANGE, "mesh is not symmetric");
    c.rpos_valid = true;
  }
  GS_HIP(hipMemsetAsync(c.d_chunkmin.p, 0xFF, (size_t)N * PULL_CH * 4, s));
  GS_HIP(hipMemsetAsync(c.d_pctrl.p, 0, 12 * 8, s));  // every slot {lo 0, DONE, 0 records, min INF}
  for (int q = 0; q < 3; q++) GS_HIP(hipMemsetAsync(c.d_pctrl.p + q * 4 + 3, 0xFF, 8, s));
  launch_seed(c, b, 0, N, c.d_pctrl.p + 2 * 4 + 3, c.d_chunkmin.p);
  PullArgs pa{};
  pa.keys = c.d_keys.p; pa.busy = c.d_busy.p; pa.chunkmin = c.d_chunkmin.p;
  pa.lrec = c.d_lrec.p; pa.lcnt = c.d_lcnt.p; pa.rpos = c.d_rpos.p;
  pa.mesh = c.d_mesh.p; pa.pub = c.d_pub.p; pa.stage = c.d_stage.p; pa.tables = c.d_tables.p;
  // windows on the key's high-word grain (gs_pull_kernel.h); the caller checked delta >= grain
  const uint64_t grain = pull_grain(b.tshift);
  pa.ctrl = c.d_pctrl.p; pa.counters = c.d_counters.p; pa.delta = b.delta / grain * grain;
  pa.tmax = b.tmax - grain;
  pa.N = N; pa.B = b.B; pa.L = L; pa.S = c.S; pa.sb = b.sb; pa.tshift = b.tshift;
  // 33 KB of LDS per block: 4 blocks (16 waves, 16 rows in flight) per CU
  const unsigned grid = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>(((uint64_t)N + PULL_WAVES - 1) / PULL_WAVES, (uint64_t)dev_cus * 4));
  uint32_t pass = 0;
  for (;;) {
    for (uint32_t q = 0; q < 8; q++) {
      pa.pass = pass++;
      if (c.timing) {  // (start, mid, end): the whole pass is frontier time
        GS_HIP(hipEventRecord(ev(n_ev), s));
        GS_HIP(hipEventRecord(ev(n_ev + 1), s));
        pull_dispatch(b.FP, pa, grid, s);
        GS_HIP(hipEventRecord(ev(n_ev + 2), s));
        n_ev += 3;
      } else {
        pull_dispatch(b.FP, pa, grid, s);
      }
    }
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_pctrl.p, 12 * 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    if (c.h_pinned[((pass - 1) % 3) * 4 + 1] == PM_DONE) break;
  }
  c.stats.relax_launches += pass;
}

// Largest arrival offset of a forward relative to its uplink start: latency +
// downlink excess + MESH_W serialisations (the receiver's FIFO position).
// Largest arrival after a lane's final time: the uplink FIFO behind the other
// FP - 1 fragments' sends, then MESH_W serialisations, the adjusted latency.
static uint64_t lpull_rmax(const Batch& b) {
  return b.lat_adj_max + (uint64_t)MESH_W * b.ser_max * b.FP;
}

// Entries per candidate list: at least 256, so that rows of few lanes (small
// batches) still hold several passes' appends of the same lanes.
static uint32_t lpull_stride(const Batch& b) { return std::max<uint32_t>(b.L, 256); }

// Ring size K of the list pull path (gs_lpull_kernel.h) for this batch, or 0
// when it cannot take the batch (then k_pull runs). A candidate made from a
// record of window b arrives before b*D + D (start inside the window) + the
// fragment FIFO + the largest link latency + MESH_W serialisations, so its
// destination is at most K - 1 windows after the emitted one; the entry
// packs (t - window start) | hops | src | lane into 64 bits; the seed list
// packs row << 11 | lane (N < 2^21); the lists must fit the device memory left.
// rows: the pass's rows (batch slices: slices x peers)
static uint32_t lpull_ring(Ctx& c, const Batch& b, uint64_t delta, uint32_t* lb, bool gos = false, bool chn = false,
                           uint32_t rows = 0) {
  if (!c.mesh_dmax) {  // widest mesh row, once per mesh
    std::vector<uint32_t> m((size_t)c.cfg.peers * MESH_W);
    GS_HIP(hipMemcpyAsync(m.data(), c.d_mesh.p, m.size() * 4, hipMemcpyDeviceToHost, c.stream));
    GS_HIP(hipStreamSynchronize(c.stream));
    uint32_t dmax = 1;
    for (size_t u = 0; u < c.cfg.peers; u++) {
      uint32_t d = 0;
      while (d < MESH_W && m[u * MESH_W + d] != EMPTY) d++;
      dmax = std::max(dmax, d);
    }
    c.mesh_dmax = dmax;
  }
  const uint32_t N = rows ? rows : c.cfg.peers;
  if (b.tshift >= 32 || b.L > PULL_LMAX || delta < 2 || N >= (1u << 21)) return 0;  // seed list: row << 11
  // a fragment waits behind at most the other FP - 1 fragments' sends to the
  // row's mesh peers (c.mesh_dmax, the widest mesh row)
  // (churn: each epoch has its own mesh, bounded by the ELL width)
  const uint64_t dm = chn ? MESH_W : c.mesh_dmax ? c.mesh_dmax : MESH_W;
  const uint64_t fifo = (uint64_t)(b.FP - 1) * dm * b.ser_max;
  const uint64_t span = delta + fifo + b.lat_adj_max + dm * b.ser_max;
  // k_seed's first sends (every fragment to every mesh peer, or to every
  // connection with flood publish) land in windows 1 .. K of source window 0
  const uint64_t sdeg = c.cfg.flood_publish ? std::max<uint64_t>(c.max_degree, 1) : dm;
  const uint64_t seed_span = (uint64_t)b.FP * sdeg * b.ser_max + b.lat_adj_max;
  uint64_t K = std::max(span / delta + 2, seed_span / delta + 1);
  // GOS: an IWANT answer is appended from the window of its IHAVE's arrival
  if (gos) K = std::max<uint64_t>(K, (delta + b.ans_max) / delta + 2);
  if (K > LP_KMAX) return 0;
  // test knob: a ring smaller than the bound forces ERR_RING and the k_pull re-run
  const char* kf = getenv("GS_LPULL_K");  // per batch: tests set it between runs
  if (kf && *kf) K = std::min<uint64_t>(K, (uint64_t)std::max(2, atoi(kf)));
  uint32_t tb = 0;
  while ((1ull << tb) < delta) tb++;
  *lb = bits_for(b.L);
  if (tb + b.tshift + *lb > 63) return 0;  // bit 63 of an entry marks a pushed IHAVE (gs_lpull_kernel.h)
  uint64_t need = (uint64_t)K * N * lpull_stride(b) * 8 + (uint64_t)N * b.L * 2 + (uint64_t)N * (LP_SW + LP_FW) * 4;
  uint64_t have = (uint64_t)c.d_lblk.n * 8 + (uint64_t)c.d_flane.n * 2 + (uint64_t)(c.d_lst.n + c.d_lfin.n) * 4;
  if (gos) {  // sender planes and entries
    need += (uint64_t)N * b.L * 8 + (uint64_t)N * LP_FW * 4;
    have += (uint64_t)c.d_gse.n * 8 + (uint64_t)c.d_gpl.n * 4;
  }
  if (need > have) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || need - have + (4ull << 30) > fr) return 0;
  }
  return (uint32_t)K;
}

// One batch on the list pull path: k_seed appends the first sends to a seed
// list (no dense key table to reset), k_lseed files them into the candidate
// lists, k_lpub logs the publishers' own lanes, then passes in chunks of 8 as
// on the k_pull path; completion reads the final logs (k_lcomplete) unless a
// caller needs dense rows (k_lfinal).
// Returns false (counters restored) when a list overflowed: the caller re-runs
// the batch on k_pull.
// Lazy gossip inside the passes (GOS): the batch's heartbeats relative to
// every t_pub (lockstep) and the IHAVE travel bounds.
struct GosRun {
  uint64_t rel0, hb;
};
// Churn on the list pass (gs_cpull.h): the batch's first epoch and epoch count,
// the common offset of its publishes into their epochs, heartbeat 0's relative epoch.
struct ChnRun {
  uint64_t E0, r0;
  uint32_t cE, ghoff;
  uint32_t par;  // the table set (Ctx::ct) chn_begin filled for the batch
};

// Batch slices (run_slices): S batches of the same shape as one pass over S
// copies of the graph, slice j's rows j * N1 + peer; the copies' mesh rows,
// reverse positions and stages (d_smesh, d_srpos, d_sstage), the publishers
// as slice rows (spub, k_lpull / k_lpub) and as peers (lpub, k_seed).
struct Slices {
  uint32_t S, N1;
  const uint32_t* spub;
  const uint32_t* lpub;
};

template <class EvFn>
static bool run_lpull_batch(Ctx& c, const Batch& b, uint32_t K, uint32_t lb, EvFn& ev, size_t& n_ev, int dev_cus,
                            bool dense, bool idw, const GosRun* gos = nullptr, const ChnRun* chn = nullptr,
                            const Slices* sl = nullptr) {
  const uint32_t N0 = c.cfg.peers, L = b.L;
  const uint32_t N = sl ? sl->S * N0 : N0;  // the pass's rows
  hipStream_t s = c.stream;
  const size_t NL = (size_t)N * L;
  c.d_lrec.alloc((chn ? 4 : 2) * NL);  // churn records are 16 B
  c.d_lcnt.alloc(2 * (size_t)N);
  c.d_pctrl.alloc(12);
  const uint32_t ls = lpull_stride(b);
  c.d_lblk.alloc((size_t)K * N * ls);
  c.d_lst.alloc((size_t)N * LP_SW);
  c.d_lfin.alloc((size_t)N * LP_FW);
  c.d_flane.alloc(NL);
  if (!c.rpos_valid) {
    c.d_rpos.alloc((size_t)N0 * MESH_W);
    GS_HIP(hipMemsetAsync(c.d_counters.p + C_ERR, 0, 8, s));
    k_rpos<<<(unsigned)(((uint64_t)N0 * MESH_W + TB - 1) / TB), TB, 0, s>>>(c.d_mesh.p, c.d_rpos.p, N0, c.d_counters.p);
    GS_HIP(hipGetLastError());
    if (read_counter(c, C_ERR) & ERR_MESH) c.fail(GS_ERANGE, "mesh is not symmetric");
    c.rpos_valid = true;
  }
  if (sl) {  // the graph copies of the slices (rebuilt per group: a few MB)
    c.d_smesh.alloc((size_t)N * MESH_W);
    c.d_srpos.alloc((size_t)N * MESH_W);
    c.d_sstage.alloc(N);
    k_srep<<<(unsigned)(((uint64_t)N * MESH_W + TB - 1) / TB), TB, 0, s>>>(
        N0, sl->S, c.d_mesh.p, c.d_rpos.p, c.d_stage.p, c.d_smesh.p, c.d_srpos.p, c.d_sstage.p);
    GS_HIP(hipGetLastError());
  }
  GS_HIP(hipMemsetAsync(c.d_lst.p, 0, (size_t)N * LP_SW * 4, s));
  GS_HIP(hipMemsetAsync(c.d_lfin.p, 0, (size_t)N * LP_FW * 4, s));
  GS_HIP(hipMemsetAsync(c.d_pctrl.p, 0, 12 * 8, s));  // every slot {lo 0, DONE, 0 records, min INF}
  for (int q = 0; q < 3; q++) GS_HIP(hipMemsetAsync(c.d_pctrl.p + q * 4 + 3, 0xFF, 8, s));
  c.d_lp_save.alloc(C_COUNT);
  GS_HIP(hipMemcpyAsync(c.d_lp_save.p, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
  // seeds: one entry per (target, fragment) of every publish (flood: every connection)
  const uint64_t scap = (uint64_t)(sl ? sl->S : 1) * b.B * b.Fe * std::max<uint64_t>(c.max_degree, MESH_W);
  c.d_skey.alloc(scap);
  c.d_slane.alloc(scap);
  c.d_scnt.alloc(1);
  GS_HIP(hipMemsetAsync(c.d_scnt.p, 0, 4, s));
  if (sl)
    for (uint32_t j = 0; j < sl->S; j++)
      launch_seed(c, b, 0, N0, c.d_pctrl.p + 2 * 4 + 3, nullptr, true, sl->lpub + (size_t)j * b.B, j * N0);
  else
    launch_seed(c, b, 0, N, c.d_pctrl.p + 2 * 4 + 3, nullptr, true);
  LPullArgs la{};
  la.keys = c.d_keys.p; la.flane = c.d_flane.p; la.busy = c.d_busy.p; la.blk = c.d_lblk.p;
  la.st = c.d_lst.p; la.fin = c.d_lfin.p;
  la.lrec = c.d_lrec.p; la.lcnt = c.d_lcnt.p; la.rpos = c.d_rpos.p;
  la.mesh = c.d_mesh.p; la.pub = c.d_pub.p; la.stage = c.d_stage.p; la.tables = c.d_tables.p;
  if (sl) {
    la.mesh = c.d_smesh.p;
    la.rpos = c.d_srpos.p;
    la.stage = c.d_sstage.p;
    la.pub = sl->spub;
    la.rN = N0;
  }
  const uint64_t grain = pull_grain(b.tshift);
  la.ctrl = c.d_pctrl.p; la.counters = c.d_counters.p; la.delta = b.delta / grain * grain;
  la.tmax = b.tmax - grain;
  la.N = N; la.B = b.B; la.L = L; la.S = c.S; la.sb = b.sb; la.tshift = b.tshift;
  la.K = K; la.lb = lb; la.dG = (uint32_t)(la.delta / grain);
  la.idw = idw ? 1u : 0u;
  la.rmax = lpull_rmax(b);
  la.ghk = ~0u;
  la.gsw = ~0u;  // (frozen mesh: every heartbeat's IHAVEs are decided by the receivers)
  if (chn) {  // churn (gs_cpull.h): the tables k_cprep built for this batch
    la.ccol = c.d_ccol.p;
    la.cpos = c.d_cpos.p;
    const Ctx::ChnTables& t = c.ct[chn->par & 1];
    la.cmm = t.cmm.p;
    la.cgt = t.cgt.p;
    la.coff = t.coff.p;
    la.cq = t.cq.p;
    la.pubok = t.pubok.p;
    la.calive = t.calive.p;
    c.d_luni.alloc(2 * (size_t)N);
    la.luni = c.d_luni.p;
    c.d_gnz.alloc(N);
    la.gnz = c.d_gnz.p;
    c.d_gtag.alloc(N);
    GS_HIP(hipMemsetAsync(c.d_gtag.p, 0, (size_t)N * 2, s));  // GC_BK counts from 1 per batch
    la.gtag = c.d_gtag.p;
    c.d_gpc.alloc(N);
    GS_HIP(hipMemsetAsync(c.d_gpc.p, 0, (size_t)N * 4, s));
    la.gpc = c.d_gpc.p;
    la.cr0 = chn->r0;
    la.chb = c.cfg.heartbeat_ns;
    la.cE = chn->cE;
    la.chz = c.cfg.churn_horizon;
    la.ghoff = chn->ghoff;
    la.ghk = c.cfg.churn_horizon - chn->ghoff;
    // heartbeats from gsw on push their IHAVEs to the targets that may still need
    // them (GS_GOSSIP_SWITCH, any value is exact). Off by default: at config #3's
    // shape the pushes cost more in k_gsend than the plane scans they replace
    // (121 ms per batch without, 129 ms from heartbeat 4 on, 193 ms from 1 on)
    const char* gsw = getenv("GS_GOSSIP_SWITCH");
    la.gsw = gsw && *gsw ? (uint32_t)atoi(gsw) : ~0u;
  }
  const char* cap = getenv("GS_LPULL_CAP");  // test knob: small lists force the overflow re-run
  la.ls = ls;
  la.lcap = cap && *cap ? (uint32_t)std::min<long>(std::max(1, atoi(cap)), (long)ls) : ls;
  // 40 KB of LDS per block: 4 blocks (16 waves, 16 rows in flight) resident per
  // CU. Large graphs launch up to 16 blocks per CU so that a pass's tail is
  // made of short blocks, keeping >= 32 rows per wave (1M peers: 54.3 ms per
  // step at 4 blocks per CU, 53.1 at 16; 100k peers: 7.8 ms at 16, 6.8 at 4;
  // profiles/r02_v7/lpull_grid_sweep.txt); GS_LPULL_BPC fixes blocks per CU
  const uint64_t bpc = [] {  // per batch: A/B scripts switch it in one process
    const char* e = getenv("GS_LPULL_BPC");
    return (uint64_t)(e && *e ? std::max(1, atoi(e)) : 0);
  }();
  // a power of two: 15 per CU measured 56.4 ms against 53.1 at 16 on one box
  uint64_t auto_bpc = 4;
  while (auto_bpc < 16 && (uint64_t)N >= (uint64_t)dev_cus * PULL_WAVES * 32 * auto_bpc * 2) auto_bpc *= 2;
  const uint64_t want = (uint64_t)dev_cus * (bpc ? bpc : auto_bpc);  // whole blocks per CU
  unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(((uint64_t)N + PULL_WAVES - 1) / PULL_WAVES, want));
  k_lseed<<<(unsigned)std::max<uint64_t>(1, std::min<uint64_t>((scap + TB - 1) / TB, (uint64_t)dev_cus * 4)), TB, 0, s>>>(
      la, c.d_skey.p, c.d_slane.p, c.d_scnt.p);
  {  // the rows whose emit step needs the publishers (LP_PUB); GS_LPULL_PUBW=0: every row loads them
    const char* pw = getenv("GS_LPULL_PUBW");  // per batch: A/B scripts switch it in one process
    la.pubw = pw && *pw && atoi(pw) == 0 ? 0u : 1u;
    const uint64_t nm = (uint64_t)(sl ? sl->S : 1u) * b.B, width = (chn ? CELL_W : MESH_W) + 1;
    if (la.pubw) k_lpubnb<<<(unsigned)((nm * width + TB - 1) / TB), TB, 0, s>>>(la, (uint32_t)nm);
  }
  for (uint32_t j = 0; j < (sl ? sl->S : 1u); j++) {  // (a slice's publishers are its rows)
    LPullArgs lj = la;
    if (sl) lj.pub = sl->spub + (size_t)j * b.B;
    k_lpub<<<(b.B * b.Fe + 255) / 256, 256, 0, s>>>(lj, b.Fe);
  }
  GS_HIP(hipGetLastError());
  if (gos) {  // GOS: sender planes, row-done bits, heartbeat control (gs_lpull_kernel.h)
    ensure_csrpos(c);
    c.d_gpl.alloc((size_t)N * LP_FW);
    c.d_gse.alloc(NL);
    c.d_rowdone.alloc(((size_t)N + 31) / 32);
    c.d_gctl.alloc(GC_WORDS);
    GS_HIP(hipMemsetAsync(c.d_rowdone.p, 0, ((size_t)N + 31) / 32 * 4, s));
    GS_HIP(hipMemsetAsync(c.d_gctl.p, 0, GC_WORDS * 8, s));
    GS_HIP(hipMemcpyAsync(c.d_gctl.p + GC_FD0, c.d_counters.p + C_FD, 8, hipMemcpyDeviceToDevice, s));
    GS_HIP(hipMemcpyAsync(c.d_gctl.p + GC_FDP, c.d_counters.p + C_FD, 8, hipMemcpyDeviceToDevice, s));
    la.grel0 = gos->rel0;
    la.ghb = gos->hb;
    la.glat_min = b.lat_min;
    la.glat_max = b.lat_max;
    la.gnf = (uint64_t)(sl ? sl->S : 1u) * b.B * b.Fe * (N0 - 1);  // lanes that can be final, less the publishers'
    la.F = b.F;
    la.collide = b.collide ? 1u : 0u;
    la.gseed = c.cfg.seed;
    la.ghist = c.cfg.history_gossip;
    la.gd_lazy = c.cfg.d_lazy;
    la.ggf = c.cfg.gossip_factor_milli;
    la.gctl = c.d_gctl.p;
    la.gpl = c.d_gpl.p;
    la.gse = c.d_gse.p;
    la.rowdone = c.d_rowdone.p;
    la.row = c.d_row.p;
    la.col = c.d_col.p;
    la.flags = c.d_flags.p;
    la.csrpos = c.d_csrpos.p;
    la.habs0 = c.d_habs0.p;
  }
  auto dispatch = [&] {
    if (gos) lpull_dispatch_gos(la, grid, s);
    else lpull_dispatch(b.FP, la, grid, s);
  };
  uint32_t pass = 0;
  for (;;) {
    for (uint32_t q = 0; q < 8; q++) {
      la.pass = pass++;
      if (c.timing) {  // (start, mid, end): the whole pass is frontier time
        GS_HIP(hipEventRecord(ev(n_ev), s));
        GS_HIP(hipEventRecord(ev(n_ev + 1), s));
        dispatch();
        GS_HIP(hipEventRecord(ev(n_ev + 2), s));
        n_ev += 3;
      } else {
        dispatch();
      }
    }
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_pctrl.p, 12 * 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipMemcpyAsync(c.h_pinned + 12, c.d_counters.p + C_ERR, 8, hipMemcpyDeviceToHost, s));  // same sync
    if (c.pass_poll) c.pass_poll();  // (while these passes run: the next batch's epoch chain is enqueued)
    GS_HIP(hipStreamSynchronize(s));
    static const bool dbg_pass = getenv("GS_DEBUG_PASSES") != nullptr;
    if (dbg_pass && pass % 256 == 0)
      fprintf(stderr, "[gs] pass %u: mode %llu lo %llu records %llu min %llx err %llx\n", pass,
              (unsigned long long)c.h_pinned[((pass - 1) % 3) * 4 + 1], (unsigned long long)c.h_pinned[((pass - 1) % 3) * 4],
              (unsigned long long)c.h_pinned[((pass - 1) % 3) * 4 + 2],
              (unsigned long long)c.h_pinned[((pass - 1) % 3) * 4 + 3], (unsigned long long)c.h_pinned[12]);
    // a batch's passes end (every window of its lifetime emitted); a count far
    // past that is a bug, reported instead of looping
    if (pass > (1u << 20)) c.fail(GS_ERANGE, "internal: the list pass did not finish in 2^20 passes");
    if (c.h_pinned[((pass - 1) % 3) * 4 + 1] == PM_DONE) break;
    if (c.h_pinned[12] & (ERR_LIST | ERR_RING)) break;  // lost already: stop early, re-run on k_pull
  }
  c.stats.relax_launches += pass;
  if (c.h_pinned[12] & (ERR_LIST | ERR_RING)) {  // the error word as of the last pass read
    GS_HIP(hipMemcpyAsync(c.d_counters.p, c.d_lp_save.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
    return false;
  }
  c.stats.list_pull_batches++;
  if (idw) return true;  // the final keys are dense rows already
  if (dense) {  // a sink, the traffic pass or a fragment group needs [N][L] rows
    k_lfinal<<<grid, TB, 0, s>>>(la);
    GS_HIP(hipGetLastError());
  } else {
    c.keys_log = true;
  }
  return true;
}

#ifdef GS_PULL_PROF
extern "C" int gs_debug_pull_prof(uint64_t* out) {  // 32 passes x 8 slots; read and clear
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pull_prof), sizeof(g_pull_prof)) != hipSuccess) return -1;
  static const uint64_t zero[32 * 8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pull_prof), zero, sizeof(g_pull_prof)) == hipSuccess ? 0 : -1;
}
#endif

// Blocks per CU of the split (push) path's scan / frontier / gossip grid: 4
// measured best on config #3 (k_scan 177 -> 136 us, k_frontier 65 -> 38 us per
// bucket vs 16; 1-2 and 32-64 slower, profiles/r01_v10/c3_grid_sweep.txt).
// GS_SPLIT_BLOCKS_PER_CU overrides it (read once per context).
static uint32_t split_blocks_per_cu(Ctx& c) {
  if (!c.split_bpc) {
    const char* e = getenv("GS_SPLIT_BLOCKS_PER_CU");
    c.split_bpc = e && *e ? (uint32_t)std::max(1, atoi(e)) : 4u;
  }
  return c.split_bpc;
}

// Lazy gossip is a no-op for message q when every non-publisher completed and
// the last completion lies before the first IHAVE can arrive: the earliest
// gossip heartbeat is rel0 (the first one at or after t_pub; every gossiping
// peer holds the message by then at the latest) and an IHAVE travels at least
// the smallest link latency. Then every IHAVE target has seen the message, no
// IWANT is sent and no key changes.
static bool gossip_noop(const Batch& b, const uint64_t* ms, const std::vector<uint64_t>& rel0) {
  for (uint32_t q = 0; q < b.B; q++)
    if (ms[(size_t)q * MS_COLS + MS_UNDEL] || ms[(size_t)q * MS_COLS + MS_TMAX] >= rel0[q] + b.lat_min) return false;
  return true;
}

// The churn list pass's per-batch tables (gs_cpull.h) for epochs [E0, E0 + cE)
// and the batch's publish epochs q0 (lanes). chn_begin before the epoch chain
// runs; chn_chunks then puts k_cprep of every chunk of 64 epochs whose epochs
// the chain has enqueued on the side stream (the chain is latency-bound, the
// target selection compute-bound: they overlap), chn_end the rest, the
// offline lanes per relative epoch (k_coff) and the join.
struct ChnPrep {
  uint64_t E0 = 0;
  uint32_t cE = 0, cW = 0, next = 0, par = 0;  // par: the table set (Ctx::ct) this batch fills
  bool offe = false;
  size_t nev = 0;
  hipStream_t s = nullptr;  // the stream the epoch chain runs on (chunk events are recorded there)
  CPrepArgs pa{};
  unsigned grid = 1;
};
static hipEvent_t cp_event(Ctx& c, uint32_t par, size_t i) {
  std::vector<hipEvent_t>& v = c.cp_ev[par & 1];
  while (v.size() <= i) {
    hipEvent_t e;
    GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    v.push_back(e);
  }
  return v[i];
}
static void chn_begin(Ctx& c, ChnPrep& cp, uint32_t par, hipStream_t s, uint64_t E0, uint32_t cE, const uint64_t* q0,
                      const gs_publish* sched, uint32_t B, uint32_t FP) {
  const uint32_t N = c.cfg.peers, H = c.cfg.churn_horizon, R = c.ring_R;
  const uint32_t cW = (cE + 63) / 64;
  Ctx::ChnTables& t = c.ct[par & 1];
  if (!c.cell_valid) {
    c.d_ccol.alloc((size_t)N * CELL_W);
    c.d_cpos.alloc((size_t)N * CELL_W);
    k_cell<<<(unsigned)(((uint64_t)N * CELL_W + TB - 1) / TB), TB, 0, s>>>(N, c.d_row.p, c.d_col.p, c.d_rev.p,
                                                                          c.d_stage.p, c.d_ccol.p, c.d_cpos.p);
    GS_HIP(hipGetLastError());
    c.cell_valid = true;
  }
  std::vector<uint32_t> cq(B);
  std::vector<uint8_t> ok(B);
  for (uint32_t q = 0; q < B; q++) {
    cq[q] = (uint32_t)(q0[q] - E0);
    ok[q] = !offline_draw(c.cfg.seed, c.cfg.churn_ppm, c.cfg.churn_down, sched[q].publisher, q0[q]);
  }
  std::vector<uint16_t> alive(64, 0);  // lane j: bit q = lane q*64 + j published (lane l: message l / FP)
  for (uint32_t l = 0; l < B * FP; l++)
    if (ok[l / FP]) alive[l & 63] |= (uint16_t)(1u << (l >> 6));
  t.cq.alloc(c.cfg.batch);
  t.pubok.alloc(c.cfg.batch);
  t.calive.alloc(LP_FW);
  GS_HIP(hipMemcpyAsync(t.cq.p, cq.data(), B * 4, hipMemcpyHostToDevice, s));
  GS_HIP(hipMemcpyAsync(t.pubok.p, ok.data(), B, hipMemcpyHostToDevice, s));
  GS_HIP(hipMemcpyAsync(t.calive.p, alive.data(), 128, hipMemcpyHostToDevice, s));
  t.offe.alloc((size_t)N * cW);
  t.cmm.alloc((size_t)N * cE);
  t.cgt.alloc((size_t)N * cE);
  t.coff.alloc((size_t)(H + 2) * N * LP_FW);
  GS_HIP(hipStreamSynchronize(s));  // cq / ok / alive die here
  cp.E0 = E0;
  cp.cE = cE;
  cp.cW = cW;
  cp.next = 0;
  cp.par = par & 1;
  cp.offe = false;
  cp.nev = 0;
  cp.s = s;
  CPrepArgs& pa = cp.pa;
  pa = CPrepArgs{};
  pa.ccol = c.d_ccol.p; pa.ring_mm = c.d_ring_mm.p; pa.offe = t.offe.p; pa.cq = t.cq.p;
  pa.cmm = t.cmm.p; pa.cgt = c.cfg.lazy_gossip ? t.cgt.p : nullptr; pa.coff = t.coff.p;
  pa.E0 = E0; pa.N = N; pa.R = R; pa.cE = cE; pa.cW = cW; pa.B = B; pa.H = H; pa.FP = FP;
  pa.seed = c.cfg.seed; pa.d_lazy = c.cfg.d_lazy; pa.gf_milli = c.cfg.gossip_factor_milli;
  ensure_cus(c);
  cp.grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((N + 3) / 4, (uint64_t)std::max(c.num_cus, 1) * 8));
}
// The chunks whose epochs are all <= h_done (every remaining one with `all`).
static void chn_chunks(Ctx& c, ChnPrep& cp, uint64_t h_done, bool all) {
  uint32_t c1 = cp.next;
  while (c1 < cp.cW && (all || cp.E0 + std::min<uint64_t>(64ull * (c1 + 1), cp.cE) - 1 <= h_done)) c1++;
  if (c1 == cp.next) return;
  const uint32_t N = c.cfg.peers, w64 = (N + 63) / 64;
  hipStream_t side = side_stream(c);
  const hipEvent_t e = cp_event(c, cp.par, cp.nev++);
  GS_HIP(hipEventRecord(e, cp.s ? cp.s : c.stream));  // (in line: the stream churn_ring runs the chain on)
  GS_HIP(hipStreamWaitEvent(side, e, 0));
  if (!cp.offe) {  // every epoch's offline bits are in the ring once the chain's run started
    k_offe<<<dim3(w64, cp.cW), 64, 0, side>>>(N, c.d_ring_off.p, w64, c.ring_R, cp.E0, cp.cE, cp.cW,
                                              c.ct[cp.par].offe.p);
    k_coff<<<cp.grid, TB, 0, side>>>(cp.pa);  // the offline lanes need no mesh: beside the chain too
    cp.offe = true;
  }
  cp.pa.c0 = cp.next;
  cp.pa.c1 = c1;
  k_cprep<<<cp.grid, TB, 0, side>>>(cp.pa);
  GS_HIP(hipGetLastError());
  cp.next = c1;
}
// The rest of the tables, then `to` waits for them (nullptr: cp.s, and the host too).
static void chn_end(Ctx& c, ChnPrep& cp, hipStream_t to = nullptr) {
  chn_chunks(c, cp, 0, true);
  const hipEvent_t e = cp_event(c, cp.par, cp.nev++);
  GS_HIP(hipEventRecord(e, side_stream(c)));
  GS_HIP(hipStreamWaitEvent(to ? to : c.stream, e, 0));
  GS_HIP(hipGetLastError());
  if (to) return;
  const uint32_t N = c.cfg.peers, R = c.ring_R, cE = cp.cE;
  const uint64_t E0 = cp.E0;
  const Ctx::ChnTables& t = c.ct[cp.par];
  hipStream_t s = c.stream;
  GS_HIP(hipStreamSynchronize(s));
  if (getenv("GS_DEBUG_CHN")) {  // diagnostic: the tables against the ELL ring and offline_draw
    std::vector<uint64_t> row(N + 1), cmm((size_t)N * cE), cge((size_t)N * cE);
    std::vector<uint32_t> col(c.nnz), ell((size_t)R * N * MESH_W);
    GS_HIP(hipMemcpy(row.data(), c.d_row.p, (N + 1) * 8, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(col.data(), c.d_col.p, c.nnz * 4, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(cmm.data(), t.cmm.p, cmm.size() * 8, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(cge.data(), t.cgt.p, cge.size() * 8, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(ell.data(), c.d_ring_mesh.p, ell.size() * 4, hipMemcpyDeviceToHost));
    uint64_t bad_mm = 0, bad_ge = 0;
    for (uint32_t w = 0; w < N; w++)
      for (uint32_t e = 0; e < cE; e++) {
        const uint64_t E = E0 + e;
        const uint32_t* er = &ell[((size_t)(E % R) * N + w) * MESH_W];
        uint64_t mm = 0, ge = 0;
        const bool woff = offline_draw(c.cfg.seed, c.cfg.churn_ppm, c.cfg.churn_down, w, E);
        std::vector<std::pair<uint64_t, uint32_t>> cand;
        for (uint64_t x = row[w]; x < row[w + 1]; x++) {
          bool in = false;
          for (uint32_t j = 0; j < MESH_W; j++) in |= er[j] != EMPTY && (er[j] & 0xFFFFFFu) == col[x];
          if (in) mm |= 1ull << (x - row[w]);
          else if (!woff && !offline_draw(c.cfg.seed, c.cfg.churn_ppm, c.cfg.churn_down, col[x], E))
            cand.push_back({rng(c.cfg.seed, P_GOSSIP, w, (uint32_t)E, col[x]), (uint32_t)(x - row[w])});
        }
        std::sort(cand.begin(), cand.end(), [&](const std::pair<uint64_t, uint32_t>& p1, const std::pair<uint64_t, uint32_t>& p2) {
          return p1.first < p2.first || (p1.first == p2.first && col[row[w] + p1.second] < col[row[w] + p2.second]);
        });
        uint32_t r = (uint32_t)(((uint64_t)cand.size() * c.cfg.gossip_factor_milli) / 1000);
        if (r < c.cfg.d_lazy) r = c.cfg.d_lazy;
        if (r > cand.size()) r = (uint32_t)cand.size();
        for (uint32_t q = 0; q < r; q++) ge |= 1ull << cand[q].second;
        if (!c.cfg.lazy_gossip) ge = 0;
        if (mm != cmm[(size_t)w * cE + e] && bad_mm++ < 5)
          fprintf(stderr, "[chn] mm w %u E %llu dev %llx host %llx\n", w, (unsigned long long)E,
                  (unsigned long long)cmm[(size_t)w * cE + e], (unsigned long long)mm);
        if (ge != cge[(size_t)w * cE + e] && bad_ge++ < 5)
          fprintf(stderr, "[chn] ge w %u E %llu dev %llx host %llx\n", w, (unsigned long long)E,
                  (unsigned long long)cge[(size_t)w * cE + e], (unsigned long long)ge);
      }
    fprintf(stderr, "[chn] E0 %llu cE %u: mm mismatches %llu, ge mismatches %llu\n", (unsigned long long)E0, cE,
            (unsigned long long)bad_mm, (unsigned long long)bad_ge);
  }
}

// The churn snapshot ring: R slots of per-epoch meshes, offline
// bitsets and (lazy gossip) inverse IHAVE lists, sized once per context.
static void ensure_ring(Ctx& c) {
  if (c.ring_R) return;
  const uint32_t N = c.cfg.peers, Bmax = c.cfg.batch;
  const bool gossip = c.cfg.lazy_gossip != 0;
  const uint64_t w64 = ((uint64_t)N + 63) / 64;
  const uint64_t per_slot = (uint64_t)N * MESH_W * 4 + w64 * 8 + (gossip ? (uint64_t)N * (GT_IN * 4 + 4) : 0) +
                            (uint64_t)N * 8;
  const char* rb = getenv("GS_RING_BUDGET_MB");  // test knob: force batch cuts at the ring size
  const uint64_t budget = rb && *rb ? (uint64_t)atoll(rb) << 20 : 16ull << 30;
  const uint64_t want = (uint64_t)Bmax + c.cfg.churn_horizon + 1;
  c.ring_R = (uint32_t)std::min<uint64_t>(want, std::max<uint64_t>(c.cfg.churn_horizon + 2, budget / per_slot));
  c.d_ring_mesh.alloc((size_t)c.ring_R * N * MESH_W);
  c.d_ring_off.alloc((size_t)c.ring_R * w64);
  if (c.max_degree <= CELL_W) c.d_ring_mm.alloc((size_t)c.ring_R * N);  // the churn list pass's meshes
  if (gossip) c.d_ring_in.alloc((size_t)c.ring_R * N * GT_IN);  // inverse IHAVE lists (ring_in_lists)
}

static void run_messages_impl(Ctx& c, const gs_publish* sched, uint64_t n_msgs, const gs_result_sink* sink,
                              const std::vector<uint8_t>* cut);

// Schedules that are not lockstep: the churn list pass and the
// gossip inside the list pass need every message of a batch at the same
// offset r = (t_pub - hb_phase) mod heartbeat (its heartbeats and epoch
// boundaries are then one relative time for all lanes). run.sh's free
// message_delay (run.sh:36; 1500 ms gives two offsets) and arbitrary POST
// /publish sequences (main.rs:146-221) are not. Messages are independent
// given the mesh of each epoch, so the run takes each group of consecutive
// messages a batch could hold (same size and chunk count, <= the batch size,
// churn: its epochs in the ring) in offset-class order — a batch per class,
// each lockstep — and hands the results back in schedule order. Classes per
// group are capped (GS_CLASS_MAX, default 64; a group with more keeps its
// order); streaming sinks (on_block, on_lat) and device sinks keep the order
// too. GS_CLASS_SPLIT=0 turns the regrouping off.
static bool class_plan(Ctx& c, const gs_publish* sched, uint64_t n, const gs_result_sink* sink,
                       std::vector<uint64_t>& perm, std::vector<uint8_t>& cut) {
  const bool churn = c.cfg.churn_ppm != 0, gossip = c.cfg.lazy_gossip != 0;
  if ((!churn && !gossip) || n < 2 || c.sink_dev) return false;
  if (sink && (sink->on_block || sink->on_lat)) return false;
  const char* e = getenv("GS_CLASS_SPLIT");
  if (e && *e && atoi(e) == 0) return false;
  const char* mx = getenv("GS_CLASS_MAX");
  const uint64_t cmax = mx && *mx ? (uint64_t)std::max(1, atoi(mx)) : 64u;
  const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
  for (uint64_t i = 0; i < n; i++)
    if (sched[i].t_pub_ns < ph) return false;  // (run_messages_impl reports what it must)
  if (churn) ensure_ring(c);
  const uint32_t Bmax = c.cfg.batch;
  perm.resize(n);
  cut.assign(n, 0);
  bool any = false;
  for (uint64_t g0 = 0; g0 < n;) {  // a group: what one batch could hold
    const uint32_t F0 = frags_of(c, sched[g0]);
    const uint64_t cap = std::max<uint32_t>(1, std::min<uint32_t>(Bmax, PULL_LMAX / pow2_at_least(F0)));
    uint64_t g1 = g0 + 1, lo = (sched[g0].t_pub_ns - ph) / hb, hi = lo;
    while (g1 < n && g1 - g0 < cap && sched[g1].msg_size == sched[g0].msg_size && frags_of(c, sched[g1]) == F0) {
      if (churn) {
        const uint64_t ep = (sched[g1].t_pub_ns - ph) / hb, lo2 = std::min(lo, ep), hi2 = std::max(hi, ep);
        if (hi2 + c.cfg.churn_horizon - lo2 + 1 > c.ring_R) break;
        lo = lo2;
        hi = hi2;
      }
      g1++;
    }
    std::vector<std::pair<uint64_t, uint64_t>> key(g1 - g0);  // (offset class, message)
    for (uint64_t i = g0; i < g1; i++) key[i - g0] = {(sched[i].t_pub_ns - ph) % hb, i};
    std::stable_sort(key.begin(), key.end(), [](const std::pair<uint64_t, uint64_t>& x,
                                                 const std::pair<uint64_t, uint64_t>& y) { return x.first < y.first; });
    uint64_t ncls = 1;
    for (size_t k = 1; k < key.size(); k++) ncls += key[k].first != key[k - 1].first;
    const bool split = ncls > 1 && ncls <= cmax && !(churn && F0 > 1);  // (fragmented churn: the push path)
    cut[g0] = 1;
    for (uint64_t i = g0; i < g1; i++) {
      perm[i] = split ? key[i - g0].second : i;
      if (split && i > g0 && key[i - g0].first != key[i - g0 - 1].first) cut[i] = 1;
    }
    any = any || split;
    g0 = g1;
  }
  return any;
}

void run_messages(Ctx& c, const gs_publish* sched, uint64_t n_msgs, const gs_result_sink* sink) {
  std::vector<uint64_t> perm;
  std::vector<uint8_t> cut;
  if (!class_plan(c, sched, n_msgs, sink, perm, cut)) return run_messages_impl(c, sched, n_msgs, sink, nullptr);
  std::vector<gs_publish> ps(n_msgs);
  for (uint64_t i = 0; i < n_msgs; i++) ps[i] = sched[perm[i]];
  if (!sink) return run_messages_impl(c, ps.data(), n_msgs, nullptr, &cut);
  // the results in class order, then every row back to its message
  const uint32_t N = c.cfg.peers;
  gs_result_sink ts = *sink;
  std::vector<uint64_t> tc(sink->t_complete_ns ? (size_t)n_msgs * N : 0);
  std::vector<uint8_t> hp(sink->hops ? (size_t)n_msgs * N : 0);
  std::vector<gs_msg_summary> sm(sink->summary ? n_msgs : 0);
  ts.t_complete_ns = sink->t_complete_ns ? tc.data() : nullptr;
  ts.hops = sink->hops ? hp.data() : nullptr;
  ts.summary = sink->summary ? sm.data() : nullptr;
  run_messages_impl(c, ps.data(), n_msgs, &ts, &cut);
  for (uint64_t i = 0; i < n_msgs; i++) {
    const uint64_t m = perm[i];
    if (sink->t_complete_ns) memcpy(sink->t_complete_ns + m * N, tc.data() + i * N, (size_t)N * 8);
    if (sink->hops) memcpy(sink->hops + m * N, hp.data() + i * N, N);
    if (sink->summary) sink->summary[m] = sm[i];
  }
}

static void run_messages_impl(Ctx& c, const gs_publish* sched, uint64_t n_msgs, const gs_result_sink* sink,
                              const std::vector<uint8_t>* cut) {
  const uint32_t N = c.cfg.peers;
  const uint32_t Bmax = c.cfg.batch;
  hipStream_t s = c.stream;
  if (c.lat_pend.on) {  // left by a run that failed: its lines are not handed out
    GS_HIP(hipStreamSynchronize(c.copy));
    c.lat_pend.on = false;
  }
  c.lat_async = true;
  struct AsyncOff {
    Ctx& c;
    int unwinding0 = std::uncaught_exceptions();
    ~AsyncOff() {
      c.lat_async = false;
      //  a run that fails after a batch completed still hands out that
      // batch's pending latency lines, as the synchronous sink did before; nothing
      // here may throw while the error unwinds
      Ctx::LatPending& p = c.lat_pend;
      if (std::uncaught_exceptions() <= unwinding0 || !p.on) return;
      p.on = false;
      if (hipEventSynchronize(c.lat_done[p.par]) != hipSuccess || (c.h_laterr[p.par] & ERR_LAT16)) return;
      for (uint32_t q0 = 0; q0 < p.B; q0 += p.bm) {
        const uint32_t n = std::min(p.bm, p.B - q0);
        p.sink->on_lat(p.sink->user, p.row0 + q0, n, p.un, c.h_lat[p.par] + (size_t)q0 * p.un);
      }
    }
  } async_off{c};
  // Churn runs (config #3): the epoch chain is latency-bound and runs as fast on
  // one XCD's 32 CUs as on all 256 (one L2 holds its per-peer state; bits 0..31
  // of the CU mask, 4 CUs on each XCD, take twice as long), and the list pass at
  // 100k peers as fast on 7 XCDs (or 4) as on 8 (profiles/r06_chain). So the
  // chain gets its own XCD (c.chain_pipe, GS_CHAIN_XCDS, default XCD 0) and the
  // rest of the run the others (c.pass_ms, GS_PASS_XCDS, default 1-7): the next
  // batch's chain then runs beside this batch's passes (ChnAhead below).
  // GS_CHN_PIPE=0 keeps one stream; GS_PASS_SKIP / GS_PASS_XCDS alone: experiments.
  ensure_cus(c);
  const char* pipe_env = getenv("GS_CHN_PIPE");
  const bool pipe_on = c.cfg.churn_ppm && !(pipe_env && *pipe_env && atoi(pipe_env) == 0) && c.num_cus == 256 &&
                       c.cfg.flood_publish && !c.traffic && !c.sink_dev && !getenv("GS_DEBUG_CHN");
  struct PassStream {
    Ctx& c;
    hipStream_t orig = nullptr;
    PassStream(Ctx& cc, bool pipe) : c(cc) {
      const char* e = getenv("GS_PASS_SKIP");
      uint32_t px = xcd_env("GS_PASS_XCDS");
      if (pipe) {
        if (!c.chain_pipe) {
          const uint32_t cx = xcd_env("GS_CHAIN_XCDS");
          c.chain_pipe = xcd_stream(c, cx ? cx : 0x01u);
        }
        if (!px) px = 0xFEu & ~xcd_env("GS_CHAIN_XCDS");
      }
      if (!px && (!e || !*e || atoi(e) <= 0)) return;
      if (!c.pass_ms) {  // created once per context (a CU-masked stream costs ~10 ms)
        c.pass_ms = px ? xcd_stream(c, px) : cu_stream_except(c, 0, (uint32_t)atoi(e));
        for (auto& ev : c.pass_ev) GS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      }
      orig = c.stream;
      GS_HIP(hipEventRecord(c.pass_ev[0], orig));
      GS_HIP(hipStreamWaitEvent(c.pass_ms, c.pass_ev[0], 0));
      c.stream = c.pass_ms;
    }
    ~PassStream() {
      if (!orig) return;
      (void)hipEventRecord(c.pass_ev[1], c.pass_ms);
      (void)hipStreamWaitEvent(orig, c.pass_ev[1], 0);
      (void)hipStreamSynchronize(orig);
      c.stream = orig;
    }
  } pass_stream{c, pipe_on};
  s = c.stream;
  GS_HIP(hipMemsetAsync(c.d_counters.p + C_ERR, 0, 8, s));
  check_schedule(c, sched, n_msgs);
  uint32_t Fmax = 1;
  for (uint64_t i = 0; i < n_msgs; i++) Fmax = std::max(Fmax, frags_of(c, sched[i]));
  const uint32_t FPmax = pow2_at_least(Fmax);
  const char* var_env = getenv("GS_RELAX_VARIANT");
  // default: owner-computes pull over candidate lists (64 | 32), fragmented batches
  // too (128; config #2 7.2e8 against 6.7e8/s on k_pull's dense rows, round 4);
  // k_pull's dense rows without 64; without 32 the push path: split (8) + final
  // bitset (4) + read filter (1)
  uint32_t variant = var_env && *var_env ? (uint32_t)atoi(var_env) : 237u;
  const bool lanes32 = (uint64_t)N * Bmax * FPmax < (1ull << 32);  // frontier indices are u32
  if (!lanes32) variant &= ~8u;
  const bool gossip = c.cfg.lazy_gossip != 0;
  // the pull path needs rows in LDS and one mesh per batch (churn uses one per
  // epoch: the push path). IDONTWANT batches run on the list pass with dense
  // final keys when their rows are single-fragment (k_lpull<1, CH, true>),
  // else on the push path. Lazy gossip runs on the pull path when the batch
  // proves it a no-op (gossip_noop), else the batch is re-run on the push path.
  const bool churn = c.cfg.churn_ppm != 0;  // per-epoch mesh lookups live on the push path
  const bool pull_any = (variant & 32) && !churn;
  // churn on the list pass (gs_cpull.h): lockstep batches (rows of fragment groups
  // included) without IDONTWANT, CSR rows of <= 64 entries (<= 58 with lazy gossip: the IHAVE entry's
  // target mask); GS_CHURN_LIST=0 keeps them on the push path
  const char* chl_env = getenv("GS_CHURN_LIST");
  const bool chn_any = churn && (variant & 32) && (variant & 64) && !(chl_env && *chl_env && atoi(chl_env) == 0) &&
                       c.max_degree <= (gossip ? GSE_HOPS : CELL_W) && N < (1u << 21);
  // the push path with gossip or churn runs split, without tile skip
  // the push path with gossip or churn runs split + tile skip (its long tail of
  // IHAVE and churn buckets touches few tiles); GS_RELAX_VARIANT can turn the skip off
  const uint32_t pvariant = (gossip || churn) ? (((variant | 8u) & ~32u) | (var_env && *var_env ? 0u : 2u))
                                              : (variant & ~32u);
  if (churn && !lanes32) c.fail(GS_EUNSUPPORTED, "churn needs peers*batch*FP < 2^32");
  std::vector<uint64_t> q0v(Bmax), r0v(Bmax), ep(churn ? n_msgs : 0);
  if (churn) {  // epoch of every publish; the snapshot ring
    const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
    for (uint64_t i = 0; i < n_msgs; i++) {
      if (sched[i].t_pub_ns < ph || (sched[i].t_pub_ns - ph) / hb >= (1ull << 20))
        c.fail(GS_EINVAL, "churn needs every publish within 2^20 heartbeats after hb_phase_ns");
      ep[i] = (sched[i].t_pub_ns - ph) / hb;
    }
    ensure_ring(c);
  }
  const size_t max_tiles = ((size_t)N * Bmax * FPmax + 63) / 64;
  c.d_keys.alloc((size_t)N * Bmax * FPmax);
  c.d_meta.alloc(max_tiles * sizeof(TileMeta) / 8);
  c.d_fbits.alloc(max_tiles);
  if (FPmax > 1) c.d_busy.alloc((size_t)N * Bmax);
  c.d_tc.alloc((size_t)N * Bmax);
  c.d_hops.alloc((size_t)N * Bmax);
  c.d_cnt_save.alloc(C_COUNT);
  std::vector<uint64_t> rel0(Bmax), habs0(Bmax);
  std::vector<uint8_t> malive(Bmax);
  uint64_t g0 = INF64;
  // Timing events come from a per-context pool: [0] run start, [1] run end,
  // then one (start, scan end, end) triple around every relaxation launch.
  size_t n_ev = 0;
  auto ev = [&](size_t i) {
    while (c.ev_pool.size() <= i) {
      hipEvent_t e;
      GS_HIP(hipEventCreate(&e));
      c.ev_pool.push_back(e);
    }
    return c.ev_pool[i];
  };
  if (c.timing) {
    GS_HIP(hipEventRecord(ev(0), s));
    ev(1);
    n_ev = 2;
  }
  ensure_cus(c);
  const int dev_cus = c.num_cus;
  // Batch slices: consecutive full batches of one shape on a small graph run as
  // one list pass over S copies of the graph (run_lpull_batch's Slices), so that
  // a launch has S x N rows instead of N: a pass of a few rows per resident wave
  // is mostly latency (config #2's 10k-peer F = 8 rows: 98 us per pass at 10k
  // rows, 340 us at 80k; scripts/c2_probe.py). Frozen mesh, no IDONTWANT, no
  // per-peer traffic; lazy gossip through the eager pass's no-op proof, per slice,
  // and when that fails (or failed before: glp_prefer) inside the group's passes
  // as run_glp does, if the whole group is lockstep (else single batches take
  // it). GS_SLICES=0 turns them off, GS_SLICES=n caps a group at n slices.
  const char* sl_env = getenv("GS_SLICES");
  const uint32_t sl_max = sl_env && *sl_env ? (uint32_t)std::max(0, atoi(sl_env)) : 64u;
  constexpr uint64_t SL_ROWS = 1ull << 19;  // rows per pass a group aims at (memory: ~S x N x L x 40 B)
  uint64_t slice_skip = 0;                  // messages before it run as single batches
  auto try_slices = [&](uint64_t i0, uint64_t& i_end) -> bool {
    if (sl_max < 2 || !pull_any || !(variant & 64) || c.traffic || (uint64_t)N * 2 >= (1u << 21)) return false;
    const uint32_t F0 = frags_of(c, sched[i0]), FP0 = pow2_at_least(F0);
    if (FP0 > 1 && !(variant & 128)) return false;
    const uint32_t Bc = std::min<uint32_t>(Bmax, PULL_LMAX / FP0);
    const uint64_t s_cap = std::min<uint64_t>({(uint64_t)sl_max, std::max<uint64_t>(1, SL_ROWS / N), ((1ull << 21) - 1) / N});
    uint64_t n_same = 1;  // messages of this shape from i0 (as far as a group can take)
    while (n_same < s_cap * Bc && i0 + n_same < n_msgs && !(cut && (*cut)[i0 + n_same]) &&
           sched[i0 + n_same].msg_size == sched[i0].msg_size &&
           frags_of(c, sched[i0 + n_same]) == F0)
      n_same++;
    const uint32_t S = (uint32_t)std::min<uint64_t>(n_same / Bc, s_cap);
    if (S < 2) return false;
    slice_skip = i0 + (uint64_t)S * Bc;  // unless the group completes below
    std::vector<Batch> bs(S);
    std::vector<uint32_t> spub((size_t)S * Bc), lpub((size_t)S * Bc);
    for (uint32_t j = 0; j < S; j++) {
      const uint64_t q0 = i0 + (uint64_t)j * Bc;
      bs[j] = setup_batch(c, sched, q0, q0 + Bc, j == 0);
      for (uint32_t q = 0; q < Bc; q++) {
        lpub[(size_t)j * Bc + q] = sched[q0 + q].publisher;
        spub[(size_t)j * Bc + q] = sched[q0 + q].publisher + j * N;
      }
    }
    Batch g = bs[0];  // the slices' keys: the source field holds slice rows (S x N ids)
    g.sb = bits_for(S * N);
    g.tshift = g.sb + HOP_BITS;
    g.tmax = g.tshift >= 64 ? 0 : (INF64 >> g.tshift);
    for (Batch& bj : bs) {
      bj.sb = g.sb;
      bj.tshift = g.tshift;
      bj.tmax = g.tmax;
    }
    if (c.cfg.idontwant && g.payload >= c.cfg.idontwant) return false;
    const uint64_t grain = pull_grain(g.tshift);
    if (g.delta < grain) return false;
    std::vector<uint64_t> stp((size_t)S * Bc);
    for (uint32_t j = 0; j < S; j++) std::copy(bs[j].tpub.begin(), bs[j].tpub.end(), stp.begin() + (size_t)j * Bc);
    // lazy gossip inside the passes (the group's IHAVE / IWANT as run_glp's): every
    // message of the group has its heartbeats at the same time after its publish
    std::vector<uint64_t> rel(stp.size()), hab(stp.size());
    bool lock = gossip;
    if (gossip) {
      const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
      for (size_t q = 0; q < stp.size(); q++) {
        const uint64_t tp = stp[q], h0 = tp <= ph ? 0 : (tp - ph + hb - 1) / hb;
        rel[q] = ph + h0 * hb - tp;
        hab[q] = h0;
        lock = lock && rel[q] == rel[0];
      }
    }
    const char* glp_env = getenv("GS_GOSSIP_LIST");
    Batch gg = g;
    gg.delta = std::min(g.delta, g.lat_min);
    const bool glp_ok = lock && !(glp_env && *glp_env && atoi(glp_env) == 0) && c.max_degree <= GSE_HOPS &&
                        gg.delta >= grain && c.cfg.heartbeat_ns > g.lat_max + gg.delta;
    if (gossip && c.glp_prefer && !glp_ok) return false;  // single batches (the push path)
    const size_t NR = (size_t)S * N;
    c.d_spub.alloc(spub.size());
    c.d_lpub.alloc(lpub.size());
    c.d_stpub.alloc(stp.size());
    GS_HIP(hipMemcpyAsync(c.d_spub.p, spub.data(), spub.size() * 4, hipMemcpyHostToDevice, s));
    GS_HIP(hipMemcpyAsync(c.d_lpub.p, lpub.data(), lpub.size() * 4, hipMemcpyHostToDevice, s));
    GS_HIP(hipMemcpyAsync(c.d_stpub.p, stp.data(), stp.size() * 8, hipMemcpyHostToDevice, s));
    c.d_keys.alloc(NR * g.L);
    if (g.FP > 1) c.d_busy.alloc(NR * Bc);
    auto fresh = [&] {  // per-run state of the group's pass
      c.keys_log = false;
      if (g.FP > 1) GS_HIP(hipMemsetAsync(c.d_busy.p, 0, NR * Bc * 8, s));
    };
    const SinkWants sw = sink_wants(sink);
    const bool dense = sw.rows() || sw.summary || getenv("GS_LPULL_DENSE");
    const bool wants = sw.rows() || sw.lat || sw.summary;
    const Slices sl{S, N, c.d_spub.p, c.d_lpub.p};
    auto slice_in = [&](uint32_t j) {  // slice j's publishers and publish times where completion reads them
      GS_HIP(hipMemcpyAsync(c.d_pub.p, lpub.data() + (size_t)j * Bc, Bc * 4, hipMemcpyHostToDevice, s));
      GS_HIP(hipMemcpyAsync(c.d_tpub.p, bs[j].tpub.data(), Bc * 8, hipMemcpyHostToDevice, s));
    };
    auto finish = [&] {  // completion of a group whose keys stand
      if (!wants) {  // device-resident results: the counters only
        if (c.keys_log) run_complete(c, bs[0], 0, N, false, false, false, false, 0, c.d_lpub.p, c.d_stpub.p, S);
        else
          for (uint32_t j = 0; j < S; j++)
            run_complete(c, bs[j], 0, N, false, false, false, false, (size_t)j * N, c.d_lpub.p + (size_t)j * Bc,
                         c.d_stpub.p + (size_t)j * Bc);
      } else {
        for (uint32_t j = 0; j < S; j++) {
          slice_in(j);
          launch_complete(c, bs[j], 0, N, sink, i0 + (uint64_t)j * Bc, (size_t)j * N);
        }
      }
    };
    auto run_glp_group = [&]() -> bool {  // the gossip inside the group's passes
      uint32_t lbg = 0;
      const uint32_t Kg = lpull_ring(c, gg, gg.delta / grain * grain, &lbg, true, false, S * N);
      if (!Kg) return false;
      fresh();
      c.d_habs0.alloc(std::max<size_t>(Bmax, hab.size()));
      GS_HIP(hipMemcpyAsync(c.d_habs0.p, hab.data(), hab.size() * 8, hipMemcpyHostToDevice, s));
      const GosRun gr{rel[0], c.cfg.heartbeat_ns};
      const uint64_t iw0 = read_counter(c, C_GOSSIP);
      if (!run_lpull_batch(c, gg, Kg, lbg, ev, n_ev, dev_cus, dense, false, &gr, nullptr, &sl)) return false;
      c.stats.list_pull_batches += S - 1;
      c.stats.gossip_list_batches += S;
      if (read_counter(c, C_GOSSIP) != iw0) c.glp_quiet = 0;  // (run_glp's rule, per batch of the group)
      else if ((c.glp_quiet += S) >= GLP_QUIET) c.glp_prefer = false;
      finish();
      return true;
    };
    bool ok = false;
    if (gossip && c.glp_prefer) {
      ok = run_glp_group();
    } else {
      uint32_t lb = 0;
      const uint32_t K = lpull_ring(c, g, g.delta / grain * grain, &lb, false, false, S * N);
      if (!K) return false;
      fresh();
      if (gossip) GS_HIP(hipMemcpyAsync(c.d_cnt_save.p, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
      if (!run_lpull_batch(c, g, K, lb, ev, n_ev, dev_cus, dense, false, nullptr, nullptr, &sl))
        return false;  // (a list overflowed: counters restored; single batches take the messages)
      c.stats.list_pull_batches += S - 1;
      if (!gossip) {
        finish();
        ok = true;
      } else {  // the eager result stands only if gossip is a no-op in every slice
        // every slice's reductions into one pinned buffer, one wait
        const size_t msb = (size_t)S * Bc * MS_COLS * 8;
        if (c.h_slms_bytes < msb) {
          if (c.h_slms) GS_HIP(hipHostFree(c.h_slms));
          c.h_slms = nullptr;
          c.h_slms_bytes = 0;
          GS_HIP(hipHostMalloc((void**)&c.h_slms, msb, hipHostMallocDefault));
          c.h_slms_bytes = msb;
        }
        if (c.keys_log) {  // every slice in one launch
          run_complete(c, bs[0], 0, N, true, false, false, false, 0, c.d_lpub.p, c.d_stpub.p, S);
          GS_HIP(hipMemcpyAsync(c.h_slms, c.d_mstat.p, msb, hipMemcpyDeviceToHost, s));
        } else {
          for (uint32_t j = 0; j < S; j++) {
            run_complete(c, bs[j], 0, N, true, false, false, false, (size_t)j * N, c.d_lpub.p + (size_t)j * Bc,
                         c.d_stpub.p + (size_t)j * Bc);
            GS_HIP(hipMemcpyAsync(c.h_slms + (size_t)j * Bc * MS_COLS, c.d_mstat.p, (size_t)Bc * MS_COLS * 8,
                                  hipMemcpyDeviceToHost, s));
          }
        }
        GS_HIP(hipStreamSynchronize(s));
        bool noop = true;
        for (uint32_t j = 0; j < S && noop; j++) {
          const std::vector<uint64_t> r0(rel.begin() + (size_t)j * Bc, rel.begin() + (size_t)(j + 1) * Bc);
          noop = gossip_noop(bs[j], c.h_slms + (size_t)j * Bc * MS_COLS, r0);
        }
        if (noop) {
          c.stats.gossip_noop_msgs += (uint64_t)S * Bc;
          if (wants) {  // the sink's results: completion again per slice, its counters not counted twice
            c.d_cnt_save2.alloc(C_COUNT);
            GS_HIP(hipMemcpyAsync(c.d_cnt_save2.p, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
            for (uint32_t j = 0; j < S; j++) {
              slice_in(j);
              launch_complete(c, bs[j], 0, N, sink, i0 + (uint64_t)j * Bc, (size_t)j * N);
            }
            GS_HIP(hipMemcpyAsync(c.d_counters.p, c.d_cnt_save2.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
          }
          ok = true;
        } else {  // gossip changes the group: discard the eager run; the gossip inside the passes takes it
          GS_HIP(hipMemcpyAsync(c.d_counters.p, c.d_cnt_save.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
          c.stats.list_pull_batches -= S;
          if (glp_ok) {  // (without the in-pass gossip the single batches take it: they count their own)
            c.stats.gossip_fallback_batches++;
            c.glp_prefer = true;
            c.glp_quiet = 0;
            ok = run_glp_group();
          }
        }
      }
    }
    if (!ok) return false;
    GS_HIP(hipStreamSynchronize(s));  // (lpub / tpub / habs0 host copies die here)
    c.stats.messages += (uint64_t)S * Bc;
    c.stats.batches += S;
    i_end = i0 + (uint64_t)S * Bc;
    return true;
  };
  // a batch: up to B messages of equal size and chunk count (serialisation
  // tables and the lane layout are per batch); the pull path holds a row in
  // registers, so its batch is capped at PULL_LMAX / FP messages. Returns the
  // end; churn: the batch's publish epochs [h_lo, h_hi] (+ lifetime) fit the ring.
  auto form = [&](uint64_t a0, uint64_t& h_lo, uint64_t& h_hi) -> uint64_t {
    const uint32_t F0 = frags_of(c, sched[a0]);
    const uint32_t Bcap = pull_any || (chn_any && F0 == 1)
                              ? std::max<uint32_t>(1, std::min<uint32_t>(Bmax, PULL_LMAX / pow2_at_least(F0)))
                              : Bmax;
    uint64_t a1 = a0 + 1;
    h_lo = churn ? ep[a0] : 0;
    h_hi = churn ? ep[a0] : 0;
    while (a1 < n_msgs && a1 - a0 < Bcap && !(cut && (*cut)[a1]) && sched[a1].msg_size == sched[a0].msg_size &&
           frags_of(c, sched[a1]) == F0) {
      if (churn) {
        const uint64_t lo2 = std::min(h_lo, ep[a1]), hi2 = std::max(h_hi, ep[a1]);
        if (hi2 + c.cfg.churn_horizon - lo2 + 1 > c.ring_R) break;
        h_lo = lo2;
        h_hi = hi2;
      }
      a1++;
    }
    return a1;
  };
  // churn: the batch runs on the churn list pass (gs_cpull.h) — lockstep
  // batches (fragment groups included) without IDONTWANT whose windows fit the rules
  auto chn_decide = [&](const Batch& bb, const uint64_t* r0, uint64_t h_lo, uint64_t h_hi) -> bool {
    if (!chn_any || bb.collide || !c.d_ring_mm.p) return false;
    const uint64_t hb = c.cfg.heartbeat_ns;
    const bool idw = c.cfg.idontwant && bb.payload >= c.cfg.idontwant;
    bool lock = true;
    for (uint32_t q = 1; q < bb.B && lock; q++) lock = r0[q] == r0[0];
    const uint64_t dl = gossip ? std::min(bb.delta, bb.lat_min) : bb.delta;
    const uint64_t cE = h_hi + c.cfg.churn_horizon - h_lo + 1;
    return !idw && lock && cE <= 4096 && dl >= pull_grain(bb.tshift) && hb > lpull_rmax(bb) + 2 * dl &&
           (!gossip || hb > bb.lat_max + dl);
  };
  // ChnAhead: the next churn list-pass batch's epoch chain and tables, enqueued
  // on the chain's XCD (c.chain_pipe) while this batch's passes run on the
  // others (the host enqueues the chain in slices between pass groups, at most
  // AH_LEAD epochs ahead of what the GPU finished). The list pass reads only the
  // batch tables, so the chain may overwrite ring slots of the batch whose
  // passes run; a batch that falls back to the push path joins the chain first
  // and has churn_ring replay its ring slots.
  constexpr uint64_t AH_MARK = 16, AH_LEAD = 192, AH_SLICE = 64;
  struct Ahead {
    bool on = false, joined = false;
    uint64_t i0 = 0, i1 = 0, h1 = 0;
    ChnPrep cp;
    EvRun* run = nullptr;
    hipEvent_t ready = nullptr;
    std::vector<hipEvent_t> marks;  // ring of events every AH_MARK epochs on the chain stream
    uint64_t mark_n = 0, done_h = 0, enq_h = 0;
  } ah;
  struct AheadFree {
    Ahead& ah;
    ~AheadFree() {
      if (ah.run) chain_free(ah.run);
      if (ah.ready) (void)hipEventDestroy(ah.ready);
      for (auto e : ah.marks) (void)hipEventDestroy(e);
    }
  } ah_free{ah};
  std::vector<uint64_t> q0a(Bmax), r0a(Bmax);
  static const bool dbg_ah = getenv("GS_DEBUG_AHEAD") != nullptr;
  auto ah_enqueue_end = [&] {  // every epoch is enqueued: the rest of the tables, then `ready`
    if (dbg_ah) fprintf(stderr, "[ah] batch %llu: chain enqueued (%llu epochs)\n", (unsigned long long)ah.i0,
                        (unsigned long long)ah.enq_h);
    chain_free(ah.run);
    ah.run = nullptr;
    chn_end(c, ah.cp, c.chain_pipe);
    if (!ah.ready) GS_HIP(hipEventCreateWithFlags(&ah.ready, hipEventDisableTiming));
    GS_HIP(hipEventRecord(ah.ready, c.chain_pipe));
  };
  auto ah_pump = [&](bool all) {  // more of the chain, keeping at most AH_LEAD epochs in flight
    if (!ah.on || !ah.run) return;
    while (ah.run) {
      if (!all) {
        while (ah.mark_n && ah.done_h + AH_MARK <= ah.enq_h) {  // the oldest outstanding mark
          const uint64_t k = ah.done_h / AH_MARK + 1;  // mark k: after epoch k * AH_MARK of the run
          if (k > ah.mark_n) break;
          if (hipEventQuery(ah.marks[(k - 1) % ah.marks.size()]) != hipSuccess) break;
          ah.done_h = k * AH_MARK;
        }
        if (ah.enq_h >= ah.done_h + AH_LEAD) return;
      }
      const uint64_t n = all ? ~0ull : std::min<uint64_t>(AH_SLICE, ah.done_h + AH_LEAD - ah.enq_h);
      for (uint64_t k = 0; k < n && ah.run; k++) {
        const bool fin = chain_advance(c, *ah.run, 1);
        ah.enq_h++;
        if (ah.enq_h % AH_MARK == 0) {
          if (ah.marks.size() < 2 * AH_LEAD / AH_MARK + 2) {
            hipEvent_t e;
            GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ah.marks.push_back(e);
          }
          ah.mark_n = ah.enq_h / AH_MARK;
          GS_HIP(hipEventRecord(ah.marks[(ah.mark_n - 1) % ah.marks.size()], c.chain_pipe));
        }
        if (fin) ah_enqueue_end();
      }
      if (!all) return;
    }
  };
  auto ah_join = [&] {  // the prepared batch's tables before the main stream's next work
    if (!ah.on || ah.joined) return;
    ah_pump(true);
    GS_HIP(hipStreamWaitEvent(c.stream, ah.ready, 0));
    ah.joined = true;
    if (dbg_ah) fprintf(stderr, "[ah] batch %llu: joined\n", (unsigned long long)ah.i0);
  };
  auto ah_start = [&](uint64_t n0) {
    if (!pipe_on || ah.on || n0 >= n_msgs) return;
    uint64_t hl = 0, hh = 0;
    const uint64_t n1 = form(n0, hl, hh);
    const Batch b2 = setup_batch(c, sched, n0, n1, false);
    const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
    for (uint32_t q = 0; q < b2.B; q++) {
      q0a[q] = ep[n0 + q];
      r0a[q] = b2.tpub[q] - ph - q0a[q] * hb;
    }
    const uint64_t h1 = hh + c.cfg.churn_horizon;
    if (!chn_decide(b2, r0a.data(), hl, hh) || h1 <= c.churn_state) return;
    const uint32_t par = c.ct_par ^ 1u;
    // the chain overwrites ring slots: after every reader of this batch's slots on the main stream
    if (!ah.ready) GS_HIP(hipEventCreateWithFlags(&ah.ready, hipEventDisableTiming));
    GS_HIP(hipEventRecord(ah.ready, c.stream));
    GS_HIP(hipStreamWaitEvent(c.chain_pipe, ah.ready, 0));
    chn_begin(c, ah.cp, par, c.chain_pipe, hl, (uint32_t)(h1 - hl + 1), q0a.data(), sched + n0, b2.B, b2.FP);
    ah.run = chain_begin(c, h1, c.chain_pipe, [&](uint64_t h) { chn_chunks(c, ah.cp, h, false); });
    if (!ah.run) return;  // (not a plain continuation of the ring: the batch prepares in line)
    c.ct_par = par;
    ah.on = true;
    ah.joined = false;
    ah.i0 = n0;
    ah.i1 = n1;
    ah.h1 = h1;
    ah.mark_n = ah.done_h = ah.enq_h = 0;
    if (dbg_ah)
      fprintf(stderr, "[ah] batch %llu..%llu: chain to epoch %llu (state %llu), tables %u\n", (unsigned long long)n0,
              (unsigned long long)n1, (unsigned long long)h1, (unsigned long long)c.churn_state, par);
    ah_pump(false);
  };
  uint64_t i0 = 0;
  while (i0 < n_msgs) {
    if (i0 >= slice_skip) {
      uint64_t ie = 0;
      if (try_slices(i0, ie)) {
        i0 = ie;
        continue;
      }
    }
    uint64_t h_lo = 0, h_hi = 0;  // churn: publish epochs of the batch
    const uint64_t i1 = form(i0, h_lo, h_hi);
    const Batch b = setup_batch(c, sched, i0, i1);
    const uint32_t FP = b.FP;
    bool chn = false;  // this batch runs on the churn list pass
    ChnPrep cp;
    if (churn) {
      const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
      for (uint32_t q = 0; q < b.B; q++) {
        q0v[q] = ep[i0 + q];
        r0v[q] = b.tpub[q] - ph - q0v[q] * hb;
      }
      chn = chn_decide(b, r0v.data(), h_lo, h_hi);
      if (ah.on && !(chn && ah.i0 == i0 && ah.i1 == i1)) {  // (not expected: batches form the same way)
        ah_join();
        ah.on = false;
      }
      if (ah.on) {  // this batch's chain and tables ran ahead beside the last batch's passes
        ah_join();
        cp = ah.cp;
        ah.on = false;
      } else {
        c.ring_in_defer = chn;  // the push path's inverse IHAVE lists are not needed
        c.ring_ell_defer = chn;  // nor the ELL snapshots (the pass reads the mask ring)
        if (chn) {
          c.ct_par ^= 1u;
          chn_begin(c, cp, c.ct_par, s, h_lo, (uint32_t)(h_hi + c.cfg.churn_horizon - h_lo + 1), q0v.data(), sched + i0,
                    b.B, b.FP);
          cp.s = nullptr;  // (the chunk events go where churn_ring runs the chain)
          c.epoch_hook = [&](uint64_t h) { chn_chunks(c, cp, h, false); };
        }
        try {
          churn_ring(c, h_lo, h_hi + c.cfg.churn_horizon);
        } catch (...) {
          c.epoch_hook = nullptr;
          c.ring_in_defer = false;
          c.ring_ell_defer = false;
          throw;
        }
        c.epoch_hook = nullptr;
        c.ring_in_defer = false;
        c.ring_ell_defer = false;
        // readers of the ELL snapshots beside the list pass: seeds to the mesh (no flood
        // publish), the per-peer traffic pass, the GS_DEBUG_CHN check
        if (chn && (!c.cfg.flood_publish || c.traffic || getenv("GS_DEBUG_CHN")))
          ensure_ring_ell(c, h_lo, h_hi + c.cfg.churn_horizon);
        //  a batch for the push path may overlap the last epochs of an
        // earlier churn list-pass batch, which skipped their ELL snapshots and
        // inverse IHAVE lists: rebuild those slots (tag-checked: free when current)
        if (!chn) {
          ensure_ring_ell(c, h_lo, h_hi + c.cfg.churn_horizon);
          if (gossip) ensure_in_lists(c, h_lo, h_hi + c.cfg.churn_horizon);
        }
        if (chn) chn_end(c, cp);
      }
      c.d_q0.alloc(Bmax);
      c.d_r0.alloc(Bmax);
      GS_HIP(hipMemcpyAsync(c.d_q0.p, q0v.data(), b.B * 8, hipMemcpyHostToDevice, s));
      GS_HIP(hipMemcpyAsync(c.d_r0.p, r0v.data(), b.B * 8, hipMemcpyHostToDevice, s));
      GS_HIP(hipStreamSynchronize(s));
    }
    const uint32_t B = b.B, L = b.L;
    if (gossip) {  // heartbeats at hb_phase + h*hb: first one at or after each t_pub
      const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
      for (uint32_t q = 0; q < B; q++) {
        const uint64_t tp = b.tpub[q];
        const uint64_t h0 = tp <= ph ? 0 : (tp - ph + hb - 1) / hb;
        rel0[q] = ph + h0 * hb - tp;
        habs0[q] = h0;
      }
      c.d_rel0.alloc(Bmax);
      c.d_habs0.alloc(Bmax);
      GS_HIP(hipMemcpyAsync(c.d_rel0.p, rel0.data(), B * 8, hipMemcpyHostToDevice, s));
      GS_HIP(hipMemcpyAsync(c.d_habs0.p, habs0.data(), B * 8, hipMemcpyHostToDevice, s));
      g0 = INF64;
      if (churn) {  // per message: gossip can spread it (publisher online at t_pub, a heartbeat in its lifetime)
        for (uint32_t q = 0; q < B; q++) {
          malive[q] = habs0[q] <= q0v[q] + c.cfg.churn_horizon &&
                      !offline_draw(c.cfg.seed, c.cfg.churn_ppm, c.cfg.churn_down, sched[i0 + q].publisher, q0v[q]);
          g0 = std::min(g0, rel0[q]);
        }
        uint64_t lmin = INF64;
        for (uint64_t l : c.lat_ns) lmin = std::min(lmin, l);
        g0 += lmin;
        c.d_malive.alloc(Bmax);
        GS_HIP(hipMemcpyAsync(c.d_malive.p, malive.data(), B, hipMemcpyHostToDevice, s));
      }
      GS_HIP(hipStreamSynchronize(s));  // rel0 / habs0 host vectors are rewritten by the next batch
    }
    const uint64_t total = (uint64_t)N * L;
    auto reset = [&](uint32_t v, bool with_gossip, bool dense_keys = true) {  // fresh keys and bucket state
      c.keys_log = false;
      if (dense_keys) GS_HIP(hipMemsetAsync(c.d_keys.p, 0xFF, total * 8, s));  // the list pull path needs none
      if (FP > 1) GS_HIP(hipMemsetAsync(c.d_busy.p, 0, (size_t)N * B * 8, s));
      if (v & 32) return;
      if (v & 2) GS_HIP(hipMemsetAsync(c.d_meta.p, 0, (total + 63) / 64 * sizeof(TileMeta), s));
      if (v & 12) GS_HIP(hipMemsetAsync(c.d_fbits.p, 0, (total + 63) / 64 * 8, s));
      if ((v & 10) == 10) {  // split + tile skip: tmin 0 forces every tile's first scan
        c.d_tmin.alloc(max_tiles);
        c.d_touched.alloc(max_tiles);
        GS_HIP(hipMemsetAsync(c.d_tmin.p, 0, (total + 63) / 64 * 8, s));
        GS_HIP(hipMemsetAsync(c.d_touched.p, 0, (total + 63) / 64, s));
        if (with_gossip) {
          c.d_tgmin.alloc(max_tiles);
          c.d_tnf.alloc(max_tiles);
          c.d_tstamp.alloc(max_tiles);
          GS_HIP(hipMemsetAsync(c.d_tstamp.p, 0, (total + 63) / 64 * 4, s));
        }
      }
      GS_HIP(hipMemsetAsync(c.d_ctrl.p, 0xFF, 4 * 8, s));
      // with gossip the first bucket is [0, Delta): the publisher's own IHAVEs
      // can land before the first eager arrival
      if (with_gossip) GS_HIP(hipMemsetAsync(c.d_ctrl.p, 0, 8, s));
    };
    // One batch on the push path: k_seed, then bucket launches in chunks of 8
    // until the ctrl word of the next bucket is empty.
    auto push_run = [&](uint32_t v, bool with_gossip) {
      reset(v, with_gossip);
      launch_seed(c, b, 0, N);
      RelaxArgs ra = relax_args(c, b, with_gossip);
      if (ra.ring_in) {
        ra.malive = c.d_malive.p;
        ra.g0 = g0;
      }
      ra.busy = c.d_busy.p;
      ra.meta = reinterpret_cast<TileMeta*>(c.d_meta.p);
      ra.fbits = c.d_fbits.p;
      ra.tmin = c.d_tmin.p;
      ra.touched = c.d_touched.p;
      ra.ctrl = c.d_ctrl.p;
      ra.counters = c.d_counters.p; ra.delta = b.delta;
      const uint64_t need = (total + TB - 1) / TB;
      const unsigned grid = (unsigned)std::min<uint64_t>(need, (uint64_t)dev_cus * split_blocks_per_cu(c));
      if (v & 8) {  // frontier segments: one per scan wave
        const uint64_t nwaves = (uint64_t)grid * (TB / 64), ntiles = (total + 63) / 64;
        // tiles one scan wave can visit: groups of 64 with tile skip (k_scan), single tiles without
        const uint64_t gt = (v & 2) ? 64 : 1;
        const uint64_t wave_tiles = ((ntiles + gt - 1) / gt + nwaves - 1) / nwaves * gt;
        ra.seg_cap = (uint32_t)(wave_tiles * (64 / FP));
        c.d_fr_idx.alloc(nwaves * ra.seg_cap);
        if (FP == 1) c.d_fr_key.alloc(nwaves * ra.seg_cap);
        c.d_fr_cnt.alloc(nwaves);
        ra.fr_idx = c.d_fr_idx.p;
        ra.fr_key = c.d_fr_key.p;
        ra.fr_cnt = c.d_fr_cnt.p;
        if (with_gossip) {  // gossip list: per-lane entries, one segment per scan wave
          ra.gl_cap = (uint32_t)(wave_tiles * 64);
          c.d_gl_idx.alloc(nwaves * ra.gl_cap);
          c.d_gl_cnt.alloc(nwaves);
          c.d_nonfinal.alloc(3);
          GS_HIP(hipMemsetAsync(c.d_nonfinal.p, 0, 3 * 8, s));
          ra.gl_idx = c.d_gl_idx.p;
          ra.gl_cnt = c.d_gl_cnt.p;
          if (ra.ring_in) {
            c.d_gl_key.alloc(nwaves * ra.gl_cap);
            ra.gl_key = c.d_gl_key.p;
            // holder list (a lane is finalised once) and per-launch marks
            c.d_hl_idx.alloc(total);
            c.d_hl_key.alloc(total);
            c.d_hl_cnt.alloc(1);
            c.d_hl_mark.alloc(2 * (size_t)HL_LAUNCHES);
            c.d_hwin.alloc(total);
            GS_HIP(hipMemsetAsync(c.d_hwin.p, 0xFF, total, s));
            ra.hwin = c.d_hwin.p;
            c.d_hs_idx.alloc(nwaves * ra.gl_cap);
            c.d_hs_key.alloc(nwaves * ra.gl_cap);
            c.d_hl_min.alloc(3);
            GS_HIP(hipMemsetAsync(c.d_hl_cnt.p, 0, 8, s));
            GS_HIP(hipMemsetAsync(c.d_hl_min.p, 0xFF, 3 * 8, s));
            ra.hs_idx = c.d_hs_idx.p;
            ra.hs_key = c.d_hs_key.p;
            ra.hl_min = c.d_hl_min.p;
            ra.hl_idx = c.d_hl_idx.p;
            ra.hl_key = c.d_hl_key.p;
            ra.hl_cnt = (unsigned long long*)c.d_hl_cnt.p;
            ra.hl_lo = c.d_hl_mark.p;
            ra.hl_end = c.d_hl_mark.p + HL_LAUNCHES;
          }
          ra.nonfinal = c.d_nonfinal.p;
          if ((v & 10) == 10) {
            ra.tgmin = c.d_tgmin.p;
            ra.tnf = c.d_tnf.p;
            ra.tstamp = c.d_tstamp.p;
          }
        }
      }
      uint32_t launch = 0;
      const uint32_t chunk = 8;
      for (;;) {
        if (ra.hl_idx && launch + chunk > HL_LAUNCHES)
          c.fail(GS_EUNSUPPORTED, "churn + lazy gossip batch needs more than 65536 buckets");
        for (uint32_t q = 0; q < chunk; q++) {
          ra.launch = launch++;
          if (c.timing) {  // (start, scan end, end) per bucket
            GS_HIP(hipEventRecord(ev(n_ev), s));
            const hipEvent_t mid = ev(n_ev + 1);
            if (v & 8) relax_dispatch(FP, v, ra, grid, s, mid);
            else {
              relax_dispatch(FP, v, ra, grid, s);
              GS_HIP(hipEventRecord(mid, s));
            }
            GS_HIP(hipEventRecord(ev(n_ev + 2), s));
            n_ev += 3;
          } else {
            relax_dispatch(FP, v, ra, grid, s);
          }
        }
        GS_HIP(hipGetLastError());
        GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_ctrl.p, 3 * 8, hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        if (c.h_pinned[launch % 3] == INF64) break;
      }
      c.stats.relax_launches += launch;
    };
    // Lazy gossip on a frozen mesh: run eager forwarding first (the pull pass,
    // or the push path without gossip when IDONTWANT needs it) and keep it if
    // the batch proves gossip a no-op; otherwise discard its counters and run
    // the push path with gossip. Under churn some peers never
    // complete, so the proof cannot hold and gossip runs directly.
    const bool idw_b = c.cfg.idontwant && b.payload >= c.cfg.idontwant;  // IDONTWANT active in this batch
    // IDONTWANT on the list pass: windows no wider than the smallest latency, so
    // that a neighbour's key final in the same window as the sender's can never
    // pass the test t_y + lat(y -> u) <= t_u (the sender cannot see it yet);
    // keys of earlier windows are final and stored before the pass starts
    Batch bw = b;
    if (idw_b) bw.delta = std::min(b.delta, b.lat_min);
    const bool pull_ok = pull_any && bw.delta >= pull_grain(b.tshift) && (!idw_b || (b.FP == 1 && (variant & 64)));
    // Lazy gossip inside the list pass (GOS, gs_lpull_kernel.h): rows without
    // IDONTWANT (fragment groups too: every fragment is gossiped on its own at its
    // message's heartbeats, as the oracle's sched_gossip) on the frozen mesh, every message's heartbeats
    // the same time after its publish (lockstep), CSR rows narrow enough for a
    // 58-bit target mask, windows no wider than the smallest latency (an IHAVE
    // never shares a window with its heartbeat) and heartbeats farther apart
    // than an IHAVE travels. GS_GOSSIP_LIST=0 keeps such batches on the eager
    // pass + no-op proof, with the push path behind it.
    bool lockstep = gossip && B > 0;
    for (uint32_t q = 1; q < B && lockstep; q++) lockstep = rel0[q] == rel0[0];
    Batch bg = b;
    bg.delta = std::min(b.delta, b.lat_min);
    const uint64_t ggr = pull_grain(b.tshift);
    const char* glp_env = getenv("GS_GOSSIP_LIST");
    const bool glp = gossip && !churn && pull_ok && (b.FP == 1 || (variant & 128)) && (variant & 64) && lockstep &&
                     !(glp_env && *glp_env && atoi(glp_env) == 0) && c.max_degree <= GSE_HOPS && bg.delta >= ggr &&
                     c.cfg.heartbeat_ns > b.lat_max + bg.delta;
    bool glp_tried = false;
    auto run_glp = [&]() -> bool {
      glp_tried = true;
      uint32_t lb = 0;
      const uint32_t K = lpull_ring(c, bg, bg.delta / ggr * ggr, &lb, true);
      if (!K) return false;
      reset(variant, false, idw_b);  // IDONTWANT: dense INF keys (the finals stay dense rows)
      const GosRun gr{rel0[0], c.cfg.heartbeat_ns};
      const SinkWants sw = sink_wants(sink);
      const bool dense = sw.rows() || sw.summary || c.traffic || getenv("GS_LPULL_DENSE");
      const uint64_t iw0 = read_counter(c, C_GOSSIP);
      if (!run_lpull_batch(c, bg, K, lb, ev, n_ev, dev_cus, dense, idw_b, &gr)) return false;
      c.stats.gossip_list_batches++;
      // GLP_QUIET batches in a row whose gossip sent no IWANT: the next one tries the
      // eager pass and its no-op proof first again (glp_prefer was never
      // cleared). Not after one: batches alternating with and without IWANTs (a
      // heartbeat late in the dissemination) would pay a failed proof every other batch.
      if (read_counter(c, C_GOSSIP) != iw0) c.glp_quiet = 0;
      else if (++c.glp_quiet >= GLP_QUIET) c.glp_prefer = false;
      if (c.traffic) launch_traffic(c, b);
      launch_complete(c, b, 0, N, sink, i0);
      return true;
    };
    bool done = false;
    if (chn) {  // churn on the list pass; a list overflow falls back to the push path
      uint32_t lb = 0;
      Batch bc = b;
      if (gossip) bc.delta = std::min(b.delta, b.lat_min);
      const uint64_t grain = pull_grain(b.tshift);
      const uint32_t K = lpull_ring(c, bc, bc.delta / grain * grain, &lb, gossip, true);
      if (K) {
        reset(variant, false, false);
        const GosRun gr{rel0[0], c.cfg.heartbeat_ns};
        const ChnRun cr{h_lo, r0v[0], (uint32_t)(h_hi + c.cfg.churn_horizon - h_lo + 1),
                        gossip ? (uint32_t)(habs0[0] - q0v[0]) : 0u, cp.par};
        const SinkWants sw = sink_wants(sink);
        const bool dense = sw.rows() || sw.summary || c.traffic || getenv("GS_LPULL_DENSE");
        // the next batch's chain beside these passes, from the first pass group on:
        // the seeds (k_seed reads this batch's offline bits in the ring) are
        // enqueued by then, and the chain's stream waits for them
        bool ah_tried = false;
        if (pipe_on) c.pass_poll = [&] {
          if (!ah_tried) {
            ah_tried = true;
            ah_start(i1);
          } else {
            ah_pump(false);
          }
        };
        struct PollOff {
          Ctx& c;
          ~PollOff() { c.pass_poll = nullptr; }
        } poll_off{c};
        if (run_lpull_batch(c, bc, K, lb, ev, n_ev, dev_cus, dense, false, gossip ? &gr : nullptr, &cr)) {
          if (gossip) c.stats.gossip_list_batches++;
          if (c.traffic) launch_traffic(c, b);
          launch_complete(c, b, 0, N, sink, i0);
          done = true;
        }
      }
      if (!done && getenv("GS_REQUIRE_LPULL")) c.fail(GS_EUNSUPPORTED, "churn list pass cannot take this batch (GS_REQUIRE_LPULL)");
      if (!done) {  // the push path reads the ring: a chain ahead (of this batch or for the next one)
        ah_join();    // may have run past or overwritten this batch's slots, or a replay moved the ring
        churn_ring(c, h_lo, h_hi + c.cfg.churn_horizon);  // (no epochs when current; else runs / replays them)
      }
      if (!done) ensure_ring_ell(c, h_lo, h_hi + c.cfg.churn_horizon);  // the push path reads the ELL ring
      if (!done && gossip) ensure_in_lists(c, h_lo, h_hi + c.cfg.churn_horizon);
    }
    if (glp && c.glp_prefer) done = run_glp();
    if (!done && (pull_ok || (gossip && !churn))) {
      if (gossip) GS_HIP(hipMemcpyAsync(c.d_cnt_save.p, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
      if (pull_ok) {
        const uint64_t grain = pull_grain(b.tshift);
        uint32_t lb = 0;
        // list path for single-fragment batches; fragmented ones (FP > 1) with
        // bit 128 (the default)
        const bool lp = (variant & 64) && (b.FP == 1 || (variant & 128));
        const uint32_t K = lp ? lpull_ring(c, bw, bw.delta / grain * grain, &lb) : 0u;
        reset(variant, false, K == 0 || idw_b);  // IDONTWANT: dense INF keys
        if (lp && !K && getenv("GS_REQUIRE_LPULL"))  // test knob: no silent k_pull fallback
          c.fail(GS_EUNSUPPORTED, "list pull path cannot take this batch (GS_REQUIRE_LPULL)");
        // GS_LPULL_DENSE (diagnostic): dense rows + k_complete, whose known key
        // stream calibrates the PMC read factor (scripts/pmc_summary.py);
        // IDONTWANT batches keep their final keys dense all along
        const SinkWants sw = sink_wants(sink);
        const bool dense = !idw_b && (sw.rows() || sw.summary || c.traffic || getenv("GS_LPULL_DENSE"));
        if (!K || !run_lpull_batch(c, bw, K, lb, ev, n_ev, dev_cus, dense, idw_b)) {
          if (K && getenv("GS_REQUIRE_LPULL")) c.fail(GS_EUNSUPPORTED, "list pull overflow (GS_REQUIRE_LPULL)");
          if (idw_b) {  // k_pull has no IDONTWANT: the push path takes the batch
            push_run(variant & ~32u, false);
          } else {  // a candidate list overflowed (or no ring fits): this batch runs on k_pull
            if (K) reset(variant, false);
            run_pull_batch(c, b, ev, n_ev, dev_cus);
          }
        }
      } else {
        push_run(variant & ~32u, false);
      }
      if (!gossip) {
        if (c.traffic) launch_traffic(c, b);
        launch_complete(c, b, 0, N, sink, i0);
        done = true;
      } else {  // keep the eager result only if gossip provably changes nothing
        const SinkWants sw = sink_wants(sink);
        run_complete(c, b, 0, N, true, sw.summary, sw.rows() || sw.summary, sw.lat);
        std::vector<uint64_t> ms((size_t)B * MS_COLS);
        GS_HIP(hipMemcpyAsync(ms.data(), c.d_mstat.p, ms.size() * 8, hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        if (gossip_noop(b, ms.data(), rel0)) {
          if (c.traffic) launch_traffic(c, b);
          deliver(c, b, 0, N, sink, i0);
          c.stats.gossip_noop_msgs += B;
          done = true;
        } else {  // gossip can change this batch: discard the eager run's counters
          GS_HIP(hipMemcpyAsync(c.d_counters.p, c.d_cnt_save.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
          c.stats.gossip_fallback_batches++;
          if (glp && !glp_tried) {  // re-run with the gossip inside the passes; the context's
            c.glp_prefer = true;      // later batches go there directly (no eager run first)
            c.glp_quiet = 0;
            done = run_glp();
          }
        }
      }
    }
    if (!done) {
      if (getenv("GS_REQUIRE_LPULL")) c.fail(GS_EUNSUPPORTED, "the push path would take this batch (GS_REQUIRE_LPULL)");
      if (gossip && !lanes32)
        c.fail(GS_EUNSUPPORTED, "lazy gossip changes this batch and the push path needs "
                                "peers*batch*FP < 2^32: use a smaller batch");
      push_run(pvariant, gossip);
      if (c.traffic) launch_traffic(c, b);
      launch_complete(c, b, 0, N, sink, i0);
    }
    c.stats.messages += B;
    c.stats.batches++;
    i0 = i1;
  }
  lat_flush(c);  // the last batch's latencies
  if (c.timing) GS_HIP(hipEventRecord(ev(1), s));
  collect_stats(c);
  if (c.timing) {
    double scan = 0, front = 0;
    for (size_t q = 2; q + 2 < n_ev; q += 3) {
      float x = 0, y = 0;
      GS_HIP(hipEventElapsedTime(&x, c.ev_pool[q], c.ev_pool[q + 1]));
      GS_HIP(hipEventElapsedTime(&y, c.ev_pool[q + 1], c.ev_pool[q + 2]));
      scan += x;
      front += y;
    }
    c.stats.relax_ms += scan + front;
    c.stats.scan_ms += scan;
    c.stats.frontier_ms += front;
    float rm = 0;
    GS_HIP(hipEventElapsedTime(&rm, c.ev_pool[0], c.ev_pool[1]));
    c.stats.run_ms += rm;
  }
}

#include "gs_part.h"

}  // namespace gs
