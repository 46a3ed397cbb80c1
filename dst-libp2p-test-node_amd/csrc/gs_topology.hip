// gs_topology.hip — random ID dialing -> symmetric CSR peer graph on gfx950.
//
// Replaces connect_gossipsub_peers (rust-test-node/src/main.rs:303-389): each
// peer takes a random subset of the other ids and dials min(CONNECTTO+1,
// 2*CONNECTTO, N-1) of them (defect D4); the undirected union of accepted dials
// is the peer graph, with bit F_OUT on (u,w) when u dialed w. Optional
// MAXCONNECTIONS inbound cap (nim gossipsub-queues/main.nim:429).
//
// Kernels are one thread per peer / per dial: this runs once per simulation
// and is HBM-trivial (N*k*~40 B); determinism comes from per-row sorting, not
// from atomic order.
#include <hipcub/hipcub.hpp>

#include "gs_internal.h"

namespace gs {
namespace {

constexpr int TB = 256;

// Floyd's k-subset of the N-1 other ids, then ordered by a per-(v,id) key.
__global__ __launch_bounds__(TB) void k_dials(uint32_t N, uint32_t k, uint64_t seed,
                                              uint32_t* __restrict__ dial) {
  const uint32_t v = blockIdx.x * TB + threadIdx.x;
  if (v >= N) return;
  uint32_t out[MAX_DIALS];
  uint64_t key[MAX_DIALS];
  const uint64_t n = N - 1;
  for (uint32_t i = 0; i < k; i++) {
    const uint64_t j = n - k + i;
    const uint32_t r = (uint32_t)rand_below(rng(seed, P_DIAL, v, i, 0), j + 1);
    bool dup = false;
    for (uint32_t q = 0; q < i; q++) dup |= (out[q] == r);
    out[i] = dup ? (uint32_t)j : r;
  }
  for (uint32_t i = 0; i < k; i++) {
    const uint32_t id = out[i] < v ? out[i] : out[i] + 1;
    const uint64_t kx = rng(seed, P_DIAL_ORDER, v, id, 0);
    int32_t j = (int32_t)i - 1;
    while (j >= 0 && (key[j] > kx || (key[j] == kx && out[j] > id))) {
      out[j + 1] = out[j];
      key[j + 1] = key[j];
      j--;
    }
    out[j + 1] = id;
    key[j + 1] = kx;
  }
  for (uint32_t i = 0; i < k; i++) dial[(size_t)v * k + i] = out[i];
}

__global__ __launch_bounds__(TB) void k_inbound_count(uint64_t total, uint32_t k,
                                                      const uint32_t* __restrict__ dial,
                                                      uint64_t* __restrict__ cnt) {
  const uint64_t e = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (e >= total) return;
  atomicAdd((unsigned long long*)&cnt[dial[e]], 1ull);
}

__global__ __launch_bounds__(TB) void k_inbound_scatter(uint32_t N, uint32_t k,
                                                        const uint32_t* __restrict__ dial,
                                                        const uint64_t* __restrict__ off,
                                                        uint64_t* __restrict__ fill,
                                                        uint64_t* __restrict__ in) {
  const uint64_t e = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (e >= (uint64_t)N * k) return;
  const uint32_t v = (uint32_t)(e / k), j = (uint32_t)(e % k), t = dial[e];
  const uint64_t pos = atomicAdd((unsigned long long*)&fill[t], 1ull);
  in[off[t] + pos] = ((uint64_t)j << 32) | v;
}

// Acceptor t takes non-mutual inbound dials in (dial index, dialer) order up
// to max(0, cap - k).
__global__ __launch_bounds__(TB) void k_inbound_accept(uint32_t N, uint32_t k, uint32_t quota,
                                                       const uint32_t* __restrict__ dial,
                                                       const uint64_t* __restrict__ off,
                                                       uint64_t* __restrict__ in,
                                                       uint8_t* __restrict__ acc) {
  const uint32_t t = blockIdx.x * TB + threadIdx.x;
  if (t >= N) return;
  const uint64_t b = off[t], e = off[t + 1];
  for (uint64_t i = b + 1; i < e; i++) {  // insertion sort (rows ~ k long)
    const uint64_t x = in[i];
    uint64_t j = i;
    while (j > b && in[j - 1] > x) { in[j] = in[j - 1]; j--; }
    in[j] = x;
  }
  uint32_t taken = 0;
  for (uint64_t i = b; i < e; i++) {
    const uint32_t v = (uint32_t)in[i], j = (uint32_t)(in[i] >> 32);
    bool mutual = false;
    for (uint32_t q = 0; q < k; q++) mutual |= (dial[(size_t)t * k + q] == v);
    if (mutual) continue;
    if (taken < quota) taken++;
    else acc[(size_t)v * k + j] = 0;
  }
}

__global__ __launch_bounds__(TB) void k_deg(uint32_t N, uint32_t k, const uint32_t* __restrict__ dial,
                                            const uint8_t* __restrict__ acc,
                                            uint64_t* __restrict__ deg) {
  const uint64_t e = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (e >= (uint64_t)N * k || !acc[e]) return;
  atomicAdd((unsigned long long*)&deg[e / k], 1ull);
  atomicAdd((unsigned long long*)&deg[dial[e]], 1ull);
}

__global__ __launch_bounds__(TB) void k_half_edges(uint32_t N, uint32_t k,
                                                   const uint32_t* __restrict__ dial,
                                                   const uint8_t* __restrict__ acc,
                                                   const uint64_t* __restrict__ off,
                                                   uint64_t* __restrict__ fill,
                                                   uint64_t* __restrict__ he) {
  const uint64_t e = (uint64_t)blockIdx.x * TB + threadIdx.x;
  if (e >= (uint64_t)N * k || !acc[e]) return;
  const uint32_t v = (uint32_t)(e / k), t = dial[e];
  uint64_t p = atomicAdd((unsigned long long*)&fill[v], 1ull);
  he[off[v] + p] = ((uint64_t)t << 1) | 1ull;
  p = atomicAdd((unsigned long long*)&fill[t], 1ull);
  he[off[t] + p] = ((uint64_t)v << 1);
}

// Per-row sort + dedupe (OR of the outbound bits); ndeg[v] = distinct peers.
__global__ __launch_bounds__(TB) void k_sort_dedupe(uint32_t N, const uint64_t* __restrict__ off,
                                                    uint64_t* __restrict__ he,
                                                    uint64_t* __restrict__ ndeg) {
  const uint32_t v = blockIdx.x * TB + threadIdx.x;
  if (v >= N) return;
  const uint64_t b = off[v], e = off[v + 1];
  for (uint64_t i = b + 1; i < e; i++) {
    const uint64_t x = he[i];
    uint64_t j = i;
    while (j > b && he[j - 1] > x) { he[j] = he[j - 1]; j--; }
    he[j] = x;
  }
  uint64_t w = b;
  for (uint64_t i = b; i < e; i++) {
    if (w > b && (he[w - 1] >> 1) == (he[i] >> 1)) { he[w - 1] |= he[i] & 1ull; continue; }
    he[w++] = he[i];
  }
  ndeg[v] = w - b;
}

__global__ __launch_bounds__(TB) void k_compact(uint32_t N, const uint64_t* __restrict__ off,
                                                const uint64_t* __restrict__ he,
                                                const uint64_t* __restrict__ row,
                                                uint32_t* __restrict__ col,
                                                uint8_t* __restrict__ flags,
                                                unsigned* __restrict__ maxdeg) {
  const uint32_t v = blockIdx.x * TB + threadIdx.x;
  if (v >= N) return;
  const uint64_t b = off[v], r = row[v], n = row[v + 1] - r;
  for (uint64_t i = 0; i < n; i++) {
    col[r + i] = (uint32_t)(he[b + i] >> 1);
    flags[r + i] = (uint8_t)(he[b + i] & 1ull);
  }
  atomicMax(maxdeg, (unsigned)n);
}

// rev[e] = index of (w -> u) for e = (u -> w).
__global__ __launch_bounds__(TB) void k_reverse(uint32_t N, const uint64_t* __restrict__ row,
                                                const uint32_t* __restrict__ col,
                                                uint32_t* __restrict__ rev) {
  const uint32_t u = blockIdx.x * TB + threadIdx.x;
  if (u >= N) return;
  for (uint64_t e = row[u]; e < row[u + 1]; e++) {
    const uint32_t w = col[e];
    uint64_t lo = row[w], hi = row[w + 1];
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (col[mid] < u) lo = mid + 1; else hi = mid;
    }
    rev[e] = (uint32_t)lo;
  }
}

inline unsigned blocks(uint64_t n) { return (unsigned)((n + TB - 1) / TB); }

}  // namespace

void device_exclusive_scan(Ctx& c, const uint64_t* in, uint64_t* out, uint32_t n) {
  size_t tmp = 0;
  GS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, n, c.stream));
  DevBuf<uint8_t> t;
  t.alloc(tmp ? tmp : 1);
  GS_HIP(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, in, out, n, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
}

void launch_topology(Ctx& c) {
  const uint32_t N = c.cfg.peers, k = c.k;
  const uint64_t Nk = (uint64_t)N * k;
  hipStream_t s = c.stream;
  c.d_dial.alloc(Nk);
  c.d_acc.alloc(Nk);
  GS_HIP(hipMemsetAsync(c.d_acc.p, 1, Nk, s));
  k_dials<<<blocks(N), TB, 0, s>>>(N, k, c.cfg.seed, c.d_dial.p);
  GS_HIP(hipGetLastError());

  DevBuf<uint64_t> cnt, off, fill, tmp;
  cnt.alloc((size_t)N + 1);
  off.alloc((size_t)N + 1);
  fill.alloc(N);
  if (c.cfg.max_connections) {
    const uint32_t quota = c.cfg.max_connections > k ? c.cfg.max_connections - k : 0;
    GS_HIP(hipMemsetAsync(cnt.p, 0, ((size_t)N + 1) * 8, s));
    GS_HIP(hipMemsetAsync(fill.p, 0, (size_t)N * 8, s));
    k_inbound_count<<<blocks(Nk), TB, 0, s>>>(Nk, k, c.d_dial.p, cnt.p);
    device_exclusive_scan(c, cnt.p, off.p, N + 1);
    tmp.alloc(Nk);
    k_inbound_scatter<<<blocks(Nk), TB, 0, s>>>(N, k, c.d_dial.p, off.p, fill.p, tmp.p);
    k_inbound_accept<<<blocks(N), TB, 0, s>>>(N, k, quota, c.d_dial.p, off.p, tmp.p, c.d_acc.p);
    GS_HIP(hipGetLastError());
  }
  // half-edge buckets
  GS_HIP(hipMemsetAsync(cnt.p, 0, ((size_t)N + 1) * 8, s));
  GS_HIP(hipMemsetAsync(fill.p, 0, (size_t)N * 8, s));
  k_deg<<<blocks(Nk), TB, 0, s>>>(N, k, c.d_dial.p, c.d_acc.p, cnt.p);
  device_exclusive_scan(c, cnt.p, off.p, N + 1);
  uint64_t he_n = 0;
  GS_HIP(hipMemcpy(&he_n, off.p + N, 8, hipMemcpyDeviceToHost));
  DevBuf<uint64_t> he, ndeg;
  he.alloc(he_n ? he_n : 1);
  ndeg.alloc((size_t)N + 1);
  k_half_edges<<<blocks(Nk), TB, 0, s>>>(N, k, c.d_dial.p, c.d_acc.p, off.p, fill.p, he.p);
  GS_HIP(hipMemsetAsync(ndeg.p, 0, ((size_t)N + 1) * 8, s));
  k_sort_dedupe<<<blocks(N), TB, 0, s>>>(N, off.p, he.p, ndeg.p);
  c.d_row.alloc((size_t)N + 1);
  device_exclusive_scan(c, ndeg.p, c.d_row.p, N + 1);
  GS_HIP(hipMemcpy(&c.nnz, c.d_row.p + N, 8, hipMemcpyDeviceToHost));
  if (c.nnz >= (1ull << 32)) c.fail(GS_EUNSUPPORTED, "graph has >= 2^32 entries");
  c.d_col.alloc(c.nnz ? c.nnz : 1);
  c.d_flags.alloc(c.nnz ? c.nnz : 1);
  c.d_rev.alloc(c.nnz ? c.nnz : 1);
  DevBuf<unsigned> md;
  md.alloc(1);
  GS_HIP(hipMemsetAsync(md.p, 0, 4, s));
  k_compact<<<blocks(N), TB, 0, s>>>(N, off.p, he.p, c.d_row.p, c.d_col.p, c.d_flags.p, md.p);
  k_reverse<<<blocks(N), TB, 0, s>>>(N, c.d_row.p, c.d_col.p, c.d_rev.p);
  GS_HIP(hipGetLastError());
  unsigned maxdeg = 0;
  GS_HIP(hipMemcpyAsync(&maxdeg, md.p, 4, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  c.max_degree = maxdeg;
}

}  // namespace gs
