// gs_layout.h — the partition arithmetic of gs_run_partitioned,
// shared by the loop-back and the RCCL branches of gs_comm.hip so that both
// move the same blocks. Host-only, no HIP: tests/test_host_cpu.py compiles it
// with g++ and checks the exchanges for uneven splits and B < P on the CPU.
#pragma once
#include <stdint.h>

namespace gs {

struct PartLayout {
  uint32_t P, N, B;  // parts, peers, messages of the batch
  // part p owns peers [u0(p), u0(p + 1)) (1-D block partition)
  uint32_t u0(uint32_t p) const { return (uint32_t)((uint64_t)p * N / P); }
  uint32_t un(uint32_t p) const { return u0(p + 1) - u0(p); }
  // the part owning peer x: u0(p) <= x < u0(p + 1) (k_lpack_route / k_roff_fix compute the same)
  uint32_t part_of(uint32_t x) const { return (uint32_t)((((uint64_t)x + 1) * P - 1) / N); }
  // message-sharded batch (§5.3): part p simulates messages [m0(p), m0(p + 1))
  uint32_t m0(uint32_t p) const { return (uint32_t)((uint64_t)p * B / P); }
  uint32_t mn(uint32_t p) const { return m0(p + 1) - m0(p); }
  uint32_t mmax() const { return (B + P - 1) / P; }
  // all-to-all of a message-sharded batch: part s's results [mn(s)][N] are
  // packed per destination d as a block [mn(s)][un(d)] at ms_send_off(s, d)
  // of s's send buffer; d stores it at ms_recv_off(s, d) of its rows
  // [B][un(d)] (message-major over its own peers)
  uint64_t ms_send_off(uint32_t s, uint32_t d) const { return (uint64_t)mn(s) * u0(d); }
  uint64_t ms_count(uint32_t s, uint32_t d) const { return (uint64_t)mn(s) * un(d); }
  uint64_t ms_recv_off(uint32_t s, uint32_t d) const { return (uint64_t)m0(s) * un(d); }
};

// List-pass record exchange: part p's packed records of a pass land at
// base[p] of every part's gathered buffer (base[P] = the total), and its
// per-peer counts / offsets at its peers' global ids u0(p) ...
inline uint64_t lp_bases(const uint64_t* counts, uint32_t P, uint64_t* base) {
  base[0] = 0;
  for (uint32_t p = 0; p < P; p++) base[p + 1] = base[p] + counts[p];
  return base[P];
}

constexpr uint32_t PART_ROUTE_PMAX = 16;  // = gs_lpull_kernel.h LP_PMAX (k_lpack_route's LDS per destination)

// Routed list-pass record exchange (the default for P <= PART_ROUTE_PMAX): part p sends
// part q only its records with a receiver in q; route[p * P + q] counts them
// (route[q * P + q] = all of q's records). Part q's gathered buffer holds its
// own records first (base 0), then every other part's routed records in
// ascending part order; a sender's per-peer offsets are relative to its
// segment, the receiver adds base[p] (k_roff_fix). Returns the buffer's size.
inline uint64_t lp_route_bases(const uint64_t* route, uint32_t P, uint32_t q, uint64_t* base) {
  uint64_t b = route[(size_t)q * P + q];
  for (uint32_t p = 0; p < P; p++) {
    if (p == q) {
      base[p] = 0;
      continue;
    }
    base[p] = b;
    b += route[(size_t)p * P + q];
  }
  return b;
}

}  // namespace gs
