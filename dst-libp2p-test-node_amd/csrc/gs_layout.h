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

}  // namespace gs
