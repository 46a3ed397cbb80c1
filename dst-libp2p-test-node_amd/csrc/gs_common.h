// gs_common.h — spec-level constants and pure functions shared by the host
// code and the gfx950 kernels of libgossipsim. Nothing here
// touches the device; kernels include it for the inline helpers.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GS_HD __host__ __device__ __forceinline__
#else
#define GS_HD static inline
#endif

namespace gs {

constexpr uint64_t INF64 = ~0ull;
constexpr uint32_t EMPTY = ~0u;
constexpr uint32_t MESH_W = 16;       // ELL width of the frozen mesh (GS_MESH_W)
constexpr uint32_t HOP_BITS = 6;      // key = t_rel | hops | src
constexpr uint32_t MAX_STAGES = 16;   // link classes (topogen -st), LDS-resident
constexpr uint32_t MAX_DIALS = 64;    // dials per peer held in registers/scratch
constexpr uint32_t MAX_DEG = 256;     // per-row working sets of the mesh kernels
constexpr uint32_t GT_W = 8;          // gossip target selection: pairs kept sorted in registers
constexpr uint32_t GT_IN = 16;        // lazy gossip + churn: IHAVE senders kept per (peer, epoch)
constexpr uint32_t GT_REDO = 0xFFFFFFFEu;  // entry 0 of such a list: more senders than it holds
constexpr uint32_t MAX_FRAGS = 16;    // FRAGMENTS (topogen allows 1..9)
constexpr uint32_t STAGE_SHIFT = 24;  // packed mesh entry: stage << 24 | peer
// Subscription exchange: a connection completes HS_RTTS round
// trips after the common dial instant (TCP + multistream + Noise XX + yamux, a
// model constant); w's subscription then reaches u one lat(w->u) later.
constexpr uint32_t HS_RTTS = 3;  // default of gs_config.hs_rtts

enum : uint32_t { P_DIAL = 1, P_DIAL_ORDER = 2, P_GRAFT = 3, P_PRUNE = 4, P_OUT_GRAFT = 5, P_GOSSIP = 6, P_CHURN = 7,
                  P_MSGID = 8 };
enum : uint32_t { NODE_RUST = 0, NODE_GO = 1, NODE_NIM = 2 };  // GS_NODE_*
enum : uint8_t { F_OUT = 1, F_MESH = 2 };
enum : uint8_t { PR_GRAFT = 1, PR_PRUNE = 2, PR_ACCEPT = 4 };

// Counter-based RNG: a pure function of (seed, purpose, a, b, c). Replaces
// the unseeded rand::rng() of rust-test-node/src/main.rs:308 so the device
// and the CPU oracle draw identical streams.
GS_HD uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  z ^= z >> 31; return z;
}
GS_HD uint64_t rng(uint64_t seed, uint32_t purpose, uint32_t a, uint32_t b, uint32_t c) {
  uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(purpose + 1u));
  h = mix64(h ^ ((uint64_t)a + 0x9E3779B97F4A7C15ull));
  h = mix64(h ^ ((((uint64_t)b) << 32) | c) ^ 0xD6E8FEB86659FD93ull);
  return h;
}
// The same draw in two parts: rng_fin(rng_pre(seed, purpose, a), b, c) ==
// rng(seed, purpose, a, b, c); a loop over (b, c) of one `a` mixes once per draw.
GS_HD uint64_t rng_pre(uint64_t seed, uint32_t purpose, uint32_t a) {
  return mix64(mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(purpose + 1u)) ^ ((uint64_t)a + 0x9E3779B97F4A7C15ull));
}
GS_HD uint64_t rng_fin(uint64_t pre, uint32_t b, uint32_t c) {
  return mix64(pre ^ ((((uint64_t)b) << 32) | c) ^ 0xD6E8FEB86659FD93ull);
}
GS_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
// Uniform draw in [0, n) (multiply-high; bias <= n / 2^64).
GS_HD uint64_t rand_below(uint64_t x, uint64_t n) { return mulhi64(x, n); }

// Churn: peer u is offline during heartbeat epoch h >= 1 iff
// a departure was drawn at one of the epochs h-down+1..h.
GS_HD bool offline_draw(uint64_t seed, uint32_t ppm, uint32_t down, uint32_t u, uint64_t h) {
  if (!ppm || h == 0) return false;
  for (uint64_t k = 0; k < down && k < h; k++)
    if (rand_below(rng(seed, P_CHURN, u, (uint32_t)(h - k), 0), 1000000) < ppm) return true;
  return false;
}

GS_HD uint32_t bits_for(uint32_t n) { uint32_t b = 1; while ((1ull << b) < n) b++; return b; }

// Dials per peer: min(CONNECTTO + dial_extra, min(2*CONNECTTO, N-1))
// (rust-test-node/src/main.rs:314,337; nim gossipsub-queues/main.nim:396).
GS_HD uint32_t dials_per_peer(uint32_t peers, uint32_t connect_to, uint32_t dial_extra) {
  uint64_t lim = 2ull * connect_to;
  if (lim > (uint64_t)peers - 1) lim = peers - 1;
  uint64_t k = (uint64_t)connect_to + dial_extra;
  return (uint32_t)(k < lim ? k : lim);
}

// Fragment layout per node flavour:
//  rust publish_new_message (main.rs:109-121): msg_size/F bytes, i64 stamp in
//    [0..8) (panics below 8 B), byte 10 = chunk only when the buffer is > 10 B
//    (else every fragment is identical: one msg-id, defect D8);
//  go publishNewMessage (go-test-node/main.go:63-74): 8-byte stamp + msg_size/F
//    bytes, payload[10] = chunk (index out of range when msg_size/F <= 2);
//  nim publishNewMessage (nim gossipsub-queues/main.nim:158-175): 16-byte
//    header + msg_size div F - 16 bytes, nowBytes[16] = chunk (IndexDefect
//    when msg_size div F <= 16).
GS_HD uint64_t frag_payload(uint32_t node, uint64_t msg_size, uint32_t F) {
  return msg_size / F + (node == NODE_GO ? 8 : 0);
}
GS_HD bool frag_invalid(uint32_t node, uint64_t msg_size, uint32_t F) {
  const uint64_t q = msg_size / F;
  return node == NODE_GO ? q <= 2 : node == NODE_NIM ? q <= 16 : q < 8;
}
GS_HD bool frag_collide(uint32_t node, uint64_t msg_size, uint32_t F) {
  return node == NODE_RUST && F > 1 && msg_size / F <= 10;
}

// Serialisation time in ns of `bytes` at `bps` (ceil).
GS_HD uint64_t ser_ns(uint64_t bytes, uint64_t bps) { return (bytes * 8000000000ull + bps - 1) / bps; }

}  // namespace gs
