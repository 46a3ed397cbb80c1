/*
 * gs_oracle.h — CPU oracle for the GossipSub dissemination hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product (libgossipsim.so) never links it.
 *
 * The reference's arithmetic lives in third-party libp2p-gossipsub 0.49.2
 * (rust-test-node/Cargo.lock:1640-1666) and Shadow v3.3.0
 * (shadow/Dockerfile:38), neither vendored; the reference holds no tests or
 * golden vectors for this path. This file restates the
 * rules of DESIGN.md §2 single-threaded and sequentially (binary-heap event
 * simulation), independently of the GPU's Delta-stepping kernels.
 * Pinned: link tables (vs topogen.py outputs) and the log format (vs the awk
 * summaries). Dissemination/mesh rules: parity unpinned (no reference oracle).
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_params {
    uint32_t peers, connect_to, dial_extra, max_connections, fragments;
    uint32_t muxer, signed_msgs;
    uint32_t d, d_lo, d_hi, d_lazy, d_out, gossip_factor_milli;
    uint64_t heartbeat_ns, backoff_ns;
    uint32_t flood_publish, idontwant, lazy_gossip, self_log;
    uint64_t seed;
    uint32_t history_gossip;
    uint64_t hb_phase_ns;
    uint32_t churn_ppm, churn_down, churn_horizon; /* DESIGN.md §2.8; 0 ppm = no churn */
    uint32_t node; /* payload layout of the node flavour: 0 rust, 1 go, 2 nim */
    uint32_t sub_graft; /* subscription-time grafting before heartbeat 1 */
    uint32_t hs_rtts;   /* handshake round trips before the subscriptions (0 = 3) */
} or_params;

typedef struct or_stats {
    uint64_t messages, deliveries, frag_deliveries, relaxations, bytes_alg;
    uint64_t latency_sum_ms, latency_max_ms;
    uint64_t gossip_iwant;
} or_stats;

uint64_t or_rng(uint64_t seed, uint32_t purpose, uint32_t a, uint32_t b, uint32_t c);
uint64_t or_wire_bytes(uint64_t payload, uint32_t muxer, uint32_t signed_msgs);
void or_wire_packets(uint64_t payload, uint32_t muxer, uint32_t signed_msgs, uint64_t* packets,
                     uint64_t* header_bytes);
/* kind 0 IHAVE, 1 IWANT (one message id), 2 a pure ACK packet. */
void or_ctrl_packets(uint32_t kind, uint32_t node, uint32_t muxer, uint64_t* bytes, uint64_t* packets,
                     uint64_t* header_bytes);
/* Per-peer traffic columns (the C ABI's GS_TR_*). */
#define OR_TR_COLS 12
int or_run_traffic(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                   const uint32_t* mesh, const uint8_t* cnt, const uint8_t* stage, uint32_t S,
                   const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
                   const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
                   const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops, struct or_stats* st, uint64_t* tr);
int or_run_churn_traffic(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                         const uint32_t* snap_mesh, const uint8_t* snap_cnt, const uint8_t* snap_off,
                         uint32_t h_lo, uint32_t n_snap, const uint8_t* stage, uint32_t S,
                         const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
                         const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
                         const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops,
                         struct or_stats* st, uint64_t* tr);
int or_topogen_links(uint32_t S, uint32_t bl, uint32_t bh, uint32_t ll, uint32_t lh,
                     uint32_t mode, uint64_t* lat_ns, uint64_t* bw_bps);
uint32_t or_dials_per_peer(const or_params* p);
/* row_ptr[N+1], col/flags capacity 2*k*N; returns 0 or negative error. */
int or_build_topology(const or_params* p, uint64_t* row_ptr, uint32_t* col, uint8_t* flags,
                      uint64_t* nnz_out);
/* flags in/out (bit1 = in mesh); mesh[N*16] ascending ids, cnt[N]. */
int or_mesh_converge(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                     uint8_t* flags, const uint8_t* stage, uint32_t S, const uint64_t* lat_ns,
                     uint32_t max_hb, uint32_t* mesh, uint8_t* cnt, uint32_t* epochs_out);
/* 1 if peer u is offline during heartbeat epoch h (churn). */
int or_offline(const or_params* p, uint32_t u, uint64_t h);
/* Mesh snapshots for heartbeat epochs [h_lo, h_hi] under churn: snap_mesh
 * [(h_hi-h_lo+1)][N*16], snap_cnt / snap_off [(h_hi-h_lo+1)][N]. */
int or_mesh_churn(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, const uint8_t* flags,
                  const uint8_t* stage, uint32_t S, const uint64_t* lat_ns, uint32_t h_lo, uint32_t h_hi,
                  uint32_t* snap_mesh, uint8_t* snap_cnt, uint8_t* snap_off);
/* or_run over a time-varying mesh: the snapshot of the epoch each send falls
 * in; events past epoch(t_pub) + churn_horizon are dropped. */
int or_run_churn(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                 const uint32_t* snap_mesh, const uint8_t* snap_cnt, const uint8_t* snap_off,
                 uint32_t h_lo, uint32_t n_snap, const uint8_t* stage, uint32_t S,
                 const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
                 const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
                 const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops, or_stats* st);
/* sched_frags: chunks per message (main.rs:65-71), NULL or 0 entries = p->fragments. */
int or_run(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
           const uint32_t* mesh, const uint8_t* cnt, const uint8_t* stage, uint32_t S,
           const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
           const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
           const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops, or_stats* st);

/* or_run on `threads` host threads, messages in parallel (bench.py's all-core baseline). */
int or_run_mt(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
              const uint32_t* mesh, const uint8_t* cnt, const uint8_t* stage, uint32_t S,
              const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
              const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
              const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops, or_stats* st,
              int threads);

#ifdef __cplusplus
}
#endif
#endif
