/*
 * gossipsim.h — C ABI of the MI355X-native GossipSub dissemination simulator.
 *
 * This is the drop-in boundary for the reference's hot path: message
 * dissemination across the GossipSub peer mesh of vacp2p/dst-libp2p-test-node.
 * In the reference that path sits behind rust-libp2p's NetworkBehaviour
 * (libp2p-gossipsub 0.49.2, not vendored; pinned at
 * rust-test-node/Cargo.lock:1640) and is driven by rust-test-node/src/main.rs.
 * Every entry point below names the reference interface it replaces.
 *
 * Conventions
 *  - Plain C: fixed-width integers, plain pointers and sizes, no C++ types.
 *  - Every call returns gs_status (0 = OK, negative = error); the message of the
 *    last failure is available from gs_last_error(ctx). No exception crosses
 *    the ABI.
 *  - The caller owns every host array it passes in; the library owns the
 *    device buffers of a context.
 *  - A context is bound to ONE HIP device and is not thread-safe: use one host
 *    thread per context. Multi-GPU = one context per GPU, each simulating its
 *    own message shard (message batches are independent).
 *  - All simulated times are integer nanoseconds.
 */
#ifndef GOSSIPSIM_H
#define GOSSIPSIM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 10u

/* Sentinel for "never delivered" in t_complete_ns. */
#define GS_UNDELIVERED UINT64_MAX

typedef int32_t gs_status;
enum {
    GS_OK = 0,
    GS_EINVAL = -1,       /* bad argument / knob combination               */
    GS_ENOMEM = -2,       /* host or device allocation failed              */
    GS_EDEVICE = -3,      /* HIP runtime error or no usable device         */
    GS_ESTATE = -4,       /* call out of order (e.g. run before topology)  */
    GS_ERANGE = -5,       /* a packed field overflowed (time, hops, mesh)  */
    GS_EUNSUPPORTED = -6  /* knob recognised but not implemented yet       */
};

/* MUXER (rust-test-node/src/env.rs:48-50,69-71; nim adds mplex,
 * nim-test-node/gossipsub-queues/main.nim:433-441). */
enum { GS_MUX_YAMUX = 0, GS_MUX_QUIC = 1, GS_MUX_MPLEX = 2 };

/* Node flavour whose gossipsub settings, payload layout and log line the
 * simulator reproduces (gs_config_preset): rust-test-node (the north star),
 * go-test-node, nim-test-node/gossipsub-queues. */
enum { GS_NODE_RUST = 0, GS_NODE_GO = 1, GS_NODE_NIM = 2 };

/* Link-table mode for gs_topogen_links. */
enum {
    GS_LINKS_DIRECT = 0,   /* latency of the direct GML edge (topogen intent)       */
    GS_LINKS_SHORTEST = 1  /* shortest path over the GML graph incl. injector hub  */
};

/* Simulator configuration. Field meaning follows the reference's knobs:
 * rust-test-node/src/env.rs:27-87 (PEERS, CONNECTTO, FRAGMENTS, MUXER) and
 * rust-test-node/src/main.rs:223-241 (gossipsub ConfigBuilder). */
typedef struct gs_config {
    uint32_t abi_version;        /* must be GS_ABI_VERSION                         */
    uint32_t peers;              /* PEERS (env.rs:38-41)                           */
    uint32_t connect_to;         /* CONNECTTO (env.rs:43-46)                       */
    uint32_t dial_extra;         /* 1: rust/go dial CONNECTTO+1 (main.rs:337); 0: nim */
    uint32_t max_connections;    /* MAXCONNECTIONS inbound cap (nim main.nim:429); 0 = none */
    uint32_t fragments;          /* FRAGMENTS (env.rs:64-67)                       */
    uint32_t muxer;              /* GS_MUX_*                                       */
    uint32_t signed_msgs;        /* 1: MessageAuthenticity::Signed (main.rs:397)   */
    uint32_t d;                  /* mesh_n      (main.rs:231)                       */
    uint32_t d_lo;               /* mesh_n_low  (main.rs:232)                       */
    uint32_t d_hi;               /* mesh_n_high (main.rs:233)                       */
    uint32_t d_lazy;             /* gossip_lazy (main.rs:235)                       */
    uint32_t d_out;              /* mesh_outbound_min (main.rs:234)                 */
    uint32_t gossip_factor_milli;/* gossip_factor x 1000 (main.rs:230)              */
    uint64_t heartbeat_ns;       /* heartbeat_interval (main.rs:228)                */
    uint64_t backoff_ns;         /* prune_backoff (main.rs:229)                     */
    uint32_t flood_publish;      /* flood_publish (main.rs:227)                     */
    uint32_t idontwant;          /* IDONTWANT suppression (go main.go:165); 0 = off */
    uint32_t lazy_gossip;        /* IHAVE/IWANT gossip relaxations; 0 = off         */
    uint32_t self_log;           /* publisher logs its own message (nim SELFTRIGGER)*/
    uint64_t seed;               /* counter-RNG key (reference RNG is unseeded, main.rs:308) */
    int32_t  device;             /* HIP device ordinal                              */
    uint32_t batch;              /* messages simulated together per device batch    */
    uint32_t history_gossip;     /* mcache windows gossiped (upstream default 3)    */
    uint64_t hb_phase_ns;        /* heartbeats at hb_phase + h*heartbeat (absolute) */
    /* churn (BASELINE config #3; build-defined): each heartbeat
     * epoch every peer starts a churn_down-epoch outage with probability
     * churn_ppm / 1e6; the mesh evolves epoch by epoch and every send uses the
     * mesh of its epoch. 0 = frozen converged mesh. Needs hb_phase_ns within
     * 2^20 heartbeats of every publish. */
    uint32_t churn_ppm;
    uint32_t churn_down;         /* outage length in heartbeats (default 10)        */
    uint32_t churn_horizon;      /* message lifetime in heartbeats under churn: no  */
                                 /* event past epoch(t_pub) + horizon (default 16)  */
    uint32_t node;               /* GS_NODE_*: fragment layout + log line */
    /* subscription-time grafting (libp2p-gossipsub handle_received_subscriptions,
     * reached through the 20 s connection pump of main.rs:357-379): before
     * heartbeat 1 every peer grafts its first D_lo connections in handshake
     * order. 1 in the rust preset. */
    uint32_t sub_graft;
    /* round trips from the common dial instant until a connection carries its
     * first subscription (TCP + multistream + Noise XX + yamux; a model
     * constant of the subscription epoch); 0 = 3 (default) */
    uint32_t hs_rtts;
} gs_config;

/* One publish injection (replaces POST /publish, main.rs:50-56,152-168; the
 * PublishCommand of main.rs:65-71 carries msg_size and chunks). */
typedef struct gs_publish {
    uint64_t t_pub_ns;    /* absolute publish time = tx_time stamped at main.rs:105-111 */
    uint32_t publisher;   /* peer id that publishes                                     */
    uint32_t msg_size;    /* msgSize of the request; fragment payload = msg_size/F      */
    uint32_t frags;       /* F of this message (chunks, main.rs:163-168); 0 = cfg.fragments */
    uint32_t reserved;    /* 0                                                          */
} gs_publish;

/* Latency histogram bins of gs_msg_summary: 100 ms each (hop_lat of
 * shadow/summary_latency.awk:8), the last one open-ended. */
#define GS_HIST_BINS 64u
#define GS_HIST_MS 100u

/* Per-message reduction of one run, computed on the device:
 * latency = (t_complete - tx_time) / 1e6 truncated, as logged (main.rs:91-93),
 * over the peers that log the message (the publisher only with self_log). */
typedef struct gs_msg_summary {
    uint64_t delivered;            /* log lines of this message                          */
    uint64_t lat_sum_ms;
    uint32_t p50_ms, p95_ms;       /* nearest-rank percentiles: value at rank ceil(q*n)  */
    uint32_t max_ms;
    uint32_t reserved;
    uint32_t hist[GS_HIST_BINS];   /* hist[min(ms / 100, 63)]                            */
} gs_msg_summary;

/* Streaming receiver of results: called from gs_run on the caller's thread
 * with message-major blocks of at most `block_msgs` messages; the arrays are
 * library-owned and valid only during the call ([n_msgs][peers], either may
 * be NULL when gs_result_sink.want does not select it). */
typedef void (*gs_block_fn)(void* user, uint64_t first_msg, uint32_t n_msgs, uint32_t peers,
                            const uint64_t* t_complete_ns, const uint8_t* hops);

/* Streaming receiver of the logged latency (GS_WANT_LAT_MS, ABI 9): the
 * value each peer's log line carries, (t_complete - tx_time) / 1e6 truncated
 * (rust-test-node/src/main.rs:91-93), message-major [n_msgs][peers] u16;
 * GS_LAT_NONE where the peer logs nothing (undelivered; the publisher unless
 * cfg.self_log). 2 bytes per (peer, message) instead of the 9 of
 * t_complete + hops. A latency of 65535 ms or more fails the run (GS_ERANGE). */
typedef void (*gs_lat_fn)(void* user, uint64_t first_msg, uint32_t n_msgs, uint32_t peers, const uint16_t* lat_ms);
#define GS_LAT_NONE 0xFFFFu

/* Outputs a streaming sink delivers (gs_result_sink.want): t_complete and
 * hops through on_block, the logged latency through on_lat. */
enum { GS_WANT_T_COMPLETE = 1u, GS_WANT_HOPS = 2u, GS_WANT_LAT_MS = 4u };

/* Where gs_run puts results. Every member may be NULL / 0.
 *  - t_complete_ns / hops: caller arrays, message-major [n_msgs][peers];
 *    without on_block only; they must be NULL when on_block is set
 *    (GS_EINVAL otherwise: nothing is ever written through them then);
 *  - on_block: streaming delivery instead of the arrays (no [n_msgs][peers]
 *    host array is needed for large N); `want` selects what it receives
 *    (GS_WANT_* bits, 0 = both); ABI 7 (ABI 6 used non-NULL array pointers
 *    as the selection flags);
 *  - summary: [n_msgs] per-message latency reductions;
 *  - on_lat: the logged latency in ms, u16, streamed in the same blocks; set
 *    iff want has GS_WANT_LAT_MS (ABI 9). gs_run only (gs_run_partitioned
 *    returns GS_EUNSUPPORTED). */
typedef struct gs_result_sink {
    uint64_t* t_complete_ns;  /* completion time of message m at peer u (GS_UNDELIVERED if never) */
    uint8_t*  hops;           /* hop count of the completing fragment (0 at the publisher)        */
    gs_block_fn on_block;
    void*     user;
    uint32_t  block_msgs;     /* messages per on_block call; 0 = 64                               */
    uint32_t  want;           /* GS_WANT_T_COMPLETE | GS_WANT_HOPS (on_block; neither = both)     */
                              /* | GS_WANT_LAT_MS (on_lat)                                        */
    gs_msg_summary* summary;
    gs_lat_fn on_lat;         /* ABI 9: the logged latency stream (GS_WANT_LAT_MS)                */
} gs_result_sink;

/* Counters accumulated since gs_create / gs_reset_stats. */
typedef struct gs_stats {
    uint64_t messages;          /* messages simulated                                  */
    uint64_t deliveries;        /* (peer,msg) completions at non-publishers = log lines */
    uint64_t frag_deliveries;   /* FD: fragment first arrivals at non-publishers       */
    uint64_t relaxations;       /* R: flood-publish sends + forward sends (dups incl.) */
    uint64_t bytes_alg;         /* 16*FD + 12*R + 8*deliveries           */
    uint64_t latency_sum_ms;    /* sum of per-delivery latency in ms (truncated)       */
    uint64_t latency_max_ms;    /* max per-delivery latency in ms                      */
    uint64_t relax_launches;    /* bucket-relaxation kernel launches                   */
    uint64_t buckets;           /* non-empty Delta-buckets processed                   */
    double   relax_ms;          /* device time of relaxation launches (timing on)      */
    double   run_ms;            /* device time of whole gs_run calls (timing on)       */
    uint64_t relax_bytes_alg;   /* 16*FD + 12*R_forward: algorithmic bytes of relax    */
    uint64_t pushes;            /* atomicMin pushes issued (forward sends not dropped  */
                                /* because the target was already final)              */
    double   scan_ms;           /* relax_ms split: bucket scan + compaction kernel     */
    double   frontier_ms;       /* relax_ms split: frontier forwarding kernel          */
    uint64_t gossip_iwant;      /* IWANT responses sent (counted in relaxations too)   */
    uint64_t gossip_noop_msgs;  /* lazy gossip on the pull path: messages proven to      */
                                /* finish everywhere before their first IHAVE can land    */
                                /* (no IWANT possible)                   */
    uint64_t gossip_fallback_batches; /* batches re-run on the push path with gossip    */
    uint64_t batches;           /* device batches run (gs_run splits at cfg.batch, size /  */
                                /* chunk changes and the churn snapshot ring)             */
    uint64_t list_pull_batches; /* batches whose eager passes ran on candidate lists      */
                                /* (k_lpull) rather than dense rows       */
    uint64_t ms_batches;        /* gs_run_partitioned batches run message-sharded (ABI 8) */
    uint64_t gossip_list_batches; /* batches whose lazy gossip ran inside the list pass    */
                                /* (IHAVE / IWANT decided per window, ABI 9; §2.7)        */
} gs_stats;

/* ---- host-only helpers (no device work) ---------------------------------- */

/* Defaults of the rust preset (main.rs:36-38,223-241; env.rs:38-67). */
void gs_config_default(gs_config* cfg);

/* Overwrite cfg with the defaults of one node flavour (gs_config_default +
 * the node's own settings):
 *  GS_NODE_RUST  rust-test-node/src/main.rs:223-241 (= gs_config_default);
 *  GS_NODE_GO    go-test-node/main.go:153-175,374-385: Dout 2, IDONTWANT
 *                threshold 1000 B, StrictNoSign (unsigned), local delivery of
 *                own messages (self log), 8-byte stamp + msg_size/F payload;
 *  GS_NODE_NIM   nim-test-node/gossipsub-queues/main.nim:242-332,396,429:
 *                CONNECTTO dials (no +1), MAXCONNECTIONS 250, Dout = D/2,
 *                anonymize (unsigned), SELFTRIGGER, 16-byte header, log line
 *                keyed by msgId.
 * Returns GS_EINVAL for an unknown node. */
gs_status gs_config_preset(gs_config* cfg, uint32_t node);

/* Read the reference's env surface into cfg: PEERS, CONNECTTO, FRAGMENTS,
 * MUXER (env.rs:38-67), MAXCONNECTIONS (nim main.nim:429), GOSSIPSUB_D,
 * _D_LOW, _D_HIGH, _D_LAZY, _D_OUT, _HEARTBEAT_MS, _PRUNE_BACKOFF_SEC,
 * _GOSSIP_FACTOR, _FLOOD_PUBLISH (nim main.nim:252-284), SELFTRIGGER, plus
 * GS_SEED / GS_BATCH / GS_DEVICE. GS_NODE=rust|go|nim first applies that
 * node's preset (gs_config_preset). Validation mirrors env.rs:69-75:
 * unknown muxer and CONNECTTO >= PEERS are errors (message in err). */
gs_status gs_config_from_env(gs_config* cfg, char* err, size_t err_len);

/* Wire bytes of one fragment of `payload` bytes on one hop. */
uint64_t gs_wire_bytes(uint64_t payload, uint32_t muxer, uint32_t signed_msgs);

/* Stage link tables from topogen.py's parameters (shadow/topogen.py:39-71):
 * lat_ns[S*S] (row = sender stage), bw_bps[S] (up == down). */
gs_status gs_topogen_links(uint32_t stages, uint32_t min_bw_mbit, uint32_t max_bw_mbit,
                           uint32_t min_lat_ms, uint32_t max_lat_ms, uint32_t mode,
                           uint64_t* lat_ns, uint64_t* bw_bps);

/* Link tables from a Shadow network graph file (network_topology.gml as
 * shadow/topogen.py:39-71 writes it: node host_bandwidth_up/down, edge latency;
 * units bit/Kbit/Mbit/Gbit, ns/us/ms/s). Every GML node becomes one link class,
 * so V = *nodes classes: lat_ns[V*V], bw_up_bps[V], bw_down_bps[V]. mode as
 * gs_topogen_links (GS_LINKS_DIRECT needs an edge for every pair). Returns
 * GS_ERANGE with *nodes = V when V > max_nodes (call again with room), and
 * GS_EUNSUPPORTED for a non-zero packet_loss (not modelled). */
gs_status gs_links_from_gml(const char* gml_path, uint32_t mode, uint32_t max_nodes, uint32_t* nodes,
                            uint64_t* lat_ns, uint64_t* bw_up_bps, uint64_t* bw_down_bps);

/* Peer -> link class from a Shadow config (shadow.yaml as topogen.py:73-139
 * writes it): host "pod-<id>" (the id parse of rust env.rs:34-36) ->
 * network_node_id, incl. YAML anchors/aliases; hosts with id >= peers (the
 * injector) are skipped; a peer without a host is GS_EINVAL. */
gs_status gs_shadow_hosts(const char* yaml_path, uint32_t peers, uint8_t* stage_of_peer);

/* The publish injector of a Shadow config (shadow.yaml as topogen.py:125-136
 * writes it): the controller host's process `args`
 * "traffic_sync.py -s <msg_size> -m <messages> -d <delay> -n <peers> ..." and
 * its start_time. The delay is read in milliseconds, the unit shadow/run.sh:36
 * passes (topogen.py:26's help text says seconds). */
typedef struct gs_injector {
    uint64_t start_ns;    /* process start_time (500s in topogen.py:133)          */
    uint64_t delay_ns;    /* -d: inter-message delay                              */
    uint32_t msg_size;    /* -s                                                   */
    uint32_t messages;    /* -m                                                   */
    uint32_t peers;       /* -n                                                   */
    uint32_t reserved;
} gs_injector;
gs_status gs_shadow_injector(const char* yaml_path, gs_injector* out);

/* A publish schedule file: one row per message, "t_pub_ns publisher msg_size
 * [frags]" (whitespace separated, '#' comments). Returns GS_ERANGE with
 * *n = rows when cap is too small (call again with room), GS_EINVAL on a
 * malformed row. */
gs_status gs_read_schedule(const char* path, gs_publish* out, uint64_t cap, uint64_t* n);

/* Publish schedule of shadow/run.sh:34-36 (publisher_id, publisher_rotation,
 * inter_message_delay): row i = {t0 + i*delay, (pub0 + i*rotation) mod N, size}. */
gs_status gs_schedule_runsh(uint32_t n_msgs, uint32_t peers, uint32_t publisher_id,
                            uint32_t rotation, uint64_t t0_ns, uint64_t delay_ns,
                            uint32_t msg_size, gs_publish* out);

/* Write arrival lines exactly as `grep -rne 'milliseconds\|BW' shadow.data/`
 * would print them for rust nodes (main.rs:93; shadow/run.sh:61):
 *   shadow.data/hosts/peer<u>/main.1000.stdout:<line>:<tx_time> milliseconds: <ms>
 * grouped by peer in ascending id, line numbers counted per peer. */
gs_status gs_write_latency_log(const char* path, const gs_publish* sched, uint64_t n_msgs,
                               uint32_t peers, const uint64_t* t_complete_ns,
                               uint32_t self_log);

/* The same arrival log for the node flavour of cfg (peers, self_log, node,
 * seed): rust and go print "<tx_time> milliseconds: <ms>" (main.rs:93,
 * go-test-node/main.go:49); nim prints "<msgId> milliseconds: <ms>"
 * (nim gossipsub-queues/main.nim:150) with msgId a 63-bit id drawn from
 * (seed, publisher, t_pub) in place of the node's rand(high(int64)). */
gs_status gs_write_node_log(const gs_config* cfg, const char* path, const gs_publish* sched,
                            uint64_t n_msgs, const uint64_t* t_complete_ns);

/* Streaming arrival log (the same lines as gs_write_node_log) for runs too
 * large for a [n_msgs][peers] host array: feed it the message-major blocks of
 * gs_result_sink.on_block. Lines come out block by block (message-major within
 * a block) instead of grouped by peer; the per-peer line numbers count across
 * blocks exactly as the grouped writer counts them, so every line is
 * identical and the awk summaries are unchanged. */
typedef struct gs_log gs_log;
gs_status gs_log_open(const gs_config* cfg, const char* path, gs_log** out);
/* sched = the block's n_msgs schedule rows, t_complete_ns = [n_msgs][peers]. */
gs_status gs_log_write(gs_log* log, const gs_publish* sched, uint32_t n_msgs, const uint64_t* t_complete_ns);
/* The same from the u16 latency stream (gs_result_sink.on_lat, ABI 9):
 * lat_ms = [n_msgs][peers], GS_LAT_NONE where no line is written. */
gs_status gs_log_write_lat(gs_log* log, const gs_publish* sched, uint32_t n_msgs, const uint16_t* lat_ms);
gs_status gs_log_close(gs_log* log);

/* Packets and header bytes of one fragment send in the same model as
 * gs_wire_bytes: TCP/IPv4 segments of <= 1460 B carrying 40 B of headers each,
 * or QUIC packets of <= 1415 B carrying 65 B each. */
void gs_wire_packets(uint64_t payload, uint32_t muxer, uint32_t signed_msgs, uint64_t* packets,
                     uint64_t* header_bytes);

/* Wire size of one lazy-gossip control RPC carrying one message id (IHAVE:
 * RPC{control{ihave{topic "test", id}}}, IWANT: RPC{control{iwant{id}}}; the
 * id is 20 bytes for the rust / nim nodes' decimal hashes, 32 for go's sha256)
 * through the muxer stack, or one pure ACK packet (header only). */
enum { GS_CTRL_IHAVE = 0, GS_CTRL_IWANT = 1, GS_CTRL_ACK = 2 };
void gs_control_packets(uint32_t kind, uint32_t node, uint32_t muxer, uint64_t* bytes, uint64_t* packets,
                        uint64_t* header_bytes);

/* Columns of a per-peer traffic row (gs_get_traffic). Data columns count every
 * packet that carries bytes of a gossipsub RPC (message sends, IWANT answers,
 * IHAVE and IWANT control RPCs); the ctrl columns count the pure TCP/QUIC ACKs
 * (one per <= 2 data packets received, sent back to the sender). */
enum { GS_TR_TX_BYTES = 0, GS_TR_RX_BYTES = 1, GS_TR_TX_PKTS = 2, GS_TR_RX_PKTS = 3,
       GS_TR_TX_HDR = 4, GS_TR_RX_HDR = 5,
       GS_TR_RECEIVED = 6,   /* completed messages (main.rs:94 inc_received_message)   */
       GS_TR_PUBLISHED = 7,  /* messages published (main.rs:515 inc_messages_published) */
       GS_TR_TX_CTRL_PKTS = 8, GS_TR_RX_CTRL_PKTS = 9,  /* pure ACK packets            */
       GS_TR_TX_CTRL_HDR = 10, GS_TR_RX_CTRL_HDR = 11,  /* their (header-only) bytes    */
       GS_TRAFFIC_COLS = 12 };

/* Shadow's per-host heartbeat counters for the same runs, one "[node]" line
 * per peer as Shadow's tracker logs them (recv/send bytes, then inbound and
 * outbound localhost / remote packet, header and payload counters), so that
 * shadow/summary_shadowlog.awk:12-143 summarises them unchanged. traffic is
 * [peers][GS_TRAFFIC_COLS]. Host names are pod-<id> (topogen.py:118). */
gs_status gs_write_shadow_heartbeat(const char* path, uint32_t peers, const uint64_t* traffic,
                                    uint64_t sim_seconds);

/* The test node's Prometheus metrics (rust-test-node/src/metrics.rs:13-199,
 * names shared with the go and nim nodes) for every peer, in the OpenMetrics
 * text format prometheus-client encodes (counters with _total, "# EOF"), one
 * series per peer labelled peer="pod-<id>": connected / pubsub peers and
 * subscriptions = CSR degree, topics = 1, mesh peers = mesh_count, topic
 * health buckets against cfg->d_lo (metrics.rs:158-176), received / validated
 * and published messages from the traffic columns. Arrays are host copies:
 * row_ptr[peers+1] (gs_get_csr), mesh_count[peers] (gs_get_mesh),
 * traffic[peers][GS_TRAFFIC_COLS] (gs_get_traffic). */
gs_status gs_write_node_metrics(const gs_config* cfg, const char* path, const uint64_t* row_ptr,
                                const uint8_t* mesh_count, const uint64_t* traffic);

/* ---- context lifecycle (replaces SwarmBuilder + build_behaviour, main.rs:391-440) ---- */

gs_status gs_create(const gs_config* cfg, struct gs_ctx** out);
gs_status gs_destroy(struct gs_ctx* ctx);

/* Checkpoint / resume (no counterpart in the reference, whose
 * runs are single Shadow executions): gs_save_state writes the configuration,
 * link tables, CSR + mesh flags + PRUNE back-offs, the mesh ELL, the churn
 * mesh state's epoch, the counters and the per-peer traffic of a context to
 * `path`; gs_load_state makes a new context on `device` from such a file. A
 * schedule continued on the loaded context gives exactly the results and
 * counters the saved context would have given (every random draw is a pure
 * function of the seed: there is no generator state). GS_EINVAL for a file of
 * another ABI version or a damaged one. */
gs_status gs_save_state(struct gs_ctx* ctx, const char* path);
gs_status gs_load_state(const char* path, int32_t device, struct gs_ctx** out);
/* The configuration a context was created (or loaded) with. */
gs_status gs_get_config(const struct gs_ctx* ctx, gs_config* out);
const char* gs_last_error(const struct gs_ctx* ctx);

/* Per-stage link model. lat_ns is S x S (sender stage row), bw arrays have S
 * entries in bit/s; stage_of_peer has `peers` entries or is NULL (= u % S,
 * topogen.py:121-122). */
gs_status gs_set_links(struct gs_ctx* ctx, uint32_t stages, const uint64_t* lat_ns,
                       const uint64_t* bw_up_bps, const uint64_t* bw_down_bps,
                       const uint8_t* stage_of_peer);

/* Random ID dialing -> symmetric CSR peer graph, on the device
 * (replaces connect_gossipsub_peers, main.rs:303-389). */
gs_status gs_build_topology(struct gs_ctx* ctx);

/* Graph size after gs_build_topology. */
gs_status gs_graph_info(const struct gs_ctx* ctx, uint32_t* peers, uint64_t* nnz,
                        uint32_t* max_degree);

/* Copy the CSR out: row_ptr[peers+1], col[nnz], flags[nnz] (bit0 = outbound,
 * bit1 = in mesh). Any pointer may be NULL. */
gs_status gs_get_csr(struct gs_ctx* ctx, uint64_t* row_ptr, uint32_t* col, uint8_t* flags);

/* Heartbeat GRAFT/PRUNE to a fixed point or max_heartbeats epochs
 * (libp2p-gossipsub heartbeat, configured at main.rs:228-236). With churn
 * there is no fixed point: exactly max_heartbeats epochs run, and gs_run then
 * advances the mesh to the epochs its schedule needs. */
gs_status gs_mesh_converge(struct gs_ctx* ctx, uint32_t max_heartbeats, uint32_t* out_epochs);

/* Mesh width of gs_get_mesh rows. */
#define GS_MESH_W 16u
/* Copy the mesh out: mesh[peers*GS_MESH_W] (ascending ids, UINT32_MAX padding),
 * count[peers]. Either pointer may be NULL. */
gs_status gs_get_mesh(struct gs_ctx* ctx, uint32_t* mesh, uint8_t* count);

/* Simulate n_msgs publishes (replaces publish_new_message + the receive /
 * forward / reassembly loop, main.rs:79-143,519-528). Results go to `sink`
 * (may be NULL: device-resident run, counters only). */
gs_status gs_run(struct gs_ctx* ctx, const gs_publish* sched, uint64_t n_msgs,
                 const gs_result_sink* sink);

gs_status gs_get_stats(const struct gs_ctx* ctx, gs_stats* out);
gs_status gs_reset_stats(struct gs_ctx* ctx);

/* 1: record HIP events around every relaxation launch and around gs_run. */
gs_status gs_set_timing(struct gs_ctx* ctx, uint32_t enable);

/* 1: account every send of gs_run per peer (the counters Shadow's tracker
 * keeps per host, summary_shadowlog.awk): flood-publish and forward sends of a
 * fragment, lazy gossip's IHAVE and IWANT RPCs and IWANT answers, each to the
 * sender's tx and — unless lost to churn (receiver offline or the message's
 * lifetime over at the arrival) — the receiver's rx columns, plus the ACKs the
 * receiver returns. Counted after each batch from the final keys (extra passes
 * over them), so it is off by default. Enabling zeroes the counters, as does
 * gs_reset_stats. */
gs_status gs_set_traffic(struct gs_ctx* ctx, uint32_t enable);
/* Copy the per-peer counters out: traffic[peers][GS_TRAFFIC_COLS]. */
gs_status gs_get_traffic(struct gs_ctx* ctx, uint64_t* traffic);

/* ---- peer-partitioned mode -------------------------
 * Context `part` of `parts` owns the keys of peers [part*N/parts,
 * (part+1)*N/parts); topology and mesh are built identically (replicated) in
 * every partition. One batch (<= cfg.batch messages of equal size) is driven
 * bucket by bucket by the caller, who performs the exchange:
 *   k = min over parts of gs_part_begin(...)
 *   while k != UINT64_MAX:
 *     gs_part_scan(ctx, k, recs, cap, &n, &m1)        -- own arrivals of k's bucket
 *     all-gather the n records of every part           -- RCCL / loop-back
 *     gs_part_relax(ctx, k, all_recs, n_all, &m2)      -- edges into own peers
 *     k = min over parts of min(m1, m2)
 *   gs_part_finish(ctx, sink)                         -- sink rows hold own peers
 * Record pointers are DEVICE pointers on the context's device; the records
 * passed to gs_part_relax must be complete when it is called (synchronise the
 * stream that gathered them). A scan whose records exceed `capacity` returns
 * GS_ERANGE with *out_n = the capacity needed and changes no state: call it
 * again with a larger buffer. IDONTWANT, churn and per-peer traffic are not
 * supported in this mode, lazy gossip only as the proven no-op
 * (GS_EUNSUPPORTED). Results are bit-identical to gs_run. */
typedef struct gs_part_record {
    uint64_t key;      /* packed first-arrival key (t_rel | hops | src)          */
    uint64_t start;    /* uplink start of its forward (FIFO fold by the owner)   */
    uint32_t peer;     /* global id of the forwarding peer                        */
    uint32_t slot;     /* message * FP + fragment within the batch               */
} gs_part_record;

gs_status gs_set_partition(struct gs_ctx* ctx, uint32_t parts, uint32_t part);
gs_status gs_part_begin(struct gs_ctx* ctx, const gs_publish* sched, uint64_t n_msgs,
                        uint64_t* out_min_key);
gs_status gs_part_scan(struct gs_ctx* ctx, uint64_t bucket_key, gs_part_record* dev_records,
                       uint64_t capacity, uint64_t* out_n, uint64_t* out_min_key);
gs_status gs_part_relax(struct gs_ctx* ctx, uint64_t bucket_key, const gs_part_record* dev_records,
                        uint64_t n, uint64_t* out_min_key);
/* sink arrays are [n_msgs][own peers] (message-major over this part's peers) */
gs_status gs_part_finish(struct gs_ctx* ctx, const gs_result_sink* sink);

/* ---- multi-GPU communicator and the library-driven partitioned run ---------
 * (SURVEY §8b gs_comm_init, §8e; the reference's process boundary is one swarm
 * task per process, rust-test-node/src/main.rs:466-477.) One rank per process
 * and GPU over RCCL (xGMI), or several parts in one process (loopback device
 * copies: tests, several parts on one GPU). */
typedef struct gs_comm gs_comm;
#define GS_COMM_ID_BYTES 128
typedef struct gs_comm_id { char internal[GS_COMM_ID_BYTES]; } gs_comm_id;
/* An RCCL unique id: rank 0 creates it and hands it to the other ranks out of
 * band (as ncclGetUniqueId). GS_EUNSUPPORTED when RCCL cannot be loaded. */
gs_status gs_comm_get_id(gs_comm_id* out);
/* This process's rank of an nranks-rank RCCL communicator on HIP device
 * `device` (collective: every rank calls it). */
gs_status gs_comm_init(uint32_t nranks, uint32_t rank, const gs_comm_id* id, int32_t device, gs_comm** out);
/* nparts parts driven by this process (one context each, any devices). */
gs_status gs_comm_init_local(uint32_t nparts, gs_comm** out);
/* ABI 10: a rank whose collectives are the caller's own transport (any
 * process launcher: torch.distributed gloo, MPI, sockets). The library stages
 * every collective of the partitioned protocols through host memory and calls
 *  - allgather(user, mine, n, out): every rank's n u64 words into
 *    out[rank * n + k] (the MIN / MAX all-reduces are reduced from it);
 *  - exchange(user, send, send_bytes, recv, recv_bytes): an all-to-all-v of
 *    host bytes — send[p] (send_bytes[p] bytes) to rank p, recv[p]
 *    (recv_bytes[p] bytes, sizes known to both ends) from rank p, for every
 *    p < nranks (the own entry is 0 bytes).
 * A callback returns 0 on success; anything else fails the call on this rank
 * (the others then fail in their next collective or in the transport).
 * Collective order and sizes are the RCCL backend's, so every rank of a run
 * makes the same calls in the same order. `device` is the rank's HIP device. */
typedef struct gs_comm_ops {
    void* user;
    int (*allgather)(void* user, const uint64_t* mine, uint64_t n, uint64_t* out);
    int (*exchange)(void* user, const void* const* send, const uint64_t* send_bytes, void* const* recv,
                    const uint64_t* recv_bytes);
} gs_comm_ops;
gs_status gs_comm_init_ops(uint32_t nranks, uint32_t rank, const gs_comm_ops* ops, int32_t device, gs_comm** out);
/* Transport check (ABI 10, host memory only, no device work): one allgather of
 * (rank, nranks) words and one exchange of position-hashed buffers of
 * 1 + 977 * (sender + 3 * receiver) bytes, each checked; GS_EDEVICE names the
 * first mismatch. For gs_comm_init_ops communicators (others: GS_OK). */
gs_status gs_comm_check(gs_comm* comm);
gs_status gs_comm_destroy(gs_comm* comm);
/* gs_run with the peers partitioned over the communicator's parts: ctxs are
 * this process's contexts (RCCL: nctx = 1, the rank's; local: nctx = nparts,
 * part i = ctxs[i]), all built with the same config, topology and mesh. The
 * library sets each context's partition, runs every batch on the list pass
 * over own rows (records exchanged between window passes: loop-back parts on
 * one device store each record straight into the parts owning a receiver and
 * combine the pass control on the device; ranks exchange every part's records,
 * or with GS_PART_ROUTE=1 only the routed ones) or the bucket
 * protocol (per bucket: own scan, records routed only to the parts owning a
 * target with grouped send/recv, relax into own peers, MIN all-reduce of the
 * next bucket key) and writes part i's peers to sinks[i] ([n_msgs][own peers];
 * sinks may be NULL). Batches the peer protocols cannot take — churn,
 * IDONTWANT, lazy gossip whose IWANTs can change the result — run
 * message-sharded over the replicated graph (part p simulates its share of
 * the batch's messages for all peers, one all-to-all hands every part its own
 * peers' rows; gs_stats.ms_batches counts them). Collective over the
 * communicator. Results are bit-identical to gs_run. GS_EUNSUPPORTED: per-peer
 * traffic (gs_set_traffic), and sink summaries of a message-sharded batch. */
gs_status gs_run_partitioned(struct gs_ctx* const* ctxs, uint32_t nctx, gs_comm* comm, const gs_publish* sched,
                             uint64_t n_msgs, const gs_result_sink* sinks);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIPSIM_H */
