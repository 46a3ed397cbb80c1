//! gossipsim-sys: raw FFI bindings to libgossipsim, the MI355X GossipSub
//! dissemination simulator (C ABI `include/gossipsim.h`, ABI 9).
//!
//! Declarations only, in the header's order and layout; tests/test_rust_binding.py
//! checks every `#[repr(C)]` struct's field order and widths and every extern
//! fn's name and arity against the header. The calls the rust node would make
//! (rust-test-node/src/main.rs:123 publish, :223-241 ConfigBuilder, :526-528
//! the receive events) map to gs_config_* / gs_run / gs_result_sink
//!.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

pub type gs_status = i32;
pub const GS_OK: gs_status = 0;
pub const GS_UNDELIVERED: u64 = u64::MAX;
pub const GS_ABI_VERSION: u32 = 10;
pub const GS_NODE_RUST: u32 = 0;
pub const GS_TRAFFIC_COLS: usize = 12; // GS_TR_*: tx/rx bytes, packets, header bytes, received,
                                       // published, tx/rx ACK packets, tx/rx ACK header bytes
pub const GS_HIST_BINS: usize = 64;
pub const GS_CTRL_IHAVE: u32 = 0;
pub const GS_CTRL_IWANT: u32 = 1;
pub const GS_CTRL_ACK: u32 = 2;

#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_config {
    pub abi_version: u32, pub peers: u32, pub connect_to: u32, pub dial_extra: u32,
    pub max_connections: u32, pub fragments: u32, pub muxer: u32, pub signed_msgs: u32,
    pub d: u32, pub d_lo: u32, pub d_hi: u32, pub d_lazy: u32, pub d_out: u32,
    pub gossip_factor_milli: u32, pub heartbeat_ns: u64, pub backoff_ns: u64,
    pub flood_publish: u32, pub idontwant: u32, pub lazy_gossip: u32, pub self_log: u32,
    pub seed: u64, pub device: i32, pub batch: u32, pub history_gossip: u32, pub hb_phase_ns: u64,
    pub churn_ppm: u32, pub churn_down: u32, pub churn_horizon: u32, pub node: u32, pub sub_graft: u32,
    pub hs_rtts: u32,
}
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_publish { pub t_pub_ns: u64, pub publisher: u32, pub msg_size: u32, pub frags: u32, pub reserved: u32 }
#[repr(C)] #[derive(Clone, Copy)]
pub struct gs_msg_summary {
    pub delivered: u64, pub lat_sum_ms: u64, pub p50_ms: u32, pub p95_ms: u32, pub max_ms: u32,
    pub reserved: u32, pub hist: [u32; GS_HIST_BINS],
}
pub type gs_block_fn = Option<unsafe extern "C" fn(user: *mut c_void, first_msg: u64, n_msgs: u32, peers: u32,
                                                   t_complete_ns: *const u64, hops: *const u8)>;
pub type gs_lat_fn = Option<unsafe extern "C" fn(user: *mut c_void, first_msg: u64, n_msgs: u32, peers: u32,
                                                 lat_ms: *const u16)>;
#[repr(C)]
pub struct gs_result_sink {
    pub t_complete_ns: *mut u64, pub hops: *mut u8, pub on_block: gs_block_fn, pub user: *mut c_void,
    pub block_msgs: u32, pub want: u32, pub summary: *mut gs_msg_summary, pub on_lat: gs_lat_fn,
}
pub const GS_WANT_T_COMPLETE: u32 = 1;
pub const GS_WANT_HOPS: u32 = 2;
pub const GS_WANT_LAT_MS: u32 = 4;
pub const GS_LAT_NONE: u16 = 0xFFFF;
#[repr(C)] #[derive(Default)]
pub struct gs_stats {
    pub messages: u64, pub deliveries: u64, pub frag_deliveries: u64, pub relaxations: u64,
    pub bytes_alg: u64, pub latency_sum_ms: u64, pub latency_max_ms: u64,
    pub relax_launches: u64, pub buckets: u64, pub relax_ms: f64, pub run_ms: f64,
    pub relax_bytes_alg: u64, pub pushes: u64, pub scan_ms: f64, pub frontier_ms: f64, pub gossip_iwant: u64,
    pub gossip_noop_msgs: u64, pub gossip_fallback_batches: u64, pub batches: u64,
    pub list_pull_batches: u64, pub ms_batches: u64, pub gossip_list_batches: u64,
}
#[repr(C)] #[derive(Default)]
pub struct gs_injector { pub start_ns: u64, pub delay_ns: u64, pub msg_size: u32, pub messages: u32,
                         pub peers: u32, pub reserved: u32 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_part_record { pub key: u64, pub start: u64, pub peer: u32, pub slot: u32 }
#[repr(C)]
pub struct gs_comm_id { pub internal: [c_char; 128] }
pub enum gs_ctx {}
pub enum gs_log {}
pub enum gs_comm {}
/// ABI 10: the caller's transport for gs_comm_init_ops (host buffers; 0 = success).
#[repr(C)]
pub struct gs_comm_ops {
    pub user: *mut c_void,
    pub allgather: Option<unsafe extern "C" fn(user: *mut c_void, mine: *const u64, n: u64, out: *mut u64) -> c_int>,
    pub exchange: Option<unsafe extern "C" fn(user: *mut c_void, send: *const *const c_void, send_bytes: *const u64,
                                              recv: *const *mut c_void, recv_bytes: *const u64) -> c_int>,
}

#[link(name = "gossipsim")]
extern "C" {
    pub fn gs_config_default(cfg: *mut gs_config);
    pub fn gs_config_from_env(cfg: *mut gs_config, err: *mut c_char, err_len: usize) -> gs_status;
    pub fn gs_config_preset(cfg: *mut gs_config, node: u32) -> gs_status;
    pub fn gs_wire_bytes(payload: u64, muxer: u32, signed_msgs: u32) -> u64;
    pub fn gs_wire_packets(payload: u64, muxer: u32, signed_msgs: u32, packets: *mut u64, header_bytes: *mut u64);
    pub fn gs_control_packets(kind: u32, node: u32, muxer: u32, bytes: *mut u64, packets: *mut u64,
                              header_bytes: *mut u64);
    pub fn gs_topogen_links(stages: u32, bl: u32, bh: u32, ll: u32, lh: u32, mode: u32,
                            lat_ns: *mut u64, bw_bps: *mut u64) -> gs_status;
    pub fn gs_links_from_gml(path: *const c_char, mode: u32, max_nodes: u32, nodes: *mut u32,
                             lat_ns: *mut u64, bw_up: *mut u64, bw_down: *mut u64) -> gs_status;
    pub fn gs_shadow_hosts(path: *const c_char, peers: u32, stage_of_peer: *mut u8) -> gs_status;
    pub fn gs_shadow_injector(yaml_path: *const c_char, out: *mut gs_injector) -> gs_status;
    pub fn gs_read_schedule(path: *const c_char, out: *mut gs_publish, cap: u64, n: *mut u64) -> gs_status;
    pub fn gs_schedule_runsh(n: u32, peers: u32, publisher_id: u32, rotation: u32, t0_ns: u64,
                             delay_ns: u64, msg_size: u32, out: *mut gs_publish) -> gs_status;
    pub fn gs_write_latency_log(path: *const c_char, sched: *const gs_publish, n: u64, peers: u32,
                                t_complete_ns: *const u64, self_log: u32) -> gs_status;
    pub fn gs_write_node_log(cfg: *const gs_config, path: *const c_char, sched: *const gs_publish, n: u64,
                             t_complete_ns: *const u64) -> gs_status;
    pub fn gs_log_open(cfg: *const gs_config, path: *const c_char, out: *mut *mut gs_log) -> gs_status;
    pub fn gs_log_write(log: *mut gs_log, sched: *const gs_publish, n_msgs: u32, t_complete_ns: *const u64)
                        -> gs_status;
    pub fn gs_log_write_lat(log: *mut gs_log, sched: *const gs_publish, n_msgs: u32, lat_ms: *const u16)
                            -> gs_status;
    pub fn gs_log_close(log: *mut gs_log) -> gs_status;
    pub fn gs_write_shadow_heartbeat(path: *const c_char, peers: u32, traffic: *const u64, sim_seconds: u64)
                                     -> gs_status;
    pub fn gs_write_node_metrics(cfg: *const gs_config, path: *const c_char, row_ptr: *const u64,
                                 mesh_count: *const u8, traffic: *const u64) -> gs_status;
    pub fn gs_create(cfg: *const gs_config, out: *mut *mut gs_ctx) -> gs_status;
    pub fn gs_destroy(ctx: *mut gs_ctx) -> gs_status;
    pub fn gs_last_error(ctx: *const gs_ctx) -> *const c_char;
    pub fn gs_set_links(ctx: *mut gs_ctx, stages: u32, lat_ns: *const u64, bw_up: *const u64,
                        bw_down: *const u64, stage_of_peer: *const u8) -> gs_status;
    pub fn gs_build_topology(ctx: *mut gs_ctx) -> gs_status;
    pub fn gs_graph_info(ctx: *const gs_ctx, peers: *mut u32, nnz: *mut u64, max_deg: *mut u32) -> gs_status;
    pub fn gs_get_csr(ctx: *mut gs_ctx, row_ptr: *mut u64, col: *mut u32, flags: *mut u8) -> gs_status;
    pub fn gs_mesh_converge(ctx: *mut gs_ctx, max_heartbeats: u32, epochs: *mut u32) -> gs_status;
    pub fn gs_get_mesh(ctx: *mut gs_ctx, mesh: *mut u32, count: *mut u8) -> gs_status;
    pub fn gs_run(ctx: *mut gs_ctx, sched: *const gs_publish, n: u64, sink: *const gs_result_sink) -> gs_status;
    pub fn gs_get_stats(ctx: *const gs_ctx, out: *mut gs_stats) -> gs_status;
    pub fn gs_reset_stats(ctx: *mut gs_ctx) -> gs_status;
    pub fn gs_set_timing(ctx: *mut gs_ctx, enable: u32) -> gs_status;
    pub fn gs_set_traffic(ctx: *mut gs_ctx, enable: u32) -> gs_status;
    pub fn gs_get_traffic(ctx: *mut gs_ctx, traffic: *mut u64) -> gs_status;
    pub fn gs_get_config(ctx: *const gs_ctx, out: *mut gs_config) -> gs_status;
    pub fn gs_save_state(ctx: *mut gs_ctx, path: *const c_char) -> gs_status;
    pub fn gs_load_state(path: *const c_char, device: i32, out: *mut *mut gs_ctx) -> gs_status;
    pub fn gs_comm_get_id(out: *mut gs_comm_id) -> gs_status;
    pub fn gs_comm_init(nranks: u32, rank: u32, id: *const gs_comm_id, device: i32, out: *mut *mut gs_comm)
                        -> gs_status;
    pub fn gs_comm_init_local(nparts: u32, out: *mut *mut gs_comm) -> gs_status;
    pub fn gs_comm_init_ops(nranks: u32, rank: u32, ops: *const gs_comm_ops, device: i32, out: *mut *mut gs_comm)
        -> gs_status;
    pub fn gs_comm_check(comm: *mut gs_comm) -> gs_status;
    pub fn gs_comm_destroy(comm: *mut gs_comm) -> gs_status;
    pub fn gs_run_partitioned(ctxs: *const *mut gs_ctx, nctx: u32, comm: *mut gs_comm, sched: *const gs_publish,
                              n_msgs: u64, sinks: *const gs_result_sink) -> gs_status;
    pub fn gs_set_partition(ctx: *mut gs_ctx, parts: u32, part: u32) -> gs_status;
    pub fn gs_part_begin(ctx: *mut gs_ctx, sched: *const gs_publish, n_msgs: u64, out_min_key: *mut u64)
                         -> gs_status;
    pub fn gs_part_scan(ctx: *mut gs_ctx, bucket_key: u64, dev_records: *mut gs_part_record, capacity: u64,
                        out_n: *mut u64, out_min_key: *mut u64) -> gs_status;
    pub fn gs_part_relax(ctx: *mut gs_ctx, bucket_key: u64, dev_records: *const gs_part_record, n: u64,
                         out_min_key: *mut u64) -> gs_status;
    pub fn gs_part_finish(ctx: *mut gs_ctx, sink: *const gs_result_sink) -> gs_status;
}
