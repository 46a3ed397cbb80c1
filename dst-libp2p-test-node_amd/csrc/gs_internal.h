// gs_internal.h — context layout and kernel-launch entry points shared by the
// translation units of libgossipsim (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/gossipsim.h"
#include "gs_common.h"

#define GS_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) throw gs::Error(GS_EDEVICE, std::string(#call) + ": " +      \
                                                          hipGetErrorString(e_));      \
  } while (0)

namespace gs {

struct Error {
  gs_status code;
  std::string msg;
  Error(gs_status c, std::string m) : code(c), msg(std::move(m)) {}
};

// Device-side error word bits (set by kernels, checked by the host).
// ERR_LIST: a list pull candidate list overflowed; ERR_RING: a list pull candidate
// fell outside the K-window ring the host bound promised. Both re-run the batch on k_pull.
// ERR_LAT16: a logged latency of 65535 ms or more for the u16 stream (GS_WANT_LAT_MS).
enum : uint32_t { ERR_TIME = 1, ERR_HOPS = 2, ERR_MESH = 4, ERR_DEG = 8, ERR_LIST = 16, ERR_RING = 32, ERR_LAT16 = 64 };

// Device buffer owned by a context.
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    if (count <= n && p) return;
    release();
    if (count == 0) return;
    GS_HIP(hipMalloc((void**)&p, count * sizeof(T)));
    n = count;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DevBuf() { release(); }
};

// Counters written by kernels: index constants into Ctx::d_counters.
constexpr uint32_t H_PINNED_WORDS = 32;
constexpr uint32_t GLP_QUIET = 8;  // see run_messages run_glp

enum : uint32_t {
  C_FD = 0, C_R = 1, C_DELIV = 2, C_LAT_SUM = 3, C_LAT_MAX = 4, C_BUCKETS = 5,
  C_R_FWD = 6, C_MESH_CHANGES = 7, C_MESH_WAKE = 8, C_ERR = 9, C_PUSH = 10, C_GOSSIP = 11, C_PASSES = 12,
  C_GLISTED = 13, C_TSCANNED = 14, C_TSCANNED_G = 15,  // diagnostics (GS_DEBUG_COUNTS): gossip-listed
                                                       // lanes, tiles scanned, of them only for gossip
  C_COUNT = 16
};

// Per-batch geometry (gs_relax.hip setup_batch).
struct Batch {
  uint32_t B = 0, L = 0, F = 0, FP = 1, sb = 0, tshift = 0, Fe = 1;
  uint64_t lat_min = 0;  // smallest latency between used link classes (lazy-gossip no-op proof)
  uint64_t lat_max = 0;  // largest latency between used link classes (IHAVE travel bound)
  uint64_t ans_max = 0;  // largest IHAVE-arrival -> IWANT-answer-arrival time (lat + ser + lat + dn)
  uint64_t ser_max = 0;      // largest uplink serialisation of a used link class
  uint64_t lat_adj_max = 0;  // largest lat(x->y) + max(0, ser_dn(y) - ser_up(x)) over used classes
  bool collide = false;
  uint64_t payload = 0, tmax = 0, delta = 1;
  std::vector<uint64_t> tpub;
};

struct Ctx {
  gs_config cfg{};
  std::string last_error;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;           // second stream: churn IHAVE lists beside the epoch steps
  // churn: the epoch chain's own stream, restricted to GS_CHAIN_CUS compute units
  // (hipExtStreamCreateWithCUMask), and its join events
  hipStream_t chain = nullptr;
  hipEvent_t chain_ev[2] = {nullptr, nullptr};
  hipStream_t chain_pipe = nullptr;  // churn runs: the chain's stream on its own XCD (GS_CHAIN_XCDS, default 0)
  std::vector<hipEvent_t> side_ev;      // its chunk events
  bool timing = false;
  bool traffic = false;        // gs_set_traffic: per-peer send/receive counters
  DevBuf<uint64_t> d_traffic;  // [N][GS_TRAFFIC_COLS]

  // links
  uint32_t S = 0;
  std::vector<uint64_t> lat_ns, bw_up, bw_dn;
  std::vector<uint8_t> stage_host;
  std::vector<uint8_t> stage_used;  // [S] 1 if some peer sits on that link class
  bool links_set = false;

  // graph (device resident)
  bool topo_built = false, mesh_built = false;
  uint32_t k = 0;            // dials per peer
  uint64_t nnz = 0;
  uint32_t max_degree = 0;
  DevBuf<uint8_t> d_stage;
  DevBuf<uint32_t> d_dial;   // [N*k]
  DevBuf<uint8_t> d_acc;     // [N*k] dial accepted
  DevBuf<uint64_t> d_row;    // [N+1]
  DevBuf<uint32_t> d_col;    // [nnz]
  DevBuf<uint8_t> d_flags;   // [nnz] F_OUT | F_MESH
  DevBuf<uint32_t> d_rev;    // [nnz] index of the reverse entry
  DevBuf<uint32_t> d_until;  // [nnz] back-off: graft refused while epoch < until
  DevBuf<uint8_t> d_prop;    // [nnz] per-epoch GRAFT/PRUNE/ACCEPT bits
  DevBuf<uint8_t> d_iprop;   // [nnz] event-driven epochs: the GRAFT/PRUNE bits a neighbour proposed, at the receiver's entry
  DevBuf<uint32_t> d_mesh;   // [N*MESH_W] packed stage<<24|peer, EMPTY padded
  DevBuf<uint32_t> d_lat32;  // [S*S] u32 latency for the mesh kernels
  bool lat32_ok = false;     // d_lat32 holds the current links
  // churn: ring of per-epoch snapshots, slot = epoch % ring_R
  DevBuf<uint32_t> d_ring_mesh; // [R][N][MESH_W]
  DevBuf<uint64_t> d_ring_off;  // [R][(N+63)/64]
  DevBuf<uint32_t> d_ring_in;     // lazy gossip: [R][N][GT_IN] senders of the IHAVEs reaching a peer per epoch
  DevBuf<uint64_t> d_gout;        // scratch of ring_in_lists: IHAVE target masks over CSR rows, per (epoch, sender)
  DevBuf<uint8_t> d_csrpos;       // [nnz] position of the row's peer in its neighbour's row (ring_in_lists, GOS)
  bool csrpos_valid = false;      // d_csrpos is of the current CSR
  DevBuf<uint64_t> d_ring_mm;     // [R][N] mesh of each epoch as a mask over the CSR row (max_degree <= 64)
  std::vector<uint64_t> ring_in_tag;  // [R] epoch whose inverse IHAVE lists a slot holds (~0: none)
  bool ring_in_defer = false;         // the churn list pass takes the batch: no inverse lists beside the epochs
  // the ELL snapshots too: a churn list-pass batch reads only the mask ring, so the
  // epochs skip the ELL copy and ensure_ring_ell rebuilds a slot from its mask when
  // another reader needs it (push-path fallback, non-flood seeds, traffic)
  std::vector<uint64_t> ring_ell_tag;  // [R] epoch whose ELL snapshot a slot holds (~0: none)
  bool ring_ell_defer = false;
  // called by the epoch chain after it enqueued epoch h on the context's stream (and once with
  // h0 - 1 when the run's offline bits are written): the churn list pass's tables of the epochs
  // done so far go to the side stream (gs_relax.hip chn_chunks)
  std::function<void(uint64_t)> epoch_hook;
  std::vector<hipEvent_t> cp_ev[2];   // their events, per table set
  DevBuf<uint64_t> d_q0, d_r0;  // [B] epoch of t_pub, t_pub - start of that epoch
  uint32_t ring_R = 0;
  uint64_t churn_state = 0, ring_lo = 1, ring_hi = 0;  // mesh state epoch; valid ring epochs
  DevBuf<uint8_t> d_mcnt;    // [N]
  DevBuf<uint8_t> d_pst;     // event-driven churn epochs: [PS_PLANES][N] per-peer flags and counts
  DevBuf<uint64_t> d_offlin; // offline bitsets of a run of churn epochs, [epochs + 1][(N+63)/64]

  // dissemination (per batch)
  DevBuf<uint64_t> d_keys;   // [N * B * FP] peer-major (u, m, f)
  DevBuf<uint64_t> d_busy;   // [N * B] uplink FIFO end per (u, m) (F > 1)
  DevBuf<uint64_t> d_meta;   // per-64-lane tile metadata (TileMeta, 16 B)
  DevBuf<uint64_t> d_fbits;  // final bitset, one u64 per 64-lane tile
  DevBuf<uint32_t> d_fr_idx; // bucket frontier (per-scan-wave segments)
  DevBuf<uint64_t> d_fr_key;
  DevBuf<uint32_t> d_fr_cnt;
  DevBuf<uint64_t> d_tmin;   // split tile skip: min pending key per tile
  DevBuf<uint8_t> d_touched; // split tile skip: pushed since last scan
  DevBuf<uint64_t> d_tgmin;  // split tile skip + gossip: next IHAVE arrival per tile
  DevBuf<uint32_t> d_tnf;    // split tile skip + gossip: non-final lanes per tile
  DevBuf<uint32_t> d_tstamp; // split tile skip + gossip: launch + 1 of the last scan
  DevBuf<uint32_t> d_gl_idx; // lazy gossip: lanes with an IHAVE arrival in the bucket
  DevBuf<uint32_t> d_gl_cnt;
  DevBuf<uint64_t> d_gl_key; // receiver-centric gossip: the listed lane's key (saves its re-read)
  DevBuf<uint32_t> d_hl_idx;  // churn + gossip: holder list (RelaxArgs::hl_*): lane, key, count, launch marks
  DevBuf<uint64_t> d_hl_key;
  DevBuf<uint64_t> d_hl_cnt;
  DevBuf<uint64_t> d_hl_mark;
  DevBuf<uint32_t> d_hs_idx;  // per scan wave scratch of the holders found (copied to the list)
  DevBuf<uint64_t> d_hs_key;
  DevBuf<uint64_t> d_hl_min;
  DevBuf<uint8_t> d_hwin;     // [N][L] first gossip heartbeat of each final lane (RelaxArgs::hwin)
  DevBuf<uint64_t> d_nonfinal;  // [3]
  DevBuf<uint64_t> d_rel0;   // [B] first heartbeat >= t_pub (relative ns)
  DevBuf<uint64_t> d_habs0;  // [B] its absolute heartbeat index
  DevBuf<uint8_t> d_malive;  // [B] churn + gossip: the message can spread (publisher online at t_pub)
  DevBuf<uint32_t> d_pub;    // [B]
  DevBuf<uint64_t> d_tpub;   // [B]
  DevBuf<uint64_t> d_tc;     // [N * B] peer-major completion times (device result)
  DevBuf<uint8_t> d_hops;    // [N * B]
  DevBuf<uint64_t> d_tc_t;   // [B * N] message-major staging for the caller's sink
  DevBuf<uint8_t> d_hops_t;
  DevBuf<uint16_t> d_lat;    // [N * B] peer-major logged latency in ms (GS_WANT_LAT_MS)
  DevBuf<uint16_t> d_lat_t;  // [B * N] message-major staging of it
  hipEvent_t blk_ev[2] = {nullptr, nullptr};  // double-buffered streaming: D2H of block k done
  // latency-only sinks inside gs_run (gs_relax.hip deliver_lat_async): a finished
  // batch's u16 latencies leave on the copy stream into a whole-batch pinned
  // buffer while the next batch's passes run; its callbacks run at the next
  // batch's delivery or at the end of the run (message order kept)
  bool lat_async = false;
  hipStream_t copy = nullptr;
  DevBuf<uint16_t> d_lat_t2;                  // the other parity's message-major staging
  uint16_t* h_lat[2] = {nullptr, nullptr};    // pinned [B][un] per parity
  size_t h_lat_bytes[2] = {0, 0};
  uint64_t* h_laterr = nullptr;               // pinned: the error word after each parity's batch
  hipEvent_t lat_src[2] = {nullptr, nullptr}, lat_done[2] = {nullptr, nullptr};
  struct LatPending {
    bool on = false;
    uint32_t par = 0, B = 0, un = 0, bm = 64;
    uint64_t row0 = 0;
    const gs_result_sink* sink = nullptr;
  } lat_pend;
  uint32_t lat_par = 0;
  DevBuf<uint32_t> d_tables; // lat[S*S] | ser_up[S] | ser_dn[S] (u32 ns)
  DevBuf<uint64_t> d_ctrl;   // [4] triple-buffered next-min keys + spare
  // owner-computes pull path (gs_pull_kernel.h)
  DevBuf<uint32_t> d_chunkmin; // [N][16] per 64-lane chunk: hi word of the min key beyond the last emitted window
  DevBuf<uint64_t> d_lrec;   // [2][N][L] per-row arrival records (gs_pull_kernel.h)
  DevBuf<uint32_t> d_lcnt;   // [2][N]
  DevBuf<uint8_t> d_rpos;    // [N][MESH_W] index of w in mesh(mesh[w][j])
  // batch slices (gs_relax.hip run_slices): S copies of the graph's mesh rows, reverse
  // positions and stages; the slices' publishers as slice rows and as peers
  DevBuf<uint32_t> d_smesh;  // [S * N][MESH_W]
  DevBuf<uint8_t> d_srpos;
  DevBuf<uint8_t> d_sstage;  // [S * N]
  DevBuf<uint32_t> d_spub;   // [S][B]
  DevBuf<uint32_t> d_lpub;
  DevBuf<uint64_t> d_cnt_save2;  // [C_COUNT] counters around a slice group's repeated completions
  DevBuf<uint64_t> d_stpub;  // [S][B] the slices' publish times
  uint64_t* h_slms = nullptr;  // pinned [S][B][MS_COLS]: every slice's reductions for the gossip no-op proof
  size_t h_slms_bytes = 0;
  bool rpos_valid = false;
  bool keys_log = false;       // keys hold the list pull path's final logs (not dense rows): k_lcomplete
  uint32_t mesh_dmax = 0;      // widest frozen-mesh row (list pull ring bound); 0 = not known
  DevBuf<uint64_t> d_pctrl;  // [3][4] pass control slots
  // list pull path (gs_lpull_kernel.h)
  DevBuf<uint64_t> d_lblk;   // [K][N][L] candidate lists per destination-window slot
  DevBuf<uint32_t> d_lst;    // [N][16] list lengths per destination window, final-log length
  DevBuf<uint64_t> d_skey;   // list pull path: the publishes' first sends (k_seed -> k_lseed)
  DevBuf<uint32_t> d_slane;  // (row << 11) | lane
  DevBuf<uint32_t> d_scnt;
  DevBuf<uint64_t> d_lp_save;  // [C_COUNT] counters before a list pull batch (overflow re-run)
  DevBuf<uint32_t> d_lfin;   // [N][32] final bits
  DevBuf<uint16_t> d_flane;  // [N][L] lanes of the final log
  DevBuf<uint64_t> d_counters;  // [C_COUNT]
  DevBuf<uint64_t> d_cnt_save;  // [C_COUNT] counters before a batch (gossip fallback restores them)
  uint64_t* h_pinned = nullptr; // pinned host mirror of ctrl + counters (H_PINNED_WORDS)
  // per-message reductions of k_complete / k_pct (gs_relax.hip)
  DevBuf<uint64_t> d_mstat;     // [B][MS_COLS]
  DevBuf<uint32_t> d_hist;      // [B][GS_HIST_BINS]
  DevBuf<uint32_t> d_pbin;      // [B][2]
  DevBuf<uint32_t> d_fine;      // [B][2][GS_HIST_MS]
  void* h_block = nullptr;      // pinned staging of streamed result blocks (gs_result_sink.on_block)
  bool sink_dev = false;        // the sink's arrays are device memory (message-sharded partitioned batches)
  DevBuf<uint64_t> d_ms_tc;     // message-sharded partitioned batch: this part's messages [mp][N] ...
  DevBuf<uint8_t> d_ms_hops;
  DevBuf<uint64_t> d_ms_send;   // ... packed per destination part (RCCL)
  DevBuf<uint8_t> d_ms_sendh;
  size_t h_block_bytes = 0;

  // peer-partitioned mode (gs_part.h): this context holds keys of peers [u0, u0 + un)
  uint32_t part_parts = 1, part_idx = 0, part_u0 = 0, part_un = 0;
  bool part_open = false;       // between gs_part_begin and gs_part_finish
  Batch part_b;
  unsigned part_grid = 0;
  uint32_t part_seg_cap = 0;
  DevBuf<uint64_t> d_pcnt;      // [4] frontier groups, records, relax min key, spare
  DevBuf<uint64_t> d_dcnt, d_dpos;  // [64] records per destination part / their write cursors
  DevBuf<gs_part_record> d_pout, d_pin;  // gs_run_partitioned: records sent / received this bucket
  // gs_run_partitioned on the list pass (gs_part.h part_lp_*): this part's rows in the list
  // buffers above (local row indexing); every peer's records of the last pass, packed
  bool part_lp = false;
  uint32_t part_lpK = 0, part_lplb = 0, part_lppass = 0;
  unsigned part_lpgrid = 0;
  DevBuf<uint32_t> d_rcg;    // [N] records per peer (global ids)
  DevBuf<uint64_t> d_roffg;  // [N] their offsets in d_rpk
  DevBuf<uint64_t> d_rpk;    // every part's records of the last pass
  hipEvent_t part_xev = nullptr;  // loop-back routed stores of the last pass done (other parts wait on it)
  hipEvent_t part_pev = nullptr;  // loop-back: this part's pass done (part 0's combine waits on it)
  DevBuf<uint64_t> d_pstat;       // loop-back, part 0: every part's pass control (k_part_combine)
  uint64_t* h_pstat = nullptr;    // its pinned read-back (LP_PMAX x 4 words)
  DevBuf<uint64_t> d_pkcur;  // pack cursor (routed: one per destination part)
  // routed exchange (k_lpack_route): the records for each other part [P][cap] and
  // this part's per-peer offsets / counts for each destination [P][un]
  DevBuf<uint64_t> d_rsend;
  DevBuf<uint64_t> d_rroff;
  DevBuf<uint32_t> d_rrcg;
  // lazy gossip inside the list pass (gs_lpull_kernel.h, GOS batches)
  DevBuf<uint32_t> d_gpl;      // [N][32] sender planes of the built heartbeat
  DevBuf<uint64_t> d_gse;      // [N][L] their entries
  DevBuf<uint32_t> d_rowdone;  // [(N + 31) / 32]
  DevBuf<uint64_t> d_gctl;     // [GC_WORDS]
  bool glp_prefer = false;     // the last eager no-op proof failed: run gossip batches on the list pass first
  uint32_t glp_quiet = 0;      // list-pass gossip batches in a row without an IWANT (GLP_QUIET clears glp_prefer)
  // churn on the list pass (gs_cpull.h, k_lpull<.., CHN>): the CSR rows as 64-wide ELL rows (once
  // per topology), per batch the per-epoch mesh / IHAVE-eligible masks of every row over the
  // batch's epochs, each peer's offline epochs, and the offline lanes per relative epoch
  DevBuf<uint32_t> d_ccol;     // [N][64] stage << 24 | peer, ascending, EMPTY padded
  DevBuf<uint8_t> d_cpos;      // [N][64] position of the row's peer in that neighbour's row
  bool cell_valid = false;
  // the churn list pass's per-batch tables, two sets: the next batch's are built
  // (its epoch chain beside this batch's passes) while this batch's are read
  struct ChnTables {
    DevBuf<uint64_t> cmm, cgt;  // [N][cE] mesh / IHAVE targets of each epoch as masks over the CSR row
    DevBuf<uint64_t> offe;      // [N][cW] offline bit per epoch of the batch range
    DevBuf<uint32_t> coff;      // [H + 2][N][32] offline lanes per relative epoch (transposed like the final bits)
    DevBuf<uint32_t> cq;        // [B] epoch of t_pub - first epoch of the range
    DevBuf<uint8_t> pubok;      // [B] the publisher was online at t_pub
    DevBuf<uint32_t> calive;    // [32] published lanes in the final bits' transposed layout
  } ct[2];
  uint32_t ct_par = 0;          // the table set the next batch prepared in line uses
  std::function<void()> pass_poll;  // called by the list pass between groups of passes (the chain ahead)
  hipStream_t pass_ms = nullptr;    // churn runs: the passes' stream off the chain's XCDs (GS_PASS_XCDS)
  hipEvent_t pass_ev[2] = {nullptr, nullptr};
  DevBuf<uint8_t> d_gnz;       // [N] the row's IHAVE plane of the built heartbeat is not empty
  DevBuf<uint16_t> d_gtag;     // [N] the built heartbeat (GC_BK) whose IHAVEs the row takes by scanning planes
  DevBuf<uint32_t> d_gpc;      // [N] IHAVE entries pushed to the row per heartbeat (bk << 16 | count)
  DevBuf<uint64_t> d_luni;     // [2][N] per pass: OR of the receiver masks of a row's records

  // stats
  gs_stats stats{};
  std::vector<hipEvent_t> ev_pool;
  int num_cus = 0;
  uint32_t split_bpc = 0;  // blocks per CU of the split path's grid (split_blocks_per_cu)
  std::string gossip_why;  // the message that broke the last partitioned gossip no-op proof

  ~Ctx();
  void fail(gs_status c, const std::string& m) { throw Error(c, m); }
};

// ---- launchers (gs_topology.hip / gs_mesh.hip / gs_relax.hip) ----
void launch_topology(Ctx& c);
uint32_t run_mesh(Ctx& c, uint32_t max_heartbeats);
inline void ensure_cus(Ctx& c) {
  if (c.num_cus == 0) {
    hipDeviceProp_t prop;
    c.num_cus = hipGetDeviceProperties(&prop, c.cfg.device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
}
hipStream_t cu_stream(Ctx& c, uint32_t c0, uint32_t n);
hipStream_t cu_stream_except(Ctx& c, uint32_t c0, uint32_t stride);
hipStream_t xcd_stream(Ctx& c, uint32_t xcds);
uint32_t xcd_env(const char* name);
void churn_ring(Ctx& c, uint64_t h_lo, uint64_t h_hi);
// the epoch chain in slices (gs_mesh.hip): nullptr when [churn_state + 1, h1] is
// no plain continuation inside the ring (the caller runs churn_ring instead)
struct EvRun;
EvRun* chain_begin(Ctx& c, uint64_t h1, hipStream_t s, std::function<void(uint64_t)> hook);
bool chain_advance(Ctx& c, EvRun& r, uint64_t max_epochs);  // true once every epoch is enqueued
void chain_free(EvRun* r);
void ensure_csrpos(Ctx& c);
void ensure_in_lists(Ctx& c, uint64_t h0, uint64_t h1);
void ensure_ring_ell(Ctx& c, uint64_t h0, uint64_t h1);
hipStream_t side_stream(Ctx& c);
void run_messages(Ctx& c, const gs_publish* sched, uint64_t n_msgs, const gs_result_sink* sink);
void deliver_rows(Ctx& c, uint32_t B, uint32_t un, const gs_result_sink* sink, uint64_t sink_row0);
void part_set(Ctx& c, uint32_t parts, uint32_t part);
uint64_t part_begin(Ctx& c, const gs_publish* sched, uint64_t n_msgs);
bool part_scan(Ctx& c, uint64_t bucket_key, gs_part_record* rec, uint64_t cap, uint64_t* n, uint64_t* m1);
uint64_t part_relax(Ctx& c, uint64_t bucket_key, const gs_part_record* rec, uint64_t n);
void part_finish(Ctx& c, const gs_result_sink* sink);
// device-driven partitioned protocol (gs_comm.hip)
void part_dev_bucket(Ctx& c, uint32_t parts);
void part_dev_scan_count(Ctx& c, uint32_t parts);
void part_dev_export(Ctx& c, uint32_t parts, gs_part_record* out);
void part_dev_relax_next(Ctx& c, const gs_part_record* in, uint64_t n);
bool part_dev_complete(Ctx& c, bool hist, bool store = true);
void part_dev_finish(Ctx& c, const gs_result_sink* sink, uint64_t row0);
void part_abort(Ctx& c);
bool part_needs_ms(Ctx& c, const gs_publish* sched, uint64_t n_msgs);
// the list pass over partitioned rows (gs_part.h)
bool part_lp_begin(Ctx& c, const gs_publish* sched, uint64_t n_msgs);  // enqueued: then part_lp_seed_min
uint64_t part_lp_seed_min(Ctx& c);  // wait for the part's seeds: their min key
void part_lp_pass(Ctx& c);
void part_lp_read(Ctx& c, uint64_t out[4]);  // last pass: mode, records, min pending, error word
void part_lp_read_enqueue(Ctx& c);                   // part_lp_read in two steps
void part_lp_read_wait(Ctx& c, uint64_t out[4]);
void part_lp_combine(Ctx** cx, uint32_t P, uint64_t* st);  // loop-back on one device: read + set of all parts
void part_lp_set(Ctx& c, uint64_t records, uint64_t minp);  // the combined values into the last pass's slot
void part_lp_pack(Ctx& c, uint64_t base, uint64_t mine);
void part_lp_pack_route(Ctx& c, uint32_t P, uint32_t me, uint64_t mine);
void part_lp_pack_route_direct(Ctx** cx, uint32_t P, uint32_t me, uint64_t base);
void part_lp_route_read(Ctx& c, uint32_t P, uint64_t* counts);
void part_lp_route_fix(Ctx& c, uint32_t P, uint32_t me, const uint64_t* base);
void part_lp_end_enqueue(Ctx& c, const gs_result_sink* sink);  // completion (final logs or dense rows)
bool part_lp_end_check(Ctx& c);  // wait, then the gossip proof
void part_lp_abort(Ctx& c);

// small device helpers
void device_exclusive_scan(Ctx& c, const uint64_t* in, uint64_t* out, uint32_t n);
uint64_t read_counter(Ctx& c, uint32_t idx);

}  // namespace gs
