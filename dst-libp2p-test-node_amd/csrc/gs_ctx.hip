// gs_ctx.hip — C-ABI entry points of libgossipsim (include/gossipsim.h):
// context lifecycle, argument validation, error capture. No exception crosses
// the ABI; every failure becomes a gs_status plus gs_last_error text.
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "gs_internal.h"

struct gs_ctx : gs::Ctx {};

namespace gs {

Ctx::~Ctx() {
  static const bool dbg = getenv("GS_DEBUG_DTOR") != nullptr;
  auto say = [&](const char* w) {
    if (dbg) fprintf(stderr, "[dtor] %s\n", w);
  };
  say("sync streams");
  for (hipStream_t st : {side, chain, chain_pipe, pass_ms, copy, stream})
    if (st) (void)hipStreamSynchronize(st);
  say("events");
  for (auto e : ev_pool) (void)hipEventDestroy(e);
  for (auto e : side_ev) (void)hipEventDestroy(e);
  for (auto e : blk_ev)
    if (e) (void)hipEventDestroy(e);
  say("side");
  if (side) (void)hipStreamDestroy(side);
  say("chain");
  if (chain) (void)hipStreamDestroy(chain);
  say("chain_pipe");
  if (chain_pipe) (void)hipStreamDestroy(chain_pipe);
  for (auto e : chain_ev)
    if (e) (void)hipEventDestroy(e);
  for (int k = 0; k < 2; k++) {
    if (lat_src[k]) (void)hipEventDestroy(lat_src[k]);
    if (lat_done[k]) (void)hipEventDestroy(lat_done[k]);
    if (h_lat[k]) (void)hipHostFree(h_lat[k]);
  }
  for (auto& v : cp_ev)
    for (auto e : v) (void)hipEventDestroy(e);
  say("pass_ms");
  if (pass_ms) (void)hipStreamDestroy(pass_ms);
  for (auto e : pass_ev)
    if (e) (void)hipEventDestroy(e);
  if (h_laterr) (void)hipHostFree(h_laterr);
  if (copy) (void)hipStreamDestroy(copy);
  if (part_xev) (void)hipEventDestroy(part_xev);
  if (part_pev) (void)hipEventDestroy(part_pev);
  if (h_pstat) (void)hipHostFree(h_pstat);
  if (h_pinned) (void)hipHostFree(h_pinned);
  if (h_block) (void)hipHostFree(h_block);
  if (h_slms) (void)hipHostFree(h_slms);
  say("stream");
  if (stream) (void)hipStreamDestroy(stream);
  say("done");
}

uint64_t read_counter(Ctx& c, uint32_t idx) {
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_counters.p + idx, 8, hipMemcpyDeviceToHost, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
  return c.h_pinned[0];
}

static void validate(const gs_config& c) {
  auto bad = [](const std::string& m) { throw Error(GS_EINVAL, m); };
  if (c.abi_version != GS_ABI_VERSION) bad("abi_version mismatch");
  if (c.peers < 2) bad("PEERS must be >= 2");
  if (c.peers >= (1u << STAGE_SHIFT)) throw Error(GS_EUNSUPPORTED, "PEERS must be < 2^24");
  if (c.connect_to >= c.peers)  // env.rs:73-75
    bad("Not enough peers to make target connections. Network size: " + std::to_string(c.peers));
  if (dials_per_peer(c.peers, c.connect_to, c.dial_extra) == 0)  // main.rs:381-382
    bad("Failed to connect any peers (CONNECTTO = 0)");
  if (dials_per_peer(c.peers, c.connect_to, c.dial_extra) > MAX_DIALS)
    throw Error(GS_EUNSUPPORTED, "more than 64 dials per peer");
  if (c.fragments < 1 || c.fragments > MAX_FRAGS) bad("FRAGMENTS must be in 1..16");
  if (c.muxer > GS_MUX_MPLEX) bad("Unknown muxer type");  // env.rs:69-71
  if (!(c.d_lo <= c.d && c.d <= c.d_hi)) bad("need D_lo <= D <= D_hi");
  if (c.d > 16 || c.d_hi >= MESH_W) throw Error(GS_EUNSUPPORTED, "need D <= 16 and D_hi < 16");
  if (c.d_out > c.d) bad("need D_out <= D");
  if (c.heartbeat_ns == 0) bad("heartbeat interval must be > 0");
  if (c.batch < 1 || c.batch > 65536) bad("batch must be in 1..65536");
  if (c.churn_ppm > 1000000) bad("churn_ppm must be <= 1000000");
  if (c.churn_ppm && (c.churn_down < 1 || c.churn_horizon < 1)) bad("churn needs churn_down >= 1 and churn_horizon >= 1");
  if (c.node > GS_NODE_NIM) bad("unknown node flavour (GS_NODE_RUST / _GO / _NIM)");
}

}  // namespace gs

using namespace gs;

#define GS_API_BEGIN(ctx) \
  if (!(ctx)) return GS_EINVAL; \
  try {
#define GS_API_END(ctx)                          \
  }                                              \
  catch (const Error& e) {                       \
    (ctx)->last_error = e.msg;                   \
    return e.code;                               \
  }                                              \
  catch (const std::exception& e) {              \
    (ctx)->last_error = e.what();                \
    return GS_ENOMEM;                            \
  }                                              \
  return GS_OK;

extern "C" gs_status gs_create(const gs_config* cfg, gs_ctx** out) {
  if (!cfg || !out) return GS_EINVAL;
  *out = nullptr;
  gs_ctx* c = nullptr;
  try {
    validate(*cfg);
    c = new gs_ctx();
    c->cfg = *cfg;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
      delete c;
      return GS_EDEVICE;
    }
    if (cfg->device < 0 || cfg->device >= ndev) {
      delete c;
      return GS_EDEVICE;
    }
    GS_HIP(hipSetDevice(cfg->device));
    GS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    GS_HIP(hipHostMalloc((void**)&c->h_pinned, H_PINNED_WORDS * 8, hipHostMallocDefault));
    c->d_counters.alloc(C_COUNT);
    c->d_ctrl.alloc(4);
    GS_HIP(hipMemsetAsync(c->d_counters.p, 0, C_COUNT * 8, c->stream));
    GS_HIP(hipStreamSynchronize(c->stream));
    c->k = dials_per_peer(cfg->peers, cfg->connect_to, cfg->dial_extra);
  } catch (const Error& e) {
    delete c;
    return e.code;
  } catch (...) {
    delete c;
    return GS_ENOMEM;
  }
  *out = c;
  return GS_OK;
}

extern "C" gs_status gs_destroy(gs_ctx* ctx) {
  if (!ctx) return GS_EINVAL;
  (void)hipSetDevice(ctx->cfg.device);
  delete ctx;
  return GS_OK;
}

extern "C" const char* gs_last_error(const gs_ctx* ctx) {
  return ctx ? ctx->last_error.c_str() : "null context";
}

extern "C" gs_status gs_set_links(gs_ctx* ctx, uint32_t S, const uint64_t* lat_ns,
                                  const uint64_t* bw_up, const uint64_t* bw_dn,
                                  const uint8_t* stage_of_peer) {
  GS_API_BEGIN(ctx)
  if (S == 0 || S > MAX_STAGES || !lat_ns || !bw_up || !bw_dn)
    ctx->fail(GS_EINVAL, "need 1..16 stages and non-null link tables");
  const uint32_t N = ctx->cfg.peers;
  for (uint32_t i = 0; i < S; i++)
    if (bw_up[i] == 0 || bw_dn[i] == 0) ctx->fail(GS_EINVAL, "bandwidth must be > 0");
  for (uint64_t i = 0; i < (uint64_t)S * S; i++)
    if (lat_ns[i] == 0 || lat_ns[i] >= (1ull << 32)) ctx->fail(GS_EINVAL, "latency must be in 1..2^32-1 ns");
  ctx->S = S;
  ctx->lat_ns.assign(lat_ns, lat_ns + (size_t)S * S);
  ctx->bw_up.assign(bw_up, bw_up + S);
  ctx->bw_dn.assign(bw_dn, bw_dn + S);
  ctx->stage_host.resize(N);
  ctx->stage_used.assign(S, 0);
  for (uint32_t u = 0; u < N; u++) {
    const uint8_t st = stage_of_peer ? stage_of_peer[u] : (uint8_t)(u % S);  // topogen.py:121-122
    if (st >= S) ctx->fail(GS_EINVAL, "stage_of_peer entry >= stages");
    ctx->stage_host[u] = st;
    ctx->stage_used[st] = 1;
  }
  GS_HIP(hipSetDevice(ctx->cfg.device));
  ctx->d_stage.alloc(N);
  GS_HIP(hipMemcpyAsync(ctx->d_stage.p, ctx->stage_host.data(), N, hipMemcpyHostToDevice, ctx->stream));
  GS_HIP(hipStreamSynchronize(ctx->stream));
  ctx->links_set = true;
  ctx->mesh_built = false;  // the mesh's GRAFT order and packed stages depend on the links
  ctx->cell_valid = false;  //  so do the churn pass's 64-wide rows (stage << 24 | peer)
  ctx->lat32_ok = false;
  GS_API_END(ctx)
}

extern "C" gs_status gs_build_topology(gs_ctx* ctx) {
  GS_API_BEGIN(ctx)
  GS_HIP(hipSetDevice(ctx->cfg.device));
  launch_topology(*ctx);
  if (ctx->max_degree > MAX_DEG) ctx->fail(GS_EUNSUPPORTED, "peer degree exceeds 256");
  ctx->topo_built = true;
  ctx->csrpos_valid = false;
  ctx->cell_valid = false;
  ctx->mesh_built = false;
  ctx->glp_prefer = false;
  GS_API_END(ctx)
}

extern "C" gs_status gs_graph_info(const gs_ctx* ctx, uint32_t* peers, uint64_t* nnz,
                                   uint32_t* max_degree) {
  if (!ctx) return GS_EINVAL;
  if (!ctx->topo_built) return GS_ESTATE;
  if (peers) *peers = ctx->cfg.peers;
  if (nnz) *nnz = ctx->nnz;
  if (max_degree) *max_degree = ctx->max_degree;
  return GS_OK;
}

extern "C" gs_status gs_get_csr(gs_ctx* ctx, uint64_t* row_ptr, uint32_t* col, uint8_t* flags) {
  GS_API_BEGIN(ctx)
  if (!ctx->topo_built) ctx->fail(GS_ESTATE, "gs_build_topology first");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  hipStream_t s = ctx->stream;
  if (row_ptr) GS_HIP(hipMemcpyAsync(row_ptr, ctx->d_row.p, ((size_t)ctx->cfg.peers + 1) * 8, hipMemcpyDeviceToHost, s));
  if (col && ctx->nnz) GS_HIP(hipMemcpyAsync(col, ctx->d_col.p, ctx->nnz * 4, hipMemcpyDeviceToHost, s));
  if (flags && ctx->nnz) GS_HIP(hipMemcpyAsync(flags, ctx->d_flags.p, ctx->nnz, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  GS_API_END(ctx)
}

extern "C" gs_status gs_mesh_converge(gs_ctx* ctx, uint32_t max_heartbeats, uint32_t* out_epochs) {
  GS_API_BEGIN(ctx)
  if (!ctx->topo_built) ctx->fail(GS_ESTATE, "gs_build_topology first");
  if (!ctx->links_set) ctx->fail(GS_ESTATE, "gs_set_links first");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  const uint32_t ep = run_mesh(*ctx, max_heartbeats);
  if (out_epochs) *out_epochs = ep;
  ctx->mesh_built = true;
  GS_API_END(ctx)
}

extern "C" gs_status gs_get_mesh(gs_ctx* ctx, uint32_t* mesh, uint8_t* count) {
  GS_API_BEGIN(ctx)
  if (!ctx->mesh_built) ctx->fail(GS_ESTATE, "gs_mesh_converge first");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  const size_t N = ctx->cfg.peers;
  if (mesh) {
    GS_HIP(hipMemcpyAsync(mesh, ctx->d_mesh.p, N * MESH_W * 4, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (count) GS_HIP(hipMemcpyAsync(count, ctx->d_mcnt.p, N, hipMemcpyDeviceToHost, ctx->stream));
  GS_HIP(hipStreamSynchronize(ctx->stream));
  if (mesh)
    for (size_t i = 0; i < N * MESH_W; i++)
      if (mesh[i] != EMPTY) mesh[i] &= (1u << STAGE_SHIFT) - 1;  // unpack the stage
  GS_API_END(ctx)
}

extern "C" gs_status gs_run(gs_ctx* ctx, const gs_publish* sched, uint64_t n_msgs,
                            const gs_result_sink* sink) {
  GS_API_BEGIN(ctx)
  if (!ctx->mesh_built) ctx->fail(GS_ESTATE, "gs_mesh_converge first");
  if (!sched && n_msgs) ctx->fail(GS_EINVAL, "null schedule");
  if (sink && sink->on_block && (sink->t_complete_ns || sink->hops))
    ctx->fail(GS_EINVAL, "gs_result_sink: with on_block, t_complete_ns and hops must be NULL (select outputs "
                         "with want, ABI 7)");
  if (sink && (sink->want & ~(uint32_t)(GS_WANT_T_COMPLETE | GS_WANT_HOPS | GS_WANT_LAT_MS)))
    ctx->fail(GS_EINVAL, "gs_result_sink.want: unknown bits");
  if (sink && (sink->on_lat != nullptr) != ((sink->want & GS_WANT_LAT_MS) != 0))
    ctx->fail(GS_EINVAL, "gs_result_sink: on_lat and GS_WANT_LAT_MS go together");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  if (n_msgs) run_messages(*ctx, sched, n_msgs, sink);
  GS_API_END(ctx)
}

extern "C" gs_status gs_get_stats(const gs_ctx* ctx, gs_stats* out) {
  if (!ctx || !out) return GS_EINVAL;
  *out = ctx->stats;
  return GS_OK;
}

extern "C" gs_status gs_get_config(const gs_ctx* ctx, gs_config* out) {
  if (!ctx || !out) return GS_EINVAL;
  *out = ctx->cfg;
  return GS_OK;
}

extern "C" gs_status gs_reset_stats(gs_ctx* ctx) {
  GS_API_BEGIN(ctx)
  GS_HIP(hipSetDevice(ctx->cfg.device));
  GS_HIP(hipMemsetAsync(ctx->d_counters.p, 0, C_COUNT * 8, ctx->stream));
  if (ctx->traffic)
    GS_HIP(hipMemsetAsync(ctx->d_traffic.p, 0, (size_t)ctx->cfg.peers * GS_TRAFFIC_COLS * 8, ctx->stream));
  GS_HIP(hipStreamSynchronize(ctx->stream));
  memset(&ctx->stats, 0, sizeof(ctx->stats));
  // (glp_prefer, the path choice learnt from a failed no-op proof, is no statistic: it
  // stays until the mesh changes or GLP_QUIET IWANT-free batches clear it)
  GS_API_END(ctx)
}

extern "C" gs_status gs_set_timing(gs_ctx* ctx, uint32_t enable) {
  if (!ctx) return GS_EINVAL;
  ctx->timing = enable != 0;
  return GS_OK;
}

extern "C" gs_status gs_set_traffic(gs_ctx* ctx, uint32_t enable) {
  GS_API_BEGIN(ctx)
  GS_HIP(hipSetDevice(ctx->cfg.device));
  ctx->traffic = enable != 0;
  if (ctx->traffic) {
    ctx->d_traffic.alloc((size_t)ctx->cfg.peers * GS_TRAFFIC_COLS);
    GS_HIP(hipMemsetAsync(ctx->d_traffic.p, 0, (size_t)ctx->cfg.peers * GS_TRAFFIC_COLS * 8, ctx->stream));
    GS_HIP(hipStreamSynchronize(ctx->stream));
  }
  GS_API_END(ctx)
}

extern "C" gs_status gs_get_traffic(gs_ctx* ctx, uint64_t* traffic) {
  GS_API_BEGIN(ctx)
  if (!traffic) ctx->fail(GS_EINVAL, "null traffic array");
  if (!ctx->traffic) ctx->fail(GS_ESTATE, "gs_set_traffic(ctx, 1) first");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  GS_HIP(hipMemcpyAsync(traffic, ctx->d_traffic.p, (size_t)ctx->cfg.peers * GS_TRAFFIC_COLS * 8,
                        hipMemcpyDeviceToHost, ctx->stream));
  GS_HIP(hipStreamSynchronize(ctx->stream));
  GS_API_END(ctx)
}

// ---- peer-partitioned mode (gs_part.h) ----
extern "C" gs_status gs_set_partition(gs_ctx* ctx, uint32_t parts, uint32_t part) {
  GS_API_BEGIN(ctx)
  part_set(*ctx, parts, part);
  GS_API_END(ctx)
}

extern "C" gs_status gs_part_begin(gs_ctx* ctx, const gs_publish* sched, uint64_t n_msgs,
                                   uint64_t* out_min_key) {
  GS_API_BEGIN(ctx)
  if (!ctx->mesh_built) ctx->fail(GS_ESTATE, "gs_mesh_converge first");
  if (!sched || !out_min_key) ctx->fail(GS_EINVAL, "null schedule or output");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  *out_min_key = part_begin(*ctx, sched, n_msgs);
  GS_API_END(ctx)
}

extern "C" gs_status gs_part_scan(gs_ctx* ctx, uint64_t bucket_key, gs_part_record* dev_records,
                                  uint64_t capacity, uint64_t* out_n, uint64_t* out_min_key) {
  GS_API_BEGIN(ctx)
  if (!out_n || !out_min_key) ctx->fail(GS_EINVAL, "null output");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  if (!part_scan(*ctx, bucket_key, dev_records, capacity, out_n, out_min_key))
    ctx->fail(GS_ERANGE, "record buffer too small: need " + std::to_string(*out_n) + " records");
  GS_API_END(ctx)
}

extern "C" gs_status gs_part_relax(gs_ctx* ctx, uint64_t bucket_key, const gs_part_record* dev_records,
                                   uint64_t n, uint64_t* out_min_key) {
  GS_API_BEGIN(ctx)
  if (!out_min_key) ctx->fail(GS_EINVAL, "null output");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  *out_min_key = part_relax(*ctx, bucket_key, dev_records, n);
  GS_API_END(ctx)
}

extern "C" gs_status gs_part_finish(gs_ctx* ctx, const gs_result_sink* sink) {
  GS_API_BEGIN(ctx)
  GS_HIP(hipSetDevice(ctx->cfg.device));
  part_finish(*ctx, sink);
  GS_API_END(ctx)
}

// ---- checkpoint / resume (include/gossipsim.h gs_save_state) ----
// The file holds what a later gs_run reads: the configuration, the link
// tables, the CSR with its outbound / mesh flags, reverse entries and PRUNE
// back-offs, the mesh ELL, the churn mesh state's epoch, the counters (host and
// device) and the
// per-peer traffic. Every random draw is a pure function of (seed, purpose,
// ...), so there is no generator state to keep. Churn snapshots cached in the
// ring are not saved: a restored context recomputes any epoch at or before the
// saved state by a replay from epoch 0, which gives the same snapshots.
namespace {
const char kStateMagic[8] = {'G', 'S', 'I', 'M', 'S', 'T', '0', '1'};

struct StateFile {
  FILE* f = nullptr;
  ~StateFile() { if (f) fclose(f); }
};

void put(FILE* f, const void* p, size_t n) {
  if (n && fwrite(p, 1, n, f) != n) throw Error(GS_EINVAL, "cannot write the state file");
}
void get(FILE* f, void* p, size_t n) {
  if (n && fread(p, 1, n, f) != n) throw Error(GS_EINVAL, "truncated state file");
}
template <class T>
void put_dev(Ctx& c, FILE* f, const DevBuf<T>& b, size_t n) {
  std::vector<T> h(n);
  if (n) {
    if (!b.p || b.n < n) throw Error(GS_ESTATE, "internal: state buffer missing");
    GS_HIP(hipMemcpyAsync(h.data(), b.p, n * sizeof(T), hipMemcpyDeviceToHost, c.stream));
    GS_HIP(hipStreamSynchronize(c.stream));
  }
  put(f, h.data(), n * sizeof(T));
}
template <class T>
void get_dev(Ctx& c, FILE* f, DevBuf<T>& b, size_t n) {
  std::vector<T> h(n);
  get(f, h.data(), n * sizeof(T));
  b.alloc(n ? n : 1);
  if (n) GS_HIP(hipMemcpyAsync(b.p, h.data(), n * sizeof(T), hipMemcpyHostToDevice, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
}
}  // namespace

extern "C" gs_status gs_save_state(gs_ctx* ctx, const char* path) {
  GS_API_BEGIN(ctx)
  if (!path) ctx->fail(GS_EINVAL, "null path");
  if (!ctx->links_set || !ctx->topo_built) ctx->fail(GS_ESTATE, "gs_set_links and gs_build_topology first");
  if (ctx->part_open) ctx->fail(GS_ESTATE, "a partitioned batch is in flight");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  StateFile sf;
  if (!(sf.f = fopen(path, "wb"))) ctx->fail(GS_EINVAL, std::string("cannot open ") + path);
  FILE* f = sf.f;
  const uint32_t abi = GS_ABI_VERSION, N = ctx->cfg.peers;
  put(f, kStateMagic, 8);
  put(f, &abi, 4);
  put(f, &ctx->cfg, sizeof(gs_config));
  const uint32_t fl[4] = {ctx->links_set, ctx->topo_built, ctx->mesh_built, ctx->traffic};
  put(f, fl, sizeof fl);
  put(f, &ctx->S, 4);
  put(f, ctx->lat_ns.data(), ctx->lat_ns.size() * 8);
  put(f, ctx->bw_up.data(), ctx->S * 8);
  put(f, ctx->bw_dn.data(), ctx->S * 8);
  put(f, ctx->stage_host.data(), N);
  const uint64_t topo[3] = {ctx->k, ctx->max_degree, ctx->nnz};
  put(f, topo, sizeof topo);
  put_dev(*ctx, f, ctx->d_row, (size_t)N + 1);
  put_dev(*ctx, f, ctx->d_col, ctx->nnz);
  put_dev(*ctx, f, ctx->d_flags, ctx->nnz);
  put_dev(*ctx, f, ctx->d_rev, ctx->nnz);
  const uint32_t has_until = ctx->d_until.p ? 1u : 0u;
  put(f, &has_until, 4);
  if (has_until) put_dev(*ctx, f, ctx->d_until, ctx->nnz);
  if (ctx->mesh_built) {
    put_dev(*ctx, f, ctx->d_mesh, (size_t)N * MESH_W);
    put_dev(*ctx, f, ctx->d_mcnt, N);
  }
  put(f, &ctx->churn_state, 8);
  put(f, &ctx->stats, sizeof(gs_stats));
  put_dev(*ctx, f, ctx->d_counters, C_COUNT);  // the device counters gs_stats is read from
  if (ctx->traffic) put_dev(*ctx, f, ctx->d_traffic, (size_t)N * GS_TRAFFIC_COLS);
  put(f, kStateMagic, 8);  // end marker
  if (fflush(f) != 0) ctx->fail(GS_EINVAL, "cannot write the state file");
  GS_API_END(ctx)
}

extern "C" gs_status gs_load_state(const char* path, int32_t device, gs_ctx** out) {
  if (!path || !out) return GS_EINVAL;
  *out = nullptr;
  StateFile sf;
  gs_config cfg{};
  char magic[8];
  uint32_t abi = 0;
  if (!(sf.f = fopen(path, "rb"))) return GS_EINVAL;
  if (fread(magic, 1, 8, sf.f) != 8 || memcmp(magic, kStateMagic, 8) || fread(&abi, 4, 1, sf.f) != 1 ||
      abi != GS_ABI_VERSION || fread(&cfg, sizeof cfg, 1, sf.f) != 1)
    return GS_EINVAL;  // not a state file of this ABI (no context to hold the message)
  cfg.device = device;
  gs_ctx* c = nullptr;
  gs_status st = gs_create(&cfg, &c);
  if (st != GS_OK) return st;
  try {
    FILE* f = sf.f;
    const uint32_t N = cfg.peers;
    uint32_t fl[4], S = 0;
    get(f, fl, sizeof fl);
    get(f, &S, 4);
    if (S == 0 || S > MAX_STAGES) c->fail(GS_EINVAL, "corrupt state file (stages)");
    std::vector<uint64_t> lat((size_t)S * S), up(S), dn(S);
    std::vector<uint8_t> stage(N);
    get(f, lat.data(), lat.size() * 8);
    get(f, up.data(), S * 8);
    get(f, dn.data(), S * 8);
    get(f, stage.data(), N);
    if ((st = gs_set_links(c, S, lat.data(), up.data(), dn.data(), stage.data())) != GS_OK) throw Error(st, c->last_error);
    uint64_t topo[3];
    get(f, topo, sizeof topo);
    c->k = (uint32_t)topo[0];
    c->max_degree = (uint32_t)topo[1];
    c->nnz = topo[2];
    get_dev(*c, f, c->d_row, (size_t)N + 1);
    get_dev(*c, f, c->d_col, c->nnz);
    get_dev(*c, f, c->d_flags, c->nnz);
    get_dev(*c, f, c->d_rev, c->nnz);
    uint32_t has_until = 0;
    get(f, &has_until, 4);
    if (has_until) get_dev(*c, f, c->d_until, c->nnz);
    c->topo_built = fl[1] != 0;
    c->csrpos_valid = false;
    c->cell_valid = false;
    if (fl[2]) {
      get_dev(*c, f, c->d_mesh, (size_t)N * MESH_W);
      get_dev(*c, f, c->d_mcnt, N);
      c->mesh_built = true;
    }
    get(f, &c->churn_state, 8);
    c->ring_lo = c->churn_state + 1;  // nothing cached: earlier epochs replay from epoch 0
    c->ring_hi = c->churn_state;
    get(f, &c->stats, sizeof(gs_stats));
    get_dev(*c, f, c->d_counters, C_COUNT);
    if (fl[3]) {
      c->traffic = true;
      get_dev(*c, f, c->d_traffic, (size_t)N * GS_TRAFFIC_COLS);
    }
    get(f, magic, 8);
    if (memcmp(magic, kStateMagic, 8)) c->fail(GS_EINVAL, "corrupt state file (end marker)");
  } catch (const Error& e) {
    gs_destroy(c);
    return e.code;
  } catch (...) {
    gs_destroy(c);
    return GS_ENOMEM;
  }
  *out = c;
  return GS_OK;
}
