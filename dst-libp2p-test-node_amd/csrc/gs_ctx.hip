// gs_ctx.hip — C-ABI entry points of libgossipsim (include/gossipsim.h):
// context lifecycle, argument validation, error capture. No exception crosses
// the ABI; every failure becomes a gs_status plus gs_last_error text.
#include <string.h>

#include <algorithm>

#include "gs_internal.h"

struct gs_ctx : gs::Ctx {};

namespace gs {

Ctx::~Ctx() {
  for (auto e : ev_pool) (void)hipEventDestroy(e);
  if (h_pinned) (void)hipHostFree(h_pinned);
  if (h_block) (void)hipHostFree(h_block);
  if (stream) (void)hipStreamDestroy(stream);
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
  GS_API_END(ctx)
}

extern "C" gs_status gs_build_topology(gs_ctx* ctx) {
  GS_API_BEGIN(ctx)
  GS_HIP(hipSetDevice(ctx->cfg.device));
  launch_topology(*ctx);
  if (ctx->max_degree > MAX_DEG) ctx->fail(GS_EUNSUPPORTED, "peer degree exceeds 256");
  ctx->topo_built = true;
  ctx->mesh_built = false;
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
  if (sink && (sink->want & ~(uint32_t)(GS_WANT_T_COMPLETE | GS_WANT_HOPS)))
    ctx->fail(GS_EINVAL, "gs_result_sink.want: unknown bits");
  GS_HIP(hipSetDevice(ctx->cfg.device));
  if (n_msgs) run_messages(*ctx, sched, n_msgs, sink);
  GS_API_END(ctx)
}

extern "C" gs_status gs_get_stats(const gs_ctx* ctx, gs_stats* out) {
  if (!ctx || !out) return GS_EINVAL;
  *out = ctx->stats;
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
