// gs_comm.hip — multi-GPU communicator and the library-driven peer-partitioned
// run (include/gossipsim.h gs_comm_*, gs_run_partitioned).
//
// The reference scales by running one process per peer (Shadow / K8s pods,
// rust-test-node/src/main.rs:466-477 drives one swarm task per process); here
// one process drives one GPU, and the only data that crosses GPUs is a
// bucket's arrival records. Per bucket, every part
//   1. scans its own keys and counts its records per destination part (a
//      record goes only to the parts owning one of its forward targets),
//   2. all-gathers the count vectors (RCCL) — the one host read per bucket,
//   3. exports its records grouped by destination and exchanges them with
//      grouped send/recv (all-to-all-v),
//   4. relaxes the received records into its own peers and MIN-all-reduces
//      the next bucket key on the device (ncclUint64 / ncclMin).
// Two backends: RCCL over xGMI (one rank per process and GPU), and an
// in-process loopback for several parts driven by one thread (device copies),
// which the tests use to run P parts on one GPU.
#include <dlfcn.h>
#include <string.h>
#include <rccl/rccl.h>  // types and enums only: the functions are resolved with dlsym

#include <algorithm>
#include <new>
#include <vector>

#include "gs_internal.h"
#include "gs_layout.h"

struct gs_ctx : gs::Ctx {};

namespace gs {
namespace {

// RCCL entry points, loaded on first use so that libgossipsim loads (and
// single-GPU runs work) where no RCCL is installed.
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*ErrorString)(ncclResult_t) = nullptr;
};

Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if ((r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (r.h) {
#define GS_SYM(f, name) r.f = (decltype(r.f))dlsym(r.h, name)
      GS_SYM(GetUniqueId, "ncclGetUniqueId");
      GS_SYM(CommInitRank, "ncclCommInitRank");
      GS_SYM(CommDestroy, "ncclCommDestroy");
      GS_SYM(AllReduce, "ncclAllReduce");
      GS_SYM(AllGather, "ncclAllGather");
      GS_SYM(Send, "ncclSend");
      GS_SYM(Recv, "ncclRecv");
      GS_SYM(GroupStart, "ncclGroupStart");
      GS_SYM(GroupEnd, "ncclGroupEnd");
      GS_SYM(ErrorString, "ncclGetErrorString");
#undef GS_SYM
      if (!r.GetUniqueId || !r.CommInitRank || !r.CommDestroy || !r.AllReduce || !r.AllGather || !r.Send ||
          !r.Recv || !r.GroupStart || !r.GroupEnd || !r.ErrorString) {
        dlclose(r.h);
        r.h = nullptr;
      }
    }
  }
  return r.h ? &r : nullptr;
}

#define GS_NCCL(call)                                                                               \
  do {                                                                                              \
    ncclResult_t r_ = (call);                                                                       \
    if (r_ != ncclSuccess) throw gs::Error(GS_EDEVICE, std::string(#call) + ": " + rccl()->ErrorString(r_)); \
  } while (0)

}  // namespace
}  // namespace gs

using namespace gs;

struct gs_comm {
  uint32_t local = 0;    // 1: in-process parts, 0: RCCL or the caller's transport (ops)
  uint32_t nranks = 1, rank = 0;
  int32_t device = 0;
  ncclComm_t nc = nullptr;
  bool has_ops = false;  // gs_comm_init_ops: collectives staged through host memory into ops
  gs_comm_ops ops{};
  uint64_t* d_scratch = nullptr;  // ranks: [parts * parts] count matrix + 1 flag word + [parts][4] pass control
  // ops backend: the send / recv calls of the open group, exchanged at its end
  struct Xfer {
    const void* src;
    void* dst;
    uint64_t bytes;
    int peer;
  };
  std::vector<Xfer> xs, xr;
  hipStream_t xstream = nullptr;
};

namespace gs {
namespace {

// The rank collectives of the partitioned protocols (RCCL's names and
// arguments, less the communicator): RCCL over xGMI, or through the caller's
// gs_comm_ops on host copies — a D2H copy, the callback, an H2D copy — in the
// same order and sizes on every rank.
size_t type_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;  // ncclUint64 (the only wide type used)
  }
}
void ops_fail(int rc, const char* what) {
  if (rc) throw Error(GS_EDEVICE, std::string("gs_comm_ops.") + what + " returned " + std::to_string(rc));
}
// every rank's n u64 words of the device buffer send -> recv[rank * n + k]
void coll_AllGather(gs_comm* cm, const void* send, void* recv, size_t n, ncclDataType_t t, hipStream_t s) {
  if (!cm->has_ops) {
    GS_NCCL(rccl()->AllGather(send, recv, n, t, cm->nc, s));
    return;
  }
  if (t != ncclUint64) throw Error(GS_EINVAL, "internal: ops all-gather of u64 words only");
  std::vector<uint64_t> mine(n), all((size_t)cm->nranks * n);
  GS_HIP(hipMemcpyAsync(mine.data(), send, n * 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  ops_fail(cm->ops.allgather(cm->ops.user, mine.data(), n, all.data()), "allgather");
  GS_HIP(hipMemcpyAsync(recv, all.data(), all.size() * 8, hipMemcpyHostToDevice, s));
  GS_HIP(hipStreamSynchronize(s));
}
// in-place MIN / MAX of n u64 words over the ranks (ops: reduced from an all-gather)
void coll_AllReduce(gs_comm* cm, const void* send, void* recv, size_t n, ncclDataType_t t, ncclRedOp_t op,
                    hipStream_t s) {
  if (!cm->has_ops) {
    GS_NCCL(rccl()->AllReduce(send, recv, n, t, op, cm->nc, s));
    return;
  }
  if (t != ncclUint64 || (op != ncclMin && op != ncclMax)) throw Error(GS_EINVAL, "internal: ops all-reduce");
  std::vector<uint64_t> mine(n), all((size_t)cm->nranks * n);
  GS_HIP(hipMemcpyAsync(mine.data(), send, n * 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  ops_fail(cm->ops.allgather(cm->ops.user, mine.data(), n, all.data()), "allgather");
  for (size_t k = 0; k < n; k++) {
    uint64_t v = all[k];
    for (uint32_t p = 1; p < cm->nranks; p++)
      v = op == ncclMin ? std::min(v, all[(size_t)p * n + k]) : std::max(v, all[(size_t)p * n + k]);
    mine[k] = v;
  }
  GS_HIP(hipMemcpyAsync(recv, mine.data(), n * 8, hipMemcpyHostToDevice, s));
  GS_HIP(hipStreamSynchronize(s));
}
void coll_group_start(gs_comm* cm) {
  if (!cm->has_ops) {
    GS_NCCL(rccl()->GroupStart());
    return;
  }
  cm->xs.clear();
  cm->xr.clear();
  cm->xstream = nullptr;
}
void coll_Send(gs_comm* cm, const void* buf, size_t count, ncclDataType_t t, int peer, hipStream_t s) {
  if (!cm->has_ops) {
    GS_NCCL(rccl()->Send(buf, count, t, peer, cm->nc, s));
    return;
  }
  cm->xs.push_back({buf, nullptr, (uint64_t)count * type_bytes(t), peer});
  cm->xstream = s;
}
void coll_Recv(gs_comm* cm, void* buf, size_t count, ncclDataType_t t, int peer, hipStream_t s) {
  if (!cm->has_ops) {
    GS_NCCL(rccl()->Recv(buf, count, t, peer, cm->nc, s));
    return;
  }
  cm->xr.push_back({nullptr, buf, (uint64_t)count * type_bytes(t), peer});
  cm->xstream = s;
}
// ops: the group's sends concatenated per peer in call order (the receiver's
// recvs from that peer split the bytes in its own call order, as RCCL matches
// a group's point-to-point calls per peer), one exchange, the recvs scattered
void coll_group_end(gs_comm* cm) {
  if (!cm->has_ops) {
    GS_NCCL(rccl()->GroupEnd());
    return;
  }
  const uint32_t P = cm->nranks;
  std::vector<std::vector<uint8_t>> sb(P), rb(P);
  std::vector<uint64_t> sn(P, 0), rn(P, 0);
  for (const auto& x : cm->xs) sn[x.peer] += x.bytes;
  for (const auto& x : cm->xr) rn[x.peer] += x.bytes;
  hipStream_t s = cm->xstream;
  for (uint32_t p = 0; p < P; p++) {
    sb[p].resize(sn[p]);
    rb[p].resize(rn[p]);
  }
  std::vector<uint64_t> at(P, 0);
  for (const auto& x : cm->xs) {
    if (x.bytes) GS_HIP(hipMemcpyAsync(sb[x.peer].data() + at[x.peer], x.src, x.bytes, hipMemcpyDeviceToHost, s));
    at[x.peer] += x.bytes;
  }
  if (s) GS_HIP(hipStreamSynchronize(s));
  // a rank's own transfers (the push protocol sends a part's records to itself)
  // stay here: the transport sees 0 bytes for the own entry
  const uint32_t me = cm->rank;
  if (sn[me] != rn[me]) throw Error(GS_EINVAL, "internal: own send and receive differ in the ops exchange");
  if (rn[me]) memcpy(rb[me].data(), sb[me].data(), rn[me]);
  std::vector<uint64_t> sx = sn, rx = rn;
  sx[me] = rx[me] = 0;
  std::vector<const void*> sp(P);
  std::vector<void*> rp(P);
  for (uint32_t p = 0; p < P; p++) {
    sp[p] = sb[p].data();
    rp[p] = rb[p].data();
  }
  ops_fail(cm->ops.exchange(cm->ops.user, sp.data(), sx.data(), rp.data(), rx.data()), "exchange");
  std::fill(at.begin(), at.end(), 0);
  for (const auto& x : cm->xr) {
    if (x.bytes) GS_HIP(hipMemcpyAsync(x.dst, rb[x.peer].data() + at[x.peer], x.bytes, hipMemcpyHostToDevice, s));
    at[x.peer] += x.bytes;
  }
  if (s) GS_HIP(hipStreamSynchronize(s));
  cm->xs.clear();
  cm->xr.clear();
}

}  // namespace
}  // namespace gs

extern "C" gs_status gs_comm_get_id(gs_comm_id* out) {
  static_assert(sizeof(gs_comm_id) == sizeof(ncclUniqueId), "gs_comm_id must hold an ncclUniqueId");
  if (!out) return GS_EINVAL;
  Rccl* r = rccl();
  if (!r) return GS_EUNSUPPORTED;
  ncclUniqueId id;
  if (r->GetUniqueId(&id) != ncclSuccess) return GS_EDEVICE;
  memcpy(out, &id, sizeof id);
  return GS_OK;
}

extern "C" gs_status gs_comm_init(uint32_t nranks, uint32_t rank, const gs_comm_id* id, int32_t device,
                                  gs_comm** out) {
  if (!out || !id || nranks < 1 || nranks > 64 || rank >= nranks) return GS_EINVAL;
  *out = nullptr;
  Rccl* r = rccl();
  if (!r) return GS_EUNSUPPORTED;
  if (hipSetDevice(device) != hipSuccess) return GS_EDEVICE;
  gs_comm* c = new (std::nothrow) gs_comm();
  if (!c) return GS_ENOMEM;
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclUniqueId nid;
  memcpy(&nid, id, sizeof nid);
  if (r->CommInitRank(&c->nc, (int)nranks, nid, (int)rank) != ncclSuccess ||
      hipMalloc((void**)&c->d_scratch, ((size_t)nranks * nranks + 1 + 4 * (size_t)nranks) * 8) != hipSuccess) {
    if (c->nc) r->CommDestroy(c->nc);
    delete c;
    return GS_EDEVICE;
  }
  *out = c;
  return GS_OK;
}

extern "C" gs_status gs_comm_init_local(uint32_t nparts, gs_comm** out) {
  if (!out || nparts < 1 || nparts > 64) return GS_EINVAL;
  gs_comm* c = new (std::nothrow) gs_comm();
  if (!c) return GS_ENOMEM;
  c->local = 1;
  c->nranks = nparts;
  *out = c;
  return GS_OK;
}

extern "C" gs_status gs_comm_init_ops(uint32_t nranks, uint32_t rank, const gs_comm_ops* ops, int32_t device,
                                      gs_comm** out) {
  if (!out || !ops || !ops->allgather || !ops->exchange || nranks < 1 || nranks > 64 || rank >= nranks)
    return GS_EINVAL;
  *out = nullptr;
  gs_comm* c = new (std::nothrow) gs_comm();
  if (!c) return GS_ENOMEM;
  c->has_ops = true;
  c->ops = *ops;
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && device >= 0 && device < ndev) {  // (gs_comm_check needs none)
    if (hipSetDevice(device) != hipSuccess ||
        hipMalloc((void**)&c->d_scratch, ((size_t)nranks * nranks + 1 + 4 * (size_t)nranks) * 8) != hipSuccess) {
      delete c;
      return GS_EDEVICE;
    }
  }
  *out = c;
  return GS_OK;
}

// Host-only check of the caller's transport: the words and bytes every rank
// must see, from a position hash (sender, receiver, byte index).
extern "C" gs_status gs_comm_check(gs_comm* c) {
  if (!c) return GS_EINVAL;
  if (!c->has_ops) return GS_OK;
  const uint32_t P = c->nranks, me = c->rank;
  const uint64_t mine[2] = {me, P};
  std::vector<uint64_t> all(2 * (size_t)P);
  if (c->ops.allgather(c->ops.user, mine, 2, all.data())) return GS_EDEVICE;
  for (uint32_t p = 0; p < P; p++)
    if (all[2 * p] != p || all[2 * p + 1] != P) return GS_EDEVICE;
  auto len = [](uint32_t s, uint32_t d) { return s == d ? 0ull : 1ull + 977ull * (s + 3ull * d); };
  auto byte = [](uint32_t s, uint32_t d, uint64_t i) {
    return (uint8_t)(((i + 1) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)s << 40) ^ ((uint64_t)d << 20)) >> 56);
  };
  std::vector<std::vector<uint8_t>> sb(P), rb(P);
  std::vector<uint64_t> sn(P), rn(P);
  std::vector<const void*> sp(P);
  std::vector<void*> rp(P);
  for (uint32_t p = 0; p < P; p++) {
    sn[p] = len(me, p);
    rn[p] = len(p, me);
    sb[p].resize(sn[p]);
    for (uint64_t i = 0; i < sn[p]; i++) sb[p][i] = byte(me, p, i);
    rb[p].assign(rn[p], 0);
    sp[p] = sb[p].data();
    rp[p] = rb[p].data();
  }
  if (c->ops.exchange(c->ops.user, sp.data(), sn.data(), rp.data(), rn.data())) return GS_EDEVICE;
  for (uint32_t p = 0; p < P; p++)
    for (uint64_t i = 0; i < rn[p]; i++)
      if (rb[p][i] != byte(p, me, i)) return GS_EDEVICE;
  return GS_OK;
}

extern "C" gs_status gs_comm_destroy(gs_comm* c) {
  if (!c) return GS_EINVAL;
  if (c->nc) {
    (void)hipSetDevice(c->device);
    rccl()->CommDestroy(c->nc);
  }
  if (c->d_scratch) (void)hipFree(c->d_scratch);
  delete c;
  return GS_OK;
}

namespace {

// Bytes per ncclSend / ncclRecv piece of the record exchange: 2^30 by default
// (DESIGN.md §5); GS_RCCL_PIECE_BYTES lowers it (tests force many pieces).
uint64_t rccl_piece_bytes() {  // read per bucket: tests change it between runs
  const char* e = getenv("GS_RCCL_PIECE_BYTES");
  const long long x = e && *e ? atoll(e) : 0;
  return x > 0 ? std::min<uint64_t>((uint64_t)x, 1ull << 30) : (1ull << 30);
}

// RCCL ranks agree on a status word (MAX): a rank that failed locally makes
// every rank fail the call instead of leaving the others waiting in a
// collective (the caller's error text names the failing rank's reason only
// on that rank).
void rank_status(gs_comm* cm, Ctx& c, uint64_t mine) {
  if (cm->local) return;
  uint64_t* w = cm->d_scratch + (size_t)cm->nranks * cm->nranks;
  c.h_pinned[0] = mine;
  GS_HIP(hipMemcpyAsync(w, c.h_pinned, 8, hipMemcpyHostToDevice, c.stream));
  coll_AllReduce(cm, w, w, 1, ncclUint64, ncclMax, c.stream);
  GS_HIP(hipMemcpyAsync(c.h_pinned, w, 8, hipMemcpyDeviceToHost, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
  if (c.h_pinned[0] && !mine) throw Error(GS_EINVAL, "another rank failed this partitioned call");
}

// Every RCCL rank must run the same protocol: the knobs that decide the
// batches and the collectives they enter are compared across ranks (MIN and
// MAX of each word agree) before the first batch.
void check_same_config(gs_comm* cm, Ctx& c, const gs_publish* sched, uint64_t n_msgs) {
  if (cm->local) return;
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the schedule
  for (uint64_t i = 0; i < n_msgs; i++) {
    const uint64_t v[4] = {sched[i].t_pub_ns, sched[i].publisher, sched[i].msg_size, sched[i].frags};
    for (uint64_t x : v) h = (h ^ x) * 1099511628211ull;
  }
  const uint64_t sig[8] = {c.cfg.peers, c.cfg.batch, c.cfg.lazy_gossip, c.cfg.idontwant,
                           c.cfg.churn_ppm, c.cfg.fragments, c.cfg.seed, h ^ n_msgs};
  DevBuf<uint64_t> d;
  d.alloc(16);
  memcpy(c.h_pinned, sig, sizeof sig);
  GS_HIP(hipMemcpyAsync(d.p, c.h_pinned, sizeof sig, hipMemcpyHostToDevice, c.stream));
  GS_HIP(hipMemcpyAsync(d.p + 8, c.h_pinned, sizeof sig, hipMemcpyHostToDevice, c.stream));
  coll_AllReduce(cm, d.p, d.p, 8, ncclUint64, ncclMin, c.stream);
  coll_AllReduce(cm, d.p + 8, d.p + 8, 8, ncclUint64, ncclMax, c.stream);
  GS_HIP(hipMemcpyAsync(c.h_pinned, d.p, 16 * 8, hipMemcpyDeviceToHost, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
  for (int k = 0; k < 8; k++)
    if (c.h_pinned[k] != c.h_pinned[8 + k])
      throw Error(GS_EINVAL, "RCCL ranks disagree on the partitioned run (peers, batch, lazy_gossip, idontwant, "
                             "churn, fragments, seed or schedule)");
}

// RCCL ranks: every rank's n words (n <= 4) -> out[rank * n + k] on the host.
void rank_gather(gs_comm* cm, Ctx& c, const uint64_t* mine, uint32_t n, uint64_t* out) {
  uint64_t* w = cm->d_scratch + (size_t)cm->nranks * cm->nranks + 1;
  memcpy(c.h_pinned + 16, mine, n * 8);
  GS_HIP(hipMemcpyAsync(w + (size_t)cm->rank * n, c.h_pinned + 16, n * 8, hipMemcpyHostToDevice, c.stream));
  coll_AllGather(cm, w + (size_t)cm->rank * n, w, n, ncclUint64, c.stream);
  std::vector<uint64_t> h((size_t)cm->nranks * n);
  GS_HIP(hipMemcpyAsync(h.data(), w, h.size() * 8, hipMemcpyDeviceToHost, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
  memcpy(out, h.data(), h.size() * 8);
}

// Message-sharded batch: the batches the peer protocols
// cannot take — churn (a mesh per heartbeat epoch), IDONTWANT, and lazy gossip
// that is not a no-op (receiver-centric IWANTs read other parts' keys) — run
// over the replicated graph instead. Part p simulates messages
// [B*p/P, B*(p+1)/P) of the batch over all N peers with gs_run's engine, then
// one all-to-all transposes the results: part r receives, from every part,
// the rows of its own peers, so each sink still gets [B][own peers]. The
// per-part memory is the same N*B/P lanes as the peer protocols'; the data
// crossing GPUs is the results (9 B per lane), once per batch.
void run_batch_ms(gs_comm* cm, Ctx** cx, uint32_t nctx, const gs_publish* sched, uint64_t i0, uint32_t B,
                  const gs_result_sink* sinks) {
  const uint32_t P = cm->nranks, N = cx[0]->cfg.peers;
  const PartLayout lay{P, N, B};
  const uint32_t mpmax = lay.mmax();
  // 1. every part: its share of the messages over all N peers (device-resident rows [mp][N])
  for (uint32_t i = 0; i < nctx; i++) {
    Ctx& c = *cx[i];
    const uint32_t me = cm->local ? i : cm->rank, m0 = lay.m0(me), mp = lay.mn(me);
    GS_HIP(hipSetDevice(c.cfg.device));
    std::string why;
    gs_status code = GS_OK;
    try {
      if (c.traffic) c.fail(GS_EUNSUPPORTED, "per-peer traffic is not supported in partitioned mode");
      if (sinks && sinks[i].summary)
        c.fail(GS_EUNSUPPORTED, "per-message summaries of a message-sharded partitioned batch (churn, IDONTWANT or "
                                "lazy gossip IWANTs): use gs_run");
      c.d_ms_tc.alloc(std::max<size_t>(1, (size_t)mp * N));
      c.d_ms_hops.alloc(std::max<size_t>(1, (size_t)mp * N));
      const uint64_t batches = c.stats.batches;
      if (mp) {
        gs_result_sink ds{};
        ds.t_complete_ns = c.d_ms_tc.p;
        ds.hops = c.d_ms_hops.p;
        const uint32_t batch = c.cfg.batch;
        c.cfg.batch = mpmax;  // buffers for this part's share, not the whole batch
        c.sink_dev = true;
        try {
          run_messages(c, sched + i0 + m0, mp, &ds);
        } catch (...) {
          c.cfg.batch = batch;
          c.sink_dev = false;
          throw;
        }
        c.cfg.batch = batch;
        c.sink_dev = false;
      }
      c.stats.messages += B - mp;  // every part counts the batch, as in the peer protocols
      c.stats.batches = batches + 1;
      c.stats.ms_batches++;
    } catch (const Error& e) {
      code = e.code;
      why = e.msg;
    }
    rank_status(cm, c, code != GS_OK);
    if (code != GS_OK) throw Error(code, why);
  }
  // 2. the transposition: part r's peers of every part's messages into r's d_tc_t / d_hops_t [B][un_r]
  if (cm->local) {
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      GS_HIP(hipStreamSynchronize(cx[i]->stream));
    }
    for (uint32_t r = 0; r < nctx; r++) {
      Ctx& d = *cx[r];
      const uint32_t u0 = lay.u0(r), un = lay.un(r);
      GS_HIP(hipSetDevice(d.cfg.device));
      d.d_tc_t.alloc((size_t)un * B);
      d.d_hops_t.alloc((size_t)un * B);
      for (uint32_t p = 0; p < nctx; p++) {  // part p's block of r's peers, straight from p's rows
        const uint32_t mp = lay.mn(p);
        if (!mp) continue;
        GS_HIP(hipMemcpy2DAsync(d.d_tc_t.p + lay.ms_recv_off(p, r), (size_t)un * 8, cx[p]->d_ms_tc.p + u0,
                                (size_t)N * 8, (size_t)un * 8, mp, hipMemcpyDeviceToDevice, d.stream));
        GS_HIP(hipMemcpy2DAsync(d.d_hops_t.p + lay.ms_recv_off(p, r), un, cx[p]->d_ms_hops.p + u0, N, un, mp,
                                hipMemcpyDeviceToDevice, d.stream));
      }
    }
    for (uint32_t r = 0; r < nctx; r++) {
      GS_HIP(hipSetDevice(cx[r]->cfg.device));
      GS_HIP(hipStreamSynchronize(cx[r]->stream));
    }
  } else {
    Ctx& c = *cx[0];
    const uint32_t me = cm->rank, mme = lay.mn(me), unme = lay.un(me);
    GS_HIP(hipSetDevice(c.cfg.device));
    // pack: destination r's block [mme][un_r] at lay.ms_send_off(me, r)
    c.d_ms_send.alloc(std::max<size_t>(1, (size_t)mme * N));
    c.d_ms_sendh.alloc(std::max<size_t>(1, (size_t)mme * N));
    if (mme)
      for (uint32_t r = 0; r < P; r++) {
        const uint32_t u0 = lay.u0(r), un = lay.un(r);
        GS_HIP(hipMemcpy2DAsync(c.d_ms_send.p + lay.ms_send_off(me, r), (size_t)un * 8, c.d_ms_tc.p + u0,
                                (size_t)N * 8, (size_t)un * 8, mme, hipMemcpyDeviceToDevice, c.stream));
        GS_HIP(hipMemcpy2DAsync(c.d_ms_sendh.p + lay.ms_send_off(me, r), un, c.d_ms_hops.p + u0, N, un, mme,
                                hipMemcpyDeviceToDevice, c.stream));
      }
    c.d_tc_t.alloc((size_t)unme * B);
    c.d_hops_t.alloc((size_t)unme * B);
    const uint64_t pb = rccl_piece_bytes(), p8 = std::max<uint64_t>(1, pb / 8);
    coll_group_start(cm);
    for (uint32_t r = 0; r < P; r++) {
      const uint64_t n = lay.ms_count(me, r), off = lay.ms_send_off(me, r);
      for (uint64_t k = 0; k < n; k += p8)
        coll_Send(cm, c.d_ms_send.p + off + k, std::min(p8, n - k), ncclUint64, (int)r, c.stream);
      for (uint64_t k = 0; k < n; k += pb)
        coll_Send(cm, c.d_ms_sendh.p + off + k, std::min(pb, n - k), ncclUint8, (int)r, c.stream);
    }
    for (uint32_t p = 0; p < P; p++) {
      const uint64_t n = lay.ms_count(p, me), off = lay.ms_recv_off(p, me);
      for (uint64_t k = 0; k < n; k += p8)
        coll_Recv(cm, c.d_tc_t.p + off + k, std::min(p8, n - k), ncclUint64, (int)p, c.stream);
      for (uint64_t k = 0; k < n; k += pb)
        coll_Recv(cm, c.d_hops_t.p + off + k, std::min(pb, n - k), ncclUint8, (int)p, c.stream);
    }
    coll_group_end(cm);
    GS_HIP(hipStreamSynchronize(c.stream));
  }
  // 3. own peers' rows into the sinks
  if (!sinks) return;
  for (uint32_t i = 0; i < nctx; i++) {
    Ctx& c = *cx[i];
    const uint32_t me = cm->local ? i : cm->rank, un = lay.un(me);
    GS_HIP(hipSetDevice(c.cfg.device));
    deliver_rows(c, B, un, &sinks[i], i0);
    GS_HIP(hipStreamSynchronize(c.stream));
  }
}

// Counters of every part before a batch; restored when the peer protocols'
// eager result is discarded (lazy gossip can change the batch).
void save_counters(Ctx** cx, uint32_t nctx) {
  for (uint32_t i = 0; i < nctx; i++) {
    Ctx& c = *cx[i];
    GS_HIP(hipSetDevice(c.cfg.device));
    c.d_cnt_save.alloc(C_COUNT);
    GS_HIP(hipMemcpyAsync(c.d_cnt_save.p, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToDevice, c.stream));
  }
}

void gossip_to_ms(gs_comm* cm, Ctx** cx, uint32_t nctx, const gs_publish* sched, uint64_t i0, uint32_t B,
                  const gs_result_sink* sinks) {
  for (uint32_t i = 0; i < nctx; i++) {
    Ctx& c = *cx[i];
    part_abort(c);
    GS_HIP(hipSetDevice(c.cfg.device));
    GS_HIP(hipMemcpyAsync(c.d_counters.p, c.d_cnt_save.p, C_COUNT * 8, hipMemcpyDeviceToDevice, c.stream));
    GS_HIP(hipStreamSynchronize(c.stream));
    c.stats.gossip_fallback_batches++;
  }
  run_batch_ms(cm, cx, nctx, sched, i0, B, sinks);
}

// The list pass over partitioned rows: every part runs the
// window passes of gs_run over its own rows; between passes the parts agree
// on the pass control (records emitted, min pending key, error word) and
// exchange the pass's records, packed, with every peer's count and offset.
// Returns false, with every part's state and counters as before, when the
// list pass cannot take the batch (ring bound, memory, a knob) or a candidate
// list overflowed: the caller runs the push protocol instead.
bool run_batch_lp(gs_comm* cm, Ctx** cx, uint32_t nctx, const gs_publish* sched, uint64_t i0, uint32_t B,
                  const gs_result_sink* sinks) {
  const uint32_t P = cm->nranks, N = cx[0]->cfg.peers;
  std::vector<uint64_t> smin(nctx, INF64);
  uint64_t bad = 0;  // some part cannot take the batch on the list pass
  for (uint32_t i = 0; i < nctx; i++) {
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    if (!cm->local) {
      std::string why;
      gs_status code = GS_OK;
      bool ok = false;
      try {
        ok = part_lp_begin(*cx[i], sched + i0, B);
        if (ok) smin[i] = part_lp_seed_min(*cx[i]);
      } catch (const Error& e) {
        code = e.code;
        why = e.msg;
      }
      rank_status(cm, *cx[i], code != GS_OK);
      if (code != GS_OK) throw Error(code, why);
      bad |= ok ? 0u : 1u;
    } else if (!part_lp_begin(*cx[i], sched + i0, B)) {
      bad = 1;
    }
  }
  if (cm->local && !bad)  // every part's setup enqueued: now wait for each one's seeds
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      smin[i] = part_lp_seed_min(*cx[i]);
    }
  if (!cm->local) {
    uint64_t mine[2] = {bad, ~smin[0]}, all[2 * 64];
    rank_gather(cm, *cx[0], mine, 2, all);
    bad = 0;
    smin[0] = INF64;
    for (uint32_t k = 0; k < P; k++) {
      bad |= all[2 * k];
      smin[0] = std::min(smin[0], ~all[2 * k + 1]);
    }
  }
  if (bad) {
    for (uint32_t i = 0; i < nctx; i++) part_lp_abort(*cx[i]);
    return false;
  }
  uint64_t key = *std::min_element(smin.begin(), smin.end());
  for (uint32_t i = 0; i < nctx; i++) {
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    part_lp_set(*cx[i], 0, key);  // slot 2 as pass 0 reads it: no records, the min seeded key
  }
  std::vector<size_t> nev(nctx, 0);
  auto ev = [&](uint32_t i) {
    Ctx& c = *cx[i];
    while (c.ev_pool.size() <= nev[i]) {
      hipEvent_t e;
      GS_HIP(hipEventCreate(&e));
      c.ev_pool.push_back(e);
    }
    GS_HIP(hipEventRecord(c.ev_pool[nev[i]++], c.stream));
  };
  const PartLayout lay{P, N, B};
  const size_t RB = 8;  // bytes per record
  std::vector<uint64_t> st((size_t)P * 4);  // per part: mode, records, min pending, error word
  // the record exchange: routed per destination part (at most PART_ROUTE_PMAX
  // parts), or every part's records to every part. Loop-back parts on one
  // device route by default, each part's pack storing straight into the
  // destination contexts (no copies); ranks gather by default. GS_PART_ROUTE
  // = 1 / 0 forces routed / gathered (loop-back routed then goes through send
  // segments and copies, as ranks do, when GS_PART_DIRECT=0).
  const char* rte = getenv("GS_PART_ROUTE");
  bool one_dev = cm->local != 0;
  for (uint32_t i = 1; i < nctx; i++) one_dev = one_dev && cx[i]->cfg.device == cx[0]->cfg.device;
  const char* dre = getenv("GS_PART_DIRECT");
  const bool direct_ok = one_dev && P <= PART_ROUTE_PMAX && !(dre && *dre && atoi(dre) == 0);
  const bool routed = P <= PART_ROUTE_PMAX && ((rte && *rte) ? atoi(rte) != 0 : direct_ok);
  const bool direct = routed && direct_ok;
  for (;;) {
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      if (cx[i]->timing) ev(i);
      part_lp_pass(*cx[i]);
      if (cx[i]->timing) ev(i);
    }
    const bool dev_ctl = one_dev && P <= PART_ROUTE_PMAX;  // the parts' control combined on the device
    if (dev_ctl) {
      part_lp_combine(cx, P, st.data());
    } else if (cm->local) {
      for (uint32_t i = 0; i < nctx; i++) {  // every part's control read in flight, then each one waited for
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        part_lp_read_enqueue(*cx[i]);
      }
      for (uint32_t i = 0; i < nctx; i++) {
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        part_lp_read_wait(*cx[i], &st[(size_t)i * 4]);
      }
    } else {
      uint64_t mine[4];
      part_lp_read(*cx[0], mine);
      rank_gather(cm, *cx[0], mine, 4, st.data());
    }
    uint64_t recs = 0, minp = INF64, err = 0;
    for (uint32_t p = 0; p < P; p++) {
      recs += st[(size_t)p * 4 + 1];
      minp = std::min(minp, st[(size_t)p * 4 + 2]);
      err |= st[(size_t)p * 4 + 3];
    }
    if (err & (ERR_LIST | ERR_RING)) {  // lost entries somewhere: the push protocol takes the batch
      for (uint32_t i = 0; i < nctx; i++) {
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        part_lp_abort(*cx[i]);
      }
      return false;
    }
    if (st[0] == 0) break;  // pass mode DONE (PM_DONE, gs_pull_kernel.h): grid- and part-uniform
    if (!dev_ctl)
      for (uint32_t i = 0; i < nctx; i++) {
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        part_lp_set(*cx[i], recs, minp);
      }
    if (!recs) continue;  // the next pass emits a window: it reads no records
    std::vector<uint64_t> base(P + 1, 0), cnt(P);
    for (uint32_t p = 0; p < P; p++) cnt[p] = st[(size_t)p * 4 + 1];
    if (direct) {  // every part stores its routed records into the destinations (gathered bases, holes allowed)
      lp_bases(cnt.data(), P, base.data());
      for (uint32_t i = 0; i < nctx; i++) cx[i]->d_rpk.alloc(recs);  // (before any pack stores into it)
      for (uint32_t i = 0; i < nctx; i++) {
        part_lp_pack_route_direct(cx, P, i, base[i]);
        if (!cx[i]->part_xev) GS_HIP(hipEventCreateWithFlags(&cx[i]->part_xev, hipEventDisableTiming));
        GS_HIP(hipEventRecord(cx[i]->part_xev, cx[i]->stream));
      }
      for (uint32_t q = 0; q < nctx; q++)  // the next pass of q reads what every part stored into it
        for (uint32_t i = 0; i < nctx; i++)
          if (i != q) GS_HIP(hipStreamWaitEvent(cx[q]->stream, cx[i]->part_xev, 0));
      continue;
    }
    if (routed) {  // each part receives only the records with a receiver it owns (gs_layout.h lp_route_bases)
      std::vector<uint64_t> route((size_t)P * P), bq(P);
      for (uint32_t i = 0; i < nctx; i++) {
        const uint32_t me = cm->local ? i : cm->rank;
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        cx[i]->d_rpk.alloc(recs);
        part_lp_pack_route(*cx[i], P, me, cnt[me]);
      }
      if (cm->local) {
        for (uint32_t i = 0; i < nctx; i++) {
          GS_HIP(hipSetDevice(cx[i]->cfg.device));
          part_lp_route_read(*cx[i], P, &route[(size_t)i * P]);  // (every pack done)
        }
        for (uint32_t q = 0; q < nctx; q++) {
          Ctx& d = *cx[q];
          GS_HIP(hipSetDevice(d.cfg.device));
          lp_route_bases(route.data(), P, q, bq.data());
          for (uint32_t p = 0; p < nctx; p++) {
            if (p == q) continue;
            Ctx& src = *cx[p];
            const uint64_t n = route[(size_t)p * P + q], cap = std::max<uint64_t>(cnt[p], 1);
            const uint32_t u0 = lay.u0(p), un = lay.un(p);
            if (n) GS_HIP(hipMemcpyAsync(d.d_rpk.p + bq[p], src.d_rsend.p + (size_t)q * cap, n * RB,
                                         hipMemcpyDeviceToDevice, d.stream));
            GS_HIP(hipMemcpyAsync(d.d_rcg.p + u0, src.d_rrcg.p + (size_t)q * un, un * 4, hipMemcpyDeviceToDevice,
                                  d.stream));
            GS_HIP(hipMemcpyAsync(d.d_roffg.p + u0, src.d_rroff.p + (size_t)q * un, un * 8, hipMemcpyDeviceToDevice,
                                  d.stream));
          }
          part_lp_route_fix(d, P, q, bq.data());
        }
        for (uint32_t q = 0; q < nctx; q++) GS_HIP(hipStreamSynchronize(cx[q]->stream));  // sources reused next pass
      } else {
        Ctx& c = *cx[0];
        const uint32_t me = cm->rank;
        coll_AllGather(cm, c.d_pkcur.p, cm->d_scratch, P, ncclUint64, c.stream);  // row p: p's counts
        GS_HIP(hipMemcpyAsync(route.data(), cm->d_scratch, (size_t)P * P * 8, hipMemcpyDeviceToHost, c.stream));
        GS_HIP(hipStreamSynchronize(c.stream));
        lp_route_bases(route.data(), P, me, bq.data());
        const uint64_t piece = std::max<uint64_t>(1, rccl_piece_bytes() / RB);
        const uint64_t mycap = std::max<uint64_t>(cnt[me], 1);
        const uint32_t myun = lay.un(me);
        coll_group_start(cm);
        for (uint32_t d = 0; d < P; d++) {
          if (d == me) continue;
          const uint64_t n = route[(size_t)me * P + d];
          const uint64_t* src = c.d_rsend.p + (size_t)d * mycap;
          for (uint64_t k = 0; k < n; k += piece)
            coll_Send(cm, src + k, std::min(piece, n - k), ncclUint64, (int)d, c.stream);
          coll_Send(cm, c.d_rrcg.p + (size_t)d * myun, myun, ncclUint32, (int)d, c.stream);
          coll_Send(cm, c.d_rroff.p + (size_t)d * myun, myun, ncclUint64, (int)d, c.stream);
        }
        for (uint32_t sr = 0; sr < P; sr++) {
          if (sr == me) continue;
          const uint64_t n = route[(size_t)sr * P + me];
          const uint32_t u0 = lay.u0(sr), un = lay.un(sr);
          for (uint64_t k = 0; k < n; k += piece)
            coll_Recv(cm, c.d_rpk.p + bq[sr] + k, std::min(piece, n - k), ncclUint64, (int)sr, c.stream);
          coll_Recv(cm, c.d_rcg.p + u0, un, ncclUint32, (int)sr, c.stream);
          coll_Recv(cm, c.d_roffg.p + u0, un, ncclUint64, (int)sr, c.stream);
        }
        coll_group_end(cm);
        part_lp_route_fix(c, P, me, bq.data());
      }
      continue;
    }
    // gathered: every part's whole record range to every part
    lp_bases(cnt.data(), P, base.data());
    for (uint32_t i = 0; i < nctx; i++) {
      const uint32_t me = cm->local ? i : cm->rank;
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      cx[i]->d_rpk.alloc(recs);
      part_lp_pack(*cx[i], base[me], st[(size_t)me * 4 + 1]);
    }
    if (cm->local) {
      for (uint32_t i = 0; i < nctx; i++) GS_HIP(hipStreamSynchronize(cx[i]->stream));  // every pack done
      for (uint32_t q = 0; q < nctx; q++) {  // every other part's range (each packed its own in place)
        Ctx& d = *cx[q];
        GS_HIP(hipSetDevice(d.cfg.device));
        for (uint32_t p = 0; p < nctx; p++) {
          if (p == q) continue;
          Ctx& src = *cx[p];
          const uint64_t n = cnt[p], u0 = lay.u0(p), un = lay.un(p);
          if (n) GS_HIP(hipMemcpyAsync(d.d_rpk.p + base[p], src.d_rpk.p + base[p], n * RB, hipMemcpyDeviceToDevice,
                                       d.stream));
          GS_HIP(hipMemcpyAsync(d.d_rcg.p + u0, src.d_rcg.p + u0, un * 4, hipMemcpyDeviceToDevice, d.stream));
          GS_HIP(hipMemcpyAsync(d.d_roffg.p + u0, src.d_roffg.p + u0, un * 8, hipMemcpyDeviceToDevice, d.stream));
        }
      }
      for (uint32_t q = 0; q < nctx; q++) GS_HIP(hipStreamSynchronize(cx[q]->stream));  // sources reused next pass
    } else {
      Ctx& c = *cx[0];
      const uint32_t me = cm->rank;
      const uint64_t piece = std::max<uint64_t>(1, rccl_piece_bytes() / RB);
      const uint64_t myn = cnt[me], myu0 = lay.u0(me), myun = lay.un(me);
      const uint64_t* mine = c.d_rpk.p + base[me];  // packed in place (part_lp_pack): the own range stays
      coll_group_start(cm);
      for (uint32_t d = 0; d < P; d++) {
        if (d == me) continue;
        for (uint64_t k = 0; k < myn; k += piece)
          coll_Send(cm, mine + k, std::min(piece, myn - k), ncclUint64, (int)d, c.stream);
        coll_Send(cm, c.d_rcg.p + myu0, myun, ncclUint32, (int)d, c.stream);
        coll_Send(cm, c.d_roffg.p + myu0, myun, ncclUint64, (int)d, c.stream);
      }
      for (uint32_t sr = 0; sr < P; sr++) {
        if (sr == me) continue;
        const uint64_t n = cnt[sr], u0 = lay.u0(sr), un = lay.un(sr);
        for (uint64_t k = 0; k < n; k += piece)
          coll_Recv(cm, c.d_rpk.p + base[sr] + k, std::min(piece, n - k), ncclUint64, (int)sr, c.stream);
        coll_Recv(cm, c.d_rcg.p + u0, un, ncclUint32, (int)sr, c.stream);
        coll_Recv(cm, c.d_roffg.p + u0, un, ncclUint64, (int)sr, c.stream);
      }
      coll_group_end(cm);
    }
  }
  for (uint32_t i = 0; i < nctx; i++) {  // pass times (timing on)
    Ctx& c = *cx[i];
    if (!c.timing) continue;
    GS_HIP(hipSetDevice(c.cfg.device));
    GS_HIP(hipStreamSynchronize(c.stream));
    double front = 0;
    for (size_t q = 0; q + 1 < nev[i]; q += 2) {
      float x = 0;
      GS_HIP(hipEventElapsedTime(&x, c.ev_pool[q], c.ev_pool[q + 1]));
      front += x;
    }
    c.stats.frontier_ms += front;
    c.stats.relax_ms += front;
  }
  // completion + the lazy-gossip no-op proof of every part
  bool ok = true;
  for (uint32_t i = 0; i < nctx; i++) {  // every part's completion enqueued, then each one waited for
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    part_lp_end_enqueue(*cx[i], sinks ? &sinks[i] : nullptr);
  }
  for (uint32_t i = 0; i < nctx; i++) {
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    ok = part_lp_end_check(*cx[i]) && ok;
  }
  if (!cm->local && cx[0]->cfg.lazy_gossip) {
    uint64_t mine = ok ? 0 : 1, all[64];
    rank_gather(cm, *cx[0], &mine, 1, all);
    for (uint32_t k = 0; k < P; k++) ok = ok && !all[k];
  }
  if (!ok) {  // an IHAVE can land before the last delivery: the batch runs message-sharded with gossip
    gossip_to_ms(cm, cx, nctx, sched, i0, B, sinks);
    return true;
  }
  for (uint32_t i = 0; i < nctx; i++) {
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    part_dev_finish(*cx[i], sinks ? &sinks[i] : nullptr, i0);
  }
  return true;
}

// One batch of the partitioned protocol over this process's parts: the list
// pass when it can take the batch, else the push protocol (scan / routed
// export / receive per bucket).
void run_batch(gs_comm* cm, Ctx** cx, uint32_t nctx, const gs_publish* sched, uint64_t i0, uint32_t B,
               const gs_result_sink* sinks) {
  if (part_needs_ms(*cx[0], sched + i0, B)) {  // churn, IDONTWANT: the same decision on every rank
    run_batch_ms(cm, cx, nctx, sched, i0, B, sinks);
    return;
  }
  if (cx[0]->cfg.lazy_gossip) save_counters(cx, nctx);
  if (run_batch_lp(cm, cx, nctx, sched, i0, B, sinks)) return;
  const uint32_t P = cm->nranks;
  std::vector<uint64_t> key0(nctx);
  if (cm->local) {
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      key0[i] = part_begin(*cx[i], sched + i0, B);  // the seeded min is also left in ctrl[0]
    }
  } else {  // a rank whose batch set-up fails takes the others out with it
    GS_HIP(hipSetDevice(cx[0]->cfg.device));
    std::string why;
    gs_status code = GS_OK;
    try {
      key0[0] = part_begin(*cx[0], sched + i0, B);
    } catch (const Error& e) {
      code = e.code;
      why = e.msg;
    }
    rank_status(cm, *cx[0], code != GS_OK);
    if (code != GS_OK) throw Error(code, why);
  }
  // mat[s * P + d] = records part s sends to part d (this bucket)
  std::vector<uint64_t> mat((size_t)P * P), ctl(nctx);
  auto host_min_to_ctrl = [&](uint64_t k) {
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      cx[i]->h_pinned[0] = k;
      GS_HIP(hipMemcpyAsync(cx[i]->d_ctrl.p, cx[i]->h_pinned, 8, hipMemcpyHostToDevice, cx[i]->stream));
      GS_HIP(hipStreamSynchronize(cx[i]->stream));
    }
  };
  if (cm->local) host_min_to_ctrl(*std::min_element(key0.begin(), key0.end()));
  else coll_AllReduce(cm, cx[0]->d_ctrl.p, cx[0]->d_ctrl.p, 1, ncclUint64, ncclMin, cx[0]->stream);
  // timing (gs_set_timing): per part and bucket three events on its stream —
  // bucket start, scan + counts done (scan_ms), relax done (frontier_ms: the
  // routed export, the exchange and the receive-side relaxation)
  std::vector<size_t> nev(nctx, 0);
  auto ev = [&](uint32_t i) {
    Ctx& c = *cx[i];
    while (c.ev_pool.size() <= nev[i]) {
      hipEvent_t e;
      GS_HIP(hipEventCreate(&e));
      c.ev_pool.push_back(e);
    }
    GS_HIP(hipEventRecord(c.ev_pool[nev[i]++], c.stream));
  };
  for (;;) {
    // 1. scan + per-destination counts
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      if (cx[i]->timing) ev(i);
      part_dev_bucket(*cx[i], P);
      part_dev_scan_count(*cx[i], P);
      if (cx[i]->timing) ev(i);
    }
    // 2. the count matrix and the bucket key on the host (the one read per bucket)
    uint64_t key = INF64;
    if (cm->local) {
      for (uint32_t i = 0; i < nctx; i++) {
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        GS_HIP(hipMemcpyAsync(&mat[(size_t)i * P], cx[i]->d_dcnt.p, P * 8, hipMemcpyDeviceToHost, cx[i]->stream));
        GS_HIP(hipMemcpyAsync(&ctl[i], cx[i]->d_ctrl.p, 8, hipMemcpyDeviceToHost, cx[i]->stream));
      }
      for (uint32_t i = 0; i < nctx; i++) GS_HIP(hipStreamSynchronize(cx[i]->stream));
      key = ctl[0];
    } else {
      Ctx& c = *cx[0];
      coll_AllGather(cm, c.d_dcnt.p, cm->d_scratch, P, ncclUint64, c.stream);
      GS_HIP(hipMemcpyAsync(mat.data(), cm->d_scratch, (size_t)P * P * 8, hipMemcpyDeviceToHost, c.stream));
      GS_HIP(hipMemcpyAsync(&ctl[0], c.d_ctrl.p, 8, hipMemcpyDeviceToHost, c.stream));
      GS_HIP(hipStreamSynchronize(c.stream));
      key = ctl[0];
    }
    if (key == INF64) break;  // every part agrees: the MIN all-reduce made it the same everywhere
    // 3. export grouped by destination, exchange (all-to-all-v)
    std::vector<uint64_t> nrecv(nctx, 0);
    for (uint32_t i = 0; i < nctx; i++) {
      Ctx& c = *cx[i];
      const uint32_t me = cm->local ? i : cm->rank;
      uint64_t ns = 0, nr = 0;
      for (uint32_t d = 0; d < P; d++) ns += mat[(size_t)me * P + d];
      for (uint32_t s = 0; s < P; s++) nr += mat[(size_t)s * P + me];
      nrecv[i] = nr;
      GS_HIP(hipSetDevice(c.cfg.device));
      c.d_pout.alloc(std::max<uint64_t>(ns, 1));
      c.d_pin.alloc(std::max<uint64_t>(nr, 1));
      part_dev_export(c, P, c.d_pout.p);
    }
    const size_t RB = sizeof(gs_part_record);
    if (cm->local) {
      for (uint32_t i = 0; i < nctx; i++) GS_HIP(hipStreamSynchronize(cx[i]->stream));  // every export done
      for (uint32_t i = 0; i < nctx; i++) {  // part i receives from every s, in source order
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        uint64_t roff = 0;
        for (uint32_t s = 0; s < nctx; s++) {
          uint64_t soff = 0;
          for (uint32_t d = 0; d < i; d++) soff += mat[(size_t)s * P + d];
          const uint64_t n = mat[(size_t)s * P + i];
          if (n)
            GS_HIP(hipMemcpyAsync(cx[i]->d_pin.p + roff, cx[s]->d_pout.p + soff, n * RB, hipMemcpyDeviceToDevice,
                                  cx[i]->stream));
          roff += n;
        }
      }
    } else {
      Ctx& c = *cx[0];
      const uint32_t me = cm->rank;
      // peak buckets at 1M peers move GBs per pair: point-to-point transfers in
      // pieces of at most rccl_piece_bytes(); both ends cut the
      // same count the same way
      const uint64_t piece = std::max<uint64_t>(1, rccl_piece_bytes() / RB);
      coll_group_start(cm);
      uint64_t soff = 0, roff = 0;
      for (uint32_t d = 0; d < P; d++) {
        const uint64_t n = mat[(size_t)me * P + d];
        for (uint64_t k = 0; k < n; k += piece)
          coll_Send(cm, c.d_pout.p + soff + k, std::min(piece, n - k) * RB, ncclUint8, (int)d, c.stream);
        soff += n;
      }
      for (uint32_t s = 0; s < P; s++) {
        const uint64_t n = mat[(size_t)s * P + me];
        for (uint64_t k = 0; k < n; k += piece)
          coll_Recv(cm, c.d_pin.p + roff + k, std::min(piece, n - k) * RB, ncclUint8, (int)s, c.stream);
        roff += n;
      }
      coll_group_end(cm);
    }
    // 4. relax into own peers; next bucket = MIN over parts
    for (uint32_t i = 0; i < nctx; i++) {
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      part_dev_relax_next(*cx[i], cx[i]->d_pin.p, nrecv[i]);
      if (cx[i]->timing) ev(i);
    }
    if (cm->local) {
      for (uint32_t i = 0; i < nctx; i++) {
        GS_HIP(hipSetDevice(cx[i]->cfg.device));
        GS_HIP(hipMemcpyAsync(&ctl[i], cx[i]->d_ctrl.p, 8, hipMemcpyDeviceToHost, cx[i]->stream));
      }
      for (uint32_t i = 0; i < nctx; i++) GS_HIP(hipStreamSynchronize(cx[i]->stream));
      host_min_to_ctrl(*std::min_element(ctl.begin(), ctl.end()));
    } else {
      coll_AllReduce(cm, cx[0]->d_ctrl.p, cx[0]->d_ctrl.p, 1, ncclUint64, ncclMin, cx[0]->stream);
    }
  }
  for (uint32_t i = 0; i < nctx; i++) {  // bucket times (the loop ended on a stream sync)
    Ctx& c = *cx[i];
    if (!c.timing) continue;
    GS_HIP(hipSetDevice(c.cfg.device));
    GS_HIP(hipStreamSynchronize(c.stream));
    double scan = 0, front = 0;
    for (size_t q = 0; q + 2 < nev[i]; q += 3) {
      float x = 0, y = 0;
      GS_HIP(hipEventElapsedTime(&x, c.ev_pool[q], c.ev_pool[q + 1]));
      GS_HIP(hipEventElapsedTime(&y, c.ev_pool[q + 1], c.ev_pool[q + 2]));
      scan += x;
      front += y;
    }
    if (nev[i] % 3 == 2) {  // the last scan, which found no bucket left
      float x = 0;
      GS_HIP(hipEventElapsedTime(&x, c.ev_pool[nev[i] - 2], c.ev_pool[nev[i] - 1]));
      scan += x;
    }
    c.stats.scan_ms += scan;
    c.stats.frontier_ms += front;
    c.stats.relax_ms += scan + front;
  }
  // lazy gossip: the eager result stands only where every part proves it a no-op
  bool ok = true;
  for (uint32_t i = 0; i < nctx; i++) {
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    ok = part_dev_complete(*cx[i], sinks && sinks[i].summary) && ok;
  }
  if (!cm->local && cx[0]->cfg.lazy_gossip) {
    Ctx& c = *cx[0];
    c.h_pinned[0] = ok ? 1 : 0;
    GS_HIP(hipMemcpyAsync(cm->d_scratch + (size_t)P * P, c.h_pinned, 8, hipMemcpyHostToDevice, c.stream));
    coll_AllReduce(cm, cm->d_scratch + (size_t)P * P, cm->d_scratch + (size_t)P * P, 1, ncclUint64, ncclMin, c.stream);
    GS_HIP(hipMemcpyAsync(c.h_pinned, cm->d_scratch + (size_t)P * P, 8, hipMemcpyDeviceToHost, c.stream));
    GS_HIP(hipStreamSynchronize(c.stream));
    ok = c.h_pinned[0] != 0;
  }
  if (!ok) {
    gossip_to_ms(cm, cx, nctx, sched, i0, B, sinks);
    return;
  }
  for (uint32_t i = 0; i < nctx; i++) {
    GS_HIP(hipSetDevice(cx[i]->cfg.device));
    part_dev_finish(*cx[i], sinks ? &sinks[i] : nullptr, i0);
  }
}

}  // namespace

extern "C" gs_status gs_run_partitioned(gs_ctx* const* ctxs, uint32_t nctx, gs_comm* comm, const gs_publish* sched,
                                        uint64_t n_msgs, const gs_result_sink* sinks) {
  if (!ctxs || !nctx || !comm || (!sched && n_msgs)) return GS_EINVAL;
  for (uint32_t i = 0; i < nctx; i++)
    if (!ctxs[i]) return GS_EINVAL;
  Ctx* c0 = ctxs[0];
  try {
    if (comm->local ? nctx != comm->nranks : nctx != 1)
      c0->fail(GS_EINVAL, "gs_run_partitioned: pass one context per part (local) or this rank's context (RCCL)");
    for (uint32_t i = 0; sinks && i < nctx; i++)
      if (sinks[i].on_lat || (sinks[i].want & GS_WANT_LAT_MS))
        c0->fail(GS_EUNSUPPORTED, "gs_run_partitioned: the u16 latency stream (on_lat) is gs_run's");
    std::vector<Ctx*> cx(nctx);
    for (uint32_t i = 0; i < nctx; i++) {
      cx[i] = ctxs[i];
      if (!cx[i]->mesh_built) cx[i]->fail(GS_ESTATE, "gs_mesh_converge first");
      if (cx[i]->cfg.peers != c0->cfg.peers || cx[i]->cfg.batch != c0->cfg.batch)
        c0->fail(GS_EINVAL, "every part needs the same peers and batch");
      GS_HIP(hipSetDevice(cx[i]->cfg.device));
      part_set(*cx[i], comm->nranks, comm->local ? i : comm->rank);
    }
    if (!comm->local && c0->cfg.device != comm->device)
      c0->fail(GS_EINVAL, "the context and the communicator must use the same device");
    check_same_config(comm, *c0, sched, n_msgs);
    uint64_t i0 = 0;
    while (i0 < n_msgs) {  // batches of equal size and chunk count, at most cfg.batch messages
      uint64_t i1 = i0 + 1;
      while (i1 < n_msgs && i1 - i0 < c0->cfg.batch && sched[i1].msg_size == sched[i0].msg_size &&
             sched[i1].frags == sched[i0].frags)
        i1++;
      run_batch(comm, cx.data(), nctx, sched, i0, (uint32_t)(i1 - i0), sinks);
      i0 = i1;
    }
  } catch (const Error& e) {
    for (uint32_t i = 0; i < nctx; i++) part_abort(*ctxs[i]);  // no context is left mid-batch
    c0->last_error = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    for (uint32_t i = 0; i < nctx; i++) part_abort(*ctxs[i]);
    c0->last_error = e.what();
    return GS_ENOMEM;
  }
  return GS_OK;
}
