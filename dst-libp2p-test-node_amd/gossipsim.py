"""Python host mirror of the reference's test-node interface over libgossipsim.so.

The reference node (rust-test-node/src/main.rs) reads its knobs from the env
(env.rs:27-87), dials random peers (main.rs:303-389), accepts
`POST /publish {"topic","msgSize","version"}` (main.rs:50-56,146-221) and
prints `<tx_time> milliseconds: <latency>` per completed message (main.rs:93).
This module keeps those names and error behaviour on top of the C ABI in
include/gossipsim.h:

    cfg = PeerConfig.from_env()          # env.rs get_peer_details
    sim = Simulator(cfg)                 # SwarmBuilder + build_behaviour
    sim.set_topogen_links(...)           # shadow/topogen.py link graph
    sim.connect_gossipsub_peers()        # main.rs:303-389 -> CSR on the GPU
    sim.mesh_converge()                  # heartbeat GRAFT/PRUNE fixed point
    sim.publish(publisher, msg_size, t)  # POST /publish
    res = sim.run()                      # receive/forward/reassemble on the GPU
    sim.write_latency_log(path, res)     # awk-parseable arrival lines

Everything here is plumbing; all simulation work runs in the HIP library. The
library must be present: there is no CPU fallback (a missing .so raises).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GOSSIPSIM_LIB", os.path.join(HERE, "libgossipsim.so"))
ABI_VERSION = 10
MESH_W = 16
UNDELIVERED = np.uint64(0xFFFFFFFFFFFFFFFF)
MUXERS = {"yamux": 0, "quic": 1, "mplex": 2}
NODES = {"rust": 0, "go": 1, "nim": 2}  # GS_NODE_*: rust-test-node, go-test-node, nim gossipsub-queues
STATUS = {0: "GS_OK", -1: "GS_EINVAL", -2: "GS_ENOMEM", -3: "GS_EDEVICE", -4: "GS_ESTATE",
          -5: "GS_ERANGE", -6: "GS_EUNSUPPORTED"}

u32, u64, i32, u8 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint8
P = ctypes.POINTER


class GsConfig(ctypes.Structure):
    _fields_ = [(n, u32) for n in (
        "abi_version", "peers", "connect_to", "dial_extra", "max_connections", "fragments",
        "muxer", "signed_msgs", "d", "d_lo", "d_hi", "d_lazy", "d_out", "gossip_factor_milli")] + [
        ("heartbeat_ns", u64), ("backoff_ns", u64)] + [
        (n, u32) for n in ("flood_publish", "idontwant", "lazy_gossip", "self_log")] + [
        ("seed", u64), ("device", i32), ("batch", u32), ("history_gossip", u32), ("hb_phase_ns", u64)] + [
        (n, u32) for n in ("churn_ppm", "churn_down", "churn_horizon", "node", "sub_graft", "hs_rtts")]


class GsPublish(ctypes.Structure):
    _fields_ = [("t_pub_ns", u64), ("publisher", u32), ("msg_size", u32), ("frags", u32), ("reserved", u32)]


HIST_BINS, HIST_MS = 64, 100  # GS_HIST_BINS / GS_HIST_MS


class GsMsgSummary(ctypes.Structure):
    _fields_ = [("delivered", u64), ("lat_sum_ms", u64), ("p50_ms", u32), ("p95_ms", u32), ("max_ms", u32),
                ("reserved", u32), ("hist", u32 * HIST_BINS)]


BLOCK_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, u64, u32, u32, P(u64), P(u8))
LAT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, u64, u32, u32, P(ctypes.c_uint16))


class GsResultSink(ctypes.Structure):
    _fields_ = [("t_complete_ns", P(u64)), ("hops", P(u8)), ("on_block", BLOCK_FN), ("user", ctypes.c_void_p),
                ("block_msgs", u32), ("want", u32), ("summary", P(GsMsgSummary)), ("on_lat", LAT_FN)]


WANT_T_COMPLETE, WANT_HOPS, WANT_LAT_MS = 1, 2, 4  # gs_result_sink.want (GS_WANT_*)
LAT_NONE = 0xFFFF  # GS_LAT_NONE: the peer logs nothing for the message


class GsStats(ctypes.Structure):
    _fields_ = [(n, u64) for n in (
        "messages", "deliveries", "frag_deliveries", "relaxations", "bytes_alg",
        "latency_sum_ms", "latency_max_ms", "relax_launches", "buckets")] + [
        ("relax_ms", ctypes.c_double), ("run_ms", ctypes.c_double), ("relax_bytes_alg", u64),
        ("pushes", u64), ("scan_ms", ctypes.c_double), ("frontier_ms", ctypes.c_double),
        ("gossip_iwant", u64), ("gossip_noop_msgs", u64), ("gossip_fallback_batches", u64), ("batches", u64),
        ("list_pull_batches", u64), ("ms_batches", u64), ("gossip_list_batches", u64)]


class GsInjector(ctypes.Structure):
    _fields_ = [("start_ns", u64), ("delay_ns", u64), ("msg_size", u32), ("messages", u32), ("peers", u32),
                ("reserved", u32)]


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, P(u64), u64, P(u64))
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, P(ctypes.c_void_p), P(u64), P(ctypes.c_void_p), P(u64))


class GsCommOps(ctypes.Structure):  # gs_comm_ops (ABI 10)
    _fields_ = [("user", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("exchange", EXCHANGE_FN)]


class GsPartRecord(ctypes.Structure):
    _fields_ = [("key", u64), ("start", u64), ("peer", u32), ("slot", u32)]


# Every symbol include/gossipsim.h declares, with its ctypes signature.
SIGNATURES = {
    "gs_config_default": (None, [P(GsConfig)]),
    "gs_config_preset": (i32, [P(GsConfig), u32]),
    "gs_write_node_log": (i32, [P(GsConfig), ctypes.c_char_p, P(GsPublish), u64, P(u64)]),
    "gs_log_open": (i32, [P(GsConfig), ctypes.c_char_p, P(ctypes.c_void_p)]),
    "gs_log_write": (i32, [ctypes.c_void_p, P(GsPublish), u32, P(u64)]),
    "gs_log_write_lat": (i32, [ctypes.c_void_p, P(GsPublish), u32, P(ctypes.c_uint16)]),
    "gs_log_close": (i32, [ctypes.c_void_p]),
    "gs_config_from_env": (i32, [P(GsConfig), ctypes.c_char_p, ctypes.c_size_t]),
    "gs_wire_bytes": (u64, [u64, u32, u32]),
    "gs_wire_packets": (None, [u64, u32, u32, P(u64), P(u64)]),
    "gs_control_packets": (None, [u32, u32, u32, P(u64), P(u64), P(u64)]),
    "gs_write_shadow_heartbeat": (i32, [ctypes.c_char_p, u32, P(u64), u64]),
    "gs_links_from_gml": (i32, [ctypes.c_char_p, u32, u32, P(u32), P(u64), P(u64), P(u64)]),
    "gs_shadow_hosts": (i32, [ctypes.c_char_p, u32, P(u8)]),
    "gs_write_node_metrics": (i32, [P(GsConfig), ctypes.c_char_p, P(u64), P(u8), P(u64)]),
    "gs_set_traffic": (i32, [ctypes.c_void_p, u32]),
    "gs_get_traffic": (i32, [ctypes.c_void_p, P(u64)]),
    "gs_topogen_links": (i32, [u32, u32, u32, u32, u32, u32, P(u64), P(u64)]),
    "gs_schedule_runsh": (i32, [u32, u32, u32, u32, u64, u64, u32, P(GsPublish)]),
    "gs_shadow_injector": (i32, [ctypes.c_char_p, P(GsInjector)]),
    "gs_read_schedule": (i32, [ctypes.c_char_p, P(GsPublish), u64, P(u64)]),
    "gs_write_latency_log": (i32, [ctypes.c_char_p, P(GsPublish), u64, u32, P(u64), u32]),
    "gs_create": (i32, [P(GsConfig), P(ctypes.c_void_p)]),
    "gs_destroy": (i32, [ctypes.c_void_p]),
    "gs_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "gs_set_links": (i32, [ctypes.c_void_p, u32, P(u64), P(u64), P(u64), P(u8)]),
    "gs_build_topology": (i32, [ctypes.c_void_p]),
    "gs_graph_info": (i32, [ctypes.c_void_p, P(u32), P(u64), P(u32)]),
    "gs_get_csr": (i32, [ctypes.c_void_p, P(u64), P(u32), P(u8)]),
    "gs_mesh_converge": (i32, [ctypes.c_void_p, u32, P(u32)]),
    "gs_get_mesh": (i32, [ctypes.c_void_p, P(u32), P(u8)]),
    "gs_run": (i32, [ctypes.c_void_p, P(GsPublish), u64, P(GsResultSink)]),
    "gs_get_stats": (i32, [ctypes.c_void_p, P(GsStats)]),
    "gs_get_config": (i32, [ctypes.c_void_p, P(GsConfig)]),
    "gs_save_state": (i32, [ctypes.c_void_p, ctypes.c_char_p]),
    "gs_load_state": (i32, [ctypes.c_char_p, i32, P(ctypes.c_void_p)]),
    "gs_reset_stats": (i32, [ctypes.c_void_p]),
    "gs_set_timing": (i32, [ctypes.c_void_p, u32]),
    "gs_set_partition": (i32, [ctypes.c_void_p, u32, u32]),
    "gs_part_begin": (i32, [ctypes.c_void_p, P(GsPublish), u64, P(u64)]),
    "gs_part_scan": (i32, [ctypes.c_void_p, u64, ctypes.c_void_p, u64, P(u64), P(u64)]),
    "gs_part_relax": (i32, [ctypes.c_void_p, u64, ctypes.c_void_p, u64, P(u64)]),
    "gs_part_finish": (i32, [ctypes.c_void_p, P(GsResultSink)]),
    "gs_comm_get_id": (i32, [ctypes.c_char_p]),
    "gs_comm_init": (i32, [u32, u32, ctypes.c_char_p, i32, P(ctypes.c_void_p)]),
    "gs_comm_init_local": (i32, [u32, P(ctypes.c_void_p)]),
    "gs_comm_init_ops": (i32, [u32, u32, ctypes.c_void_p, i32, P(ctypes.c_void_p)]),
    "gs_comm_check": (i32, [ctypes.c_void_p]),
    "gs_comm_destroy": (i32, [ctypes.c_void_p]),
    "gs_run_partitioned": (i32, [P(ctypes.c_void_p), u32, ctypes.c_void_p, P(GsPublish), u64, P(GsResultSink)]),
}
COMM_ID_BYTES = 128
GS_EINVAL = -1
GS_ERANGE = -5
KEY_NONE = (1 << 64) - 1  # empty-bucket marker of the partitioned protocol

_lib = None


def lib():
    """Load libgossipsim.so; raise if it is missing (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libgossipsim.so not built at %s: run __graft_entry__.build() "
                               "(make -C dst-libp2p-test-node_amd)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class GossipSimError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("%s (%d): %s" % (STATUS.get(status, "?"), status, msg))
        self.status = status


def _ptr(a, ct):
    return a.ctypes.data_as(P(ct))


def wire_bytes(payload, muxer="yamux", signed=True):
    return int(lib().gs_wire_bytes(payload, MUXERS[muxer] if isinstance(muxer, str) else muxer,
                                   1 if signed else 0))


def wire_packets(payload, muxer="yamux", signed=True):
    """-> (packets, header bytes) of one fragment send (the model of wire_bytes)."""
    pk, hd = u64(), u64()
    lib().gs_wire_packets(payload, MUXERS[muxer] if isinstance(muxer, str) else muxer, 1 if signed else 0,
                          ctypes.byref(pk), ctypes.byref(hd))
    return pk.value, hd.value


CTRL_KINDS = {"ihave": 0, "iwant": 1, "ack": 2}


def control_packets(kind, node="rust", muxer="yamux"):
    """-> (wire bytes, packets, header bytes) of one IHAVE / IWANT RPC (one
    message id) or one pure ACK packet (gs_control_packets)."""
    b, pk, hd = u64(), u64(), u64()
    lib().gs_control_packets(CTRL_KINDS.get(kind, kind), NODES.get(node, node) if isinstance(node, str) else node,
                             MUXERS[muxer] if isinstance(muxer, str) else muxer,
                             ctypes.byref(b), ctypes.byref(pk), ctypes.byref(hd))
    return b.value, pk.value, hd.value


TRAFFIC_COLS = ("tx_bytes", "rx_bytes", "tx_packets", "rx_packets", "tx_header_bytes", "rx_header_bytes",
                "received", "published", "tx_ctrl_packets", "rx_ctrl_packets", "tx_ctrl_header_bytes",
                "rx_ctrl_header_bytes")


def write_shadow_heartbeat(path, traffic, sim_seconds=900):
    """Per-peer traffic [N, len(TRAFFIC_COLS)] as Shadow tracker "[node]" lines (shadow/summary_shadowlog.awk);
    sim_seconds defaults to topogen's 15-minute stop time (shadow/topogen.py:82)."""
    tr = np.ascontiguousarray(traffic, np.uint64)
    rc = lib().gs_write_shadow_heartbeat(path.encode(), tr.shape[0], _ptr(tr, u64), sim_seconds)
    if rc:
        raise GossipSimError(rc, "gs_write_shadow_heartbeat failed")


def write_node_metrics(cfg, path, row_ptr, mesh_count, traffic):
    """OpenMetrics text of the test node's metrics for every peer (gs_write_node_metrics)."""
    row = np.ascontiguousarray(row_ptr, np.uint64)
    mc = np.ascontiguousarray(mesh_count, np.uint8)
    tr = np.ascontiguousarray(traffic, np.uint64)
    rc = lib().gs_write_node_metrics(ctypes.byref(cfg.c), path.encode(), _ptr(row, u64), _ptr(mc, u8), _ptr(tr, u64))
    if rc:
        raise GossipSimError(rc, "gs_write_node_metrics failed")


def links_from_gml(path, shortest=False):
    """Shadow network graph (network_topology.gml) -> (lat_ns[V,V], bw_up[V], bw_down[V])."""
    V = u32()
    cap = 16
    while True:
        lat, up, dn = np.zeros(cap * cap, np.uint64), np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
        rc = lib().gs_links_from_gml(path.encode(), 1 if shortest else 0, cap, ctypes.byref(V), _ptr(lat, u64),
                                     _ptr(up, u64), _ptr(dn, u64))
        if rc == GS_ERANGE and V.value > cap:
            cap = V.value
            continue
        if rc:
            raise GossipSimError(rc, "cannot ingest %s" % path)
        n = V.value
        return lat[:n * n].reshape(n, n), up[:n], dn[:n]


def shadow_hosts(path, peers):
    """shadow.yaml hosts pod-<i> -> network_node_id, as the stage_of_peer array of set_links."""
    st = np.zeros(peers, np.uint8)
    rc = lib().gs_shadow_hosts(path.encode(), peers, _ptr(st, u8))
    if rc:
        raise GossipSimError(rc, "cannot map the %d peers of %s" % (peers, path))
    return st


def topogen_links(stages=1, min_bw=50, max_bw=50, min_lat=100, max_lat=100, shortest=False):
    """shadow/topogen.py:39-71 -> (lat_ns[S,S], bw_bps[S]); defaults = topogen.py:15-20."""
    lat = np.zeros(stages * stages, np.uint64)
    bw = np.zeros(stages, np.uint64)
    rc = lib().gs_topogen_links(stages, min_bw, max_bw, min_lat, max_lat, 1 if shortest else 0,
                                _ptr(lat, u64), _ptr(bw, u64))
    if rc:
        raise GossipSimError(rc, "invalid topogen parameters")
    return lat.reshape(stages, stages), bw


def schedule_runsh(n_msgs, peers, publisher_id, rotation, t0_ns, delay_ns, msg_size):
    """shadow/run.sh:34-36 publisher/rotation/delay -> structured schedule array."""
    out = (GsPublish * n_msgs)()
    rc = lib().gs_schedule_runsh(n_msgs, peers, publisher_id, rotation, t0_ns, delay_ns, msg_size,
                                 out)
    if rc:
        raise GossipSimError(rc, "invalid schedule")
    return out


def shadow_injector(path):
    """The injector process of a Shadow config (traffic_sync.py args + start_time, topogen.py:125-136)."""
    inj = GsInjector()
    rc = lib().gs_shadow_injector(path.encode(), ctypes.byref(inj))
    if rc:
        raise GossipSimError(rc, "no injector host in %s" % path)
    return {n: getattr(inj, n) for n, _ in GsInjector._fields_ if n != "reserved"}


def read_schedule(path):
    """Schedule file rows "t_pub_ns publisher msg_size [frags]" -> GsPublish array."""
    n = u64()
    rc = lib().gs_read_schedule(path.encode(), None, 0, ctypes.byref(n))
    if rc not in (0, GS_ERANGE):
        raise GossipSimError(rc, "malformed schedule %s" % path)
    out = (GsPublish * n.value)()
    rc = lib().gs_read_schedule(path.encode(), out, n.value, ctypes.byref(n))
    if rc:
        raise GossipSimError(rc, "malformed schedule %s" % path)
    return out


# Schedule constants of the benchmark workload: Shadow epoch 2000-01-01 plus the
# injector start (shadow/topogen.py:130), 1000 ms spacing and publisher
# (6 + i) mod N with rotation (shadow/README.md:57, run.sh:34-36). The injector
# POSTs over a fresh TCP connection across the 1 ms injector-hub links
# (topogen.py:64-69): the request reaches the node 1.5 round trips = 3 ms after
# the injector's send, and the node stamps tx_time then (main.rs:105-111).
# Heartbeats tick on whole seconds (process start 5 s, topogen.py:106, plus
# libp2p-gossipsub's 5 s heartbeat_initial_delay; hb_phase_ns = 0 is the same
# phase), so a publish lands 3 ms after a heartbeat.
INJECTOR_START_NS = 946684800_000_000_000 + 500_000_000_000
HTTP_TRANSIT_NS = 3_000_000
T0_NS = INJECTOR_START_NS + HTTP_TRANSIT_NS
# Heartbeat 0 when every node starts (Shadow starts processes at 5 s,
# shadow/topogen.py:106): the phase churn runs need.
SHADOW_START_NS = 946684800_000_000_000 + 5_000_000_000
DELAY_NS = 1_000_000_000
PUBLISHER0 = 6


def shard_messages(step, rank, world, batch, peers, msg_size):
    """Message-batch sharding across ranks: global message index
    (step*world + rank)*batch + q; messages are independent given the frozen mesh,
    so ranks share nothing on the data path."""
    idx = (np.uint64(step) * np.uint64(world) + np.uint64(rank)) * np.uint64(batch) + \
        np.arange(batch, dtype=np.uint64)
    t = np.uint64(T0_NS) + idx * np.uint64(DELAY_NS)
    pub = ((np.uint64(PUBLISHER0) + idx) % np.uint64(peers)).astype(np.uint32)
    return t, pub, np.full(batch, msg_size, np.uint32)


class PeerConfig:
    """Knobs of env.rs:14-25 + gossipsub ConfigBuilder (main.rs:223-241)."""

    def __init__(self, **kw):
        """Knobs over the defaults of `node` (rust | go | nim, gs_config_preset; default rust)."""
        self.c = GsConfig()
        node = kw.pop("node", 0)
        node = NODES[node] if isinstance(node, str) else int(node)
        rc = lib().gs_config_preset(ctypes.byref(self.c), node)
        if rc:
            raise GossipSimError(rc, "unknown node flavour %r" % node)
        for k, v in kw.items():
            if k == "muxer" and isinstance(v, str):
                v = MUXERS[v]
            if not hasattr(self.c, k):
                raise AttributeError("unknown knob %s" % k)
            setattr(self.c, k, v)

    @classmethod
    def from_env(cls):
        """get_peer_details (env.rs:27-87): same env names and validation errors."""
        self = cls()
        err = ctypes.create_string_buffer(256)
        rc = lib().gs_config_from_env(ctypes.byref(self.c), err, 256)
        if rc:
            raise GossipSimError(rc, err.value.decode())
        return self

    def __getattr__(self, k):
        if k == "c":
            raise AttributeError(k)
        return getattr(self.c, k)


class Simulator:
    """One context = one HIP device (include/gossipsim.h threading rules)."""

    def __init__(self, cfg=None, **kw):
        self.cfg = cfg if cfg is not None else PeerConfig(**kw)
        self.ctx = ctypes.c_void_p()
        rc = lib().gs_create(ctypes.byref(self.cfg.c), ctypes.byref(self.ctx))
        if rc:
            raise GossipSimError(rc, "gs_create failed")
        self.peers = self.cfg.c.peers
        self._sched = []

    # ---- checkpoint / resume (gs_save_state / gs_load_state) ----
    def save_state(self, path):
        """Links, CSR, mesh, churn mesh state, counters and traffic into `path`."""
        self._check(lib().gs_save_state(self.ctx, str(path).encode()))

    @classmethod
    def load_state(cls, path, device=0):
        """A new simulator on `device` that continues where the saved one stopped."""
        self = cls.__new__(cls)
        self.ctx = ctypes.c_void_p()
        rc = lib().gs_load_state(str(path).encode(), device, ctypes.byref(self.ctx))
        if rc:
            raise GossipSimError(rc, "gs_load_state(%s) failed" % path)
        self.cfg = PeerConfig()
        lib().gs_get_config(self.ctx, ctypes.byref(self.cfg.c))
        self.peers = self.cfg.c.peers
        self._sched = []
        return self

    def _check(self, rc):
        if rc:
            raise GossipSimError(rc, lib().gs_last_error(self.ctx).decode())

    def close(self):
        if self.ctx:
            lib().gs_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- links / topology / mesh ----
    def set_links(self, lat_ns, bw_up, bw_down=None, stage_of_peer=None):
        lat = np.ascontiguousarray(np.asarray(lat_ns, np.uint64).reshape(-1))
        S = int(round(len(lat) ** 0.5))
        up = np.ascontiguousarray(bw_up, np.uint64)
        dn = np.ascontiguousarray(bw_up if bw_down is None else bw_down, np.uint64)
        st = None if stage_of_peer is None else np.ascontiguousarray(stage_of_peer, np.uint8)
        self._check(lib().gs_set_links(self.ctx, S, _ptr(lat, u64), _ptr(up, u64), _ptr(dn, u64),
                                       None if st is None else _ptr(st, u8)))
        self._links = (lat, up, dn, st)

    def set_topogen_links(self, stages=1, min_bw=50, max_bw=50, min_lat=100, max_lat=100,
                          shortest=False):
        lat, bw = topogen_links(stages, min_bw, max_bw, min_lat, max_lat, shortest)
        self.set_links(lat, bw, bw)
        return lat, bw

    def set_shadow_links(self, gml_path, yaml_path, shortest=False):
        """Links straight from a Shadow experiment: the GML graph + shadow.yaml's host placement."""
        lat, up, dn = links_from_gml(gml_path, shortest)
        self.set_links(lat, up, dn, shadow_hosts(yaml_path, self.peers))
        return lat, up, dn

    def connect_gossipsub_peers(self):
        """main.rs:303-389: random ID dialing -> CSR (device resident)."""
        self._check(lib().gs_build_topology(self.ctx))

    build_topology = connect_gossipsub_peers

    def graph_info(self):
        n, nnz, md = u32(), u64(), u32()
        self._check(lib().gs_graph_info(self.ctx, ctypes.byref(n), ctypes.byref(nnz),
                                        ctypes.byref(md)))
        return n.value, nnz.value, md.value

    def csr(self):
        _, nnz, _ = self.graph_info()
        row = np.zeros(self.peers + 1, np.uint64)
        col = np.zeros(max(nnz, 1), np.uint32)
        flags = np.zeros(max(nnz, 1), np.uint8)
        self._check(lib().gs_get_csr(self.ctx, _ptr(row, u64), _ptr(col, u32), _ptr(flags, u8)))
        return row, col[:nnz], flags[:nnz]

    def mesh_converge(self, max_heartbeats=400):
        ep = u32()
        self._check(lib().gs_mesh_converge(self.ctx, max_heartbeats, ctypes.byref(ep)))
        return ep.value

    def mesh(self):
        m = np.zeros(self.peers * MESH_W, np.uint32)
        c = np.zeros(self.peers, np.uint8)
        self._check(lib().gs_get_mesh(self.ctx, _ptr(m, u32), _ptr(c, u8)))
        return m.reshape(self.peers, MESH_W), c

    # ---- publish / run ----
    def publish(self, publisher, msg_size, t_pub_ns):
        """POST /publish (main.rs:152-168): queue one injection."""
        if not 0 <= publisher < self.peers:
            raise GossipSimError(-1, "publisher out of range")
        self._sched.append((int(t_pub_ns), int(publisher), int(msg_size)))

    def _schedule(self, schedule):
        """(t, publisher, msg_size[, frags]) arrays or a GsPublish array -> GsPublish array."""
        if schedule is None:
            schedule = (GsPublish * len(self._sched))(*[GsPublish(*r) for r in self._sched])
            self._sched = []
        elif not isinstance(schedule, ctypes.Array):
            t, p, s = schedule[:3]
            fr = schedule[3] if len(schedule) > 3 else 0
            # one vectorised fill of the gs_publish layout (a per-element struct loop cost
            # ~0.7 ms per 1024 messages, most of a config #1 run)
            rec = np.zeros(len(t), np.dtype([("t_pub_ns", "<u8"), ("publisher", "<u4"), ("msg_size", "<u4"),
                                             ("frags", "<u4"), ("reserved", "<u4")]))
            assert rec.dtype.itemsize == ctypes.sizeof(GsPublish)
            rec["t_pub_ns"] = np.asarray(t, np.uint64)
            rec["publisher"] = np.asarray(p, np.uint32)
            rec["msg_size"] = np.asarray(s, np.uint32)
            rec["frags"] = np.asarray(fr, np.uint32)
            schedule = (GsPublish * len(t)).from_buffer_copy(rec.tobytes())
        return schedule

    def run(self, schedule=None, collect=True, summary=False, on_block=None, block_msgs=0,
            want=WANT_T_COMPLETE | WANT_HOPS, on_lat=None):
        """Simulate the queued publishes (or `schedule`); returns t_complete/hops [M, N].

        summary: also return the device's per-message latency reductions
        (gs_msg_summary: delivered, lat_sum_ms, p50/p95/max ms, 100 ms histogram).
        on_block(first_msg, t_complete[n, N], hops[n, N]): stream the results in
        blocks of `block_msgs` messages instead of returning [M, N] arrays;
        `want` (WANT_* bits) selects which of the two it receives (None if not).
        on_lat(first_msg, lat_ms[n, N] uint16): the logged latency stream
        (GS_WANT_LAT_MS: (t_complete - tx_time) // 1e6 as main.rs:93 logs it,
        LAT_NONE where nothing is logged), in the same blocks; it may be used
        alone or beside on_block."""
        schedule = self._schedule(schedule)
        M = len(schedule)
        res = {"schedule": schedule}
        sink = GsResultSink()
        keep = []
        if on_lat is not None:
            def _lcb(user, first, n, peers, lat):
                on_lat(int(first), np.ctypeslib.as_array(lat, (n, peers)))

            lcb = LAT_FN(_lcb)
            keep.append(lcb)
            sink.on_lat = lcb
            sink.block_msgs = block_msgs
            sink.want = WANT_LAT_MS | (want & (WANT_T_COMPLETE | WANT_HOPS) if on_block is not None else 0)
        if on_block is not None:
            N = self.peers

            def _cb(user, first, n, peers, tc, hp):
                a = np.ctypeslib.as_array(tc, (n, peers)) if tc else None
                h = np.ctypeslib.as_array(hp, (n, peers)) if hp else None
                on_block(int(first), a, h)

            cb = BLOCK_FN(_cb)
            keep.append(cb)
            sink.want = want | (WANT_LAT_MS if on_lat is not None else 0)
            sink.on_block = cb
            sink.block_msgs = block_msgs
        elif collect and on_lat is None:
            tc = np.zeros(M * self.peers, np.uint64)
            hops = np.zeros(M * self.peers, np.uint8)
            sink.t_complete_ns = _ptr(tc, u64)
            sink.hops = _ptr(hops, u8)
            res["t_complete"] = tc.reshape(M, self.peers)
            res["hops"] = hops.reshape(M, self.peers)
        if summary:
            sm = (GsMsgSummary * M)()
            sink.summary = ctypes.cast(sm, P(GsMsgSummary))
            keep.append(sm)
        use_sink = on_block is not None or on_lat is not None or collect or summary
        self._check(lib().gs_run(self.ctx, schedule, M, ctypes.byref(sink) if use_sink else None))
        if summary:
            res["summary"] = {
                "delivered": np.array([x.delivered for x in sm], np.uint64),
                "lat_sum_ms": np.array([x.lat_sum_ms for x in sm], np.uint64),
                "p50_ms": np.array([x.p50_ms for x in sm], np.uint32),
                "p95_ms": np.array([x.p95_ms for x in sm], np.uint32),
                "max_ms": np.array([x.max_ms for x in sm], np.uint32),
                "hist": np.array([list(x.hist) for x in sm], np.uint32).reshape(M, HIST_BINS)}
        return res

    def stats(self):
        st = GsStats()
        self._check(lib().gs_get_stats(self.ctx, ctypes.byref(st)))
        return {n: getattr(st, n) for n, _ in GsStats._fields_}

    def reset_stats(self):
        self._check(lib().gs_reset_stats(self.ctx))

    def set_timing(self, on=True):
        self._check(lib().gs_set_timing(self.ctx, 1 if on else 0))

    def set_traffic(self, on=True):
        """Per-peer send/receive counters of later runs (zeroed now)."""
        self._check(lib().gs_set_traffic(self.ctx, 1 if on else 0))

    def traffic(self):
        """-> uint64 [N, len(TRAFFIC_COLS)] in TRAFFIC_COLS order."""
        tr = np.zeros((self.peers, len(TRAFFIC_COLS)), np.uint64)
        self._check(lib().gs_get_traffic(self.ctx, _ptr(tr, u64)))
        return tr

    def write_node_metrics(self, path):
        """Every peer's Prometheus metrics (rust-test-node/src/metrics.rs names) after traffic runs."""
        write_node_metrics(self.cfg, path, self.csr()[0], self.mesh()[1], self.traffic())

    def open_log(self, path):
        """Streaming arrival log (gs_log_open); feed it with LogStream.write(schedule_rows, t_complete)."""
        return LogStream(self.cfg, path)

    def write_latency_log(self, path, res):
        """Arrival lines as `grep -rne 'milliseconds\\|BW' shadow.data/` prints them."""
        sched = res["schedule"]
        tc = np.ascontiguousarray(res["t_complete"], np.uint64)
        rc = lib().gs_write_node_log(ctypes.byref(self.cfg.c), path.encode(), sched, len(sched), _ptr(tc, u64))
        if rc:
            raise GossipSimError(rc, "gs_write_latency_log failed")

    # ---- peer-partitioned mode (include/gossipsim.h gs_part_*; driver in partition.py) ----
    def set_partition(self, parts, part):
        self._check(lib().gs_set_partition(self.ctx, parts, part))
        self.part_range = (part * self.peers // parts, (part + 1) * self.peers // parts)

    def part_begin(self, schedule):
        schedule = self._schedule(schedule)
        if not hasattr(self, "part_range"):
            self.part_range = (0, self.peers)
        k = u64()
        self._check(lib().gs_part_begin(self.ctx, schedule, len(schedule), ctypes.byref(k)))
        self._part_sched = schedule
        return k.value

    def part_scan(self, bucket_key, dev_ptr, capacity):
        """-> (ok, n, next_key): ok False means `capacity` < n records (state unchanged)."""
        n, m = u64(), u64()
        rc = lib().gs_part_scan(self.ctx, bucket_key, dev_ptr, capacity, ctypes.byref(n), ctypes.byref(m))
        if rc == GS_ERANGE and n.value > capacity:
            return False, n.value, m.value
        self._check(rc)
        return True, n.value, m.value

    def part_relax(self, bucket_key, dev_ptr, n):
        m = u64()
        self._check(lib().gs_part_relax(self.ctx, bucket_key, dev_ptr, n, ctypes.byref(m)))
        return m.value

    def part_finish(self, collect=True):
        """-> {"t_complete", "hops"} [M, own peers] (message-major over this part's peers)."""
        M = len(self._part_sched)
        u0, u1 = self.part_range
        res = {"schedule": self._part_sched, "peer_range": (u0, u1)}
        if collect:
            tc = np.zeros(M * (u1 - u0), np.uint64)
            hops = np.zeros(M * (u1 - u0), np.uint8)
            sink = GsResultSink(_ptr(tc, u64), _ptr(hops, u8))
            self._check(lib().gs_part_finish(self.ctx, ctypes.byref(sink)))
            res["t_complete"] = tc.reshape(M, u1 - u0)
            res["hops"] = hops.reshape(M, u1 - u0)
        else:
            self._check(lib().gs_part_finish(self.ctx, None))
        return res


class LogStream:
    """gs_log_*: the arrival log written block by block (message-major blocks
    from Simulator.run(on_block=...)), identical lines to write_latency_log."""

    def __init__(self, cfg, path):
        self.h = ctypes.c_void_p()
        rc = lib().gs_log_open(ctypes.byref(cfg.c), path.encode(), ctypes.byref(self.h))
        if rc:
            raise GossipSimError(rc, "gs_log_open %s" % path)

    def write(self, sched_rows, t_complete):
        """sched_rows: GsPublish array (or slice) of the block; t_complete [n, N] uint64."""
        tc = np.ascontiguousarray(t_complete, np.uint64)
        n = tc.shape[0]
        rows = (GsPublish * n)(*sched_rows[:n]) if not isinstance(sched_rows, ctypes.Array) else sched_rows
        rc = lib().gs_log_write(self.h, rows, n, _ptr(tc, u64))
        if rc:
            raise GossipSimError(rc, "gs_log_write failed")

    def write_lat(self, sched_rows, lat_ms):
        """The same lines from a block of the u16 latency stream (run(on_lat=...))."""
        lat = np.ascontiguousarray(lat_ms, np.uint16)
        n = lat.shape[0]
        rows = (GsPublish * n)(*sched_rows[:n]) if not isinstance(sched_rows, ctypes.Array) else sched_rows
        rc = lib().gs_log_write_lat(self.h, rows, n, _ptr(lat, ctypes.c_uint16))
        if rc:
            raise GossipSimError(rc, "gs_log_write_lat failed")

    def close(self):
        if self.h:
            rc = lib().gs_log_close(self.h)
            self.h = ctypes.c_void_p()
            if rc:
                raise GossipSimError(rc, "gs_log_close failed")


class Comm:
    """gs_comm: the parts of a peer-partitioned run (include/gossipsim.h).

    Comm(local_parts=P)                     P parts driven by this process
    Comm(nranks, rank, uid, device)         one rank of an RCCL communicator;
                                            uid = Comm.get_id() on rank 0,
                                            handed to the others out of band"""

    def __init__(self, nranks=1, rank=0, uid=None, device=0, local_parts=None, transport=None):
        self.h = ctypes.c_void_p()
        if transport is not None:  # the caller's collectives (gs_comm_init_ops)
            self._ops = _ops_of(transport, nranks)
            rc = lib().gs_comm_init_ops(nranks, rank, ctypes.byref(self._ops), device, ctypes.byref(self.h))
            self.parts, self.local, self.rank = nranks, False, rank
        elif local_parts is not None:
            rc = lib().gs_comm_init_local(local_parts, ctypes.byref(self.h))
            self.parts, self.local = local_parts, True
        else:
            if uid is None:
                uid = Comm.get_id()
            rc = lib().gs_comm_init(nranks, rank, uid, device, ctypes.byref(self.h))
            self.parts, self.local, self.rank = nranks, False, rank
        if rc:
            raise GossipSimError(rc, "gs_comm_init failed")

    def check(self):
        """gs_comm_check: one all-gather and one exchange of known bytes through the transport."""
        rc = lib().gs_comm_check(self.h)
        if rc:
            raise GossipSimError(rc, "gs_comm_check: the transport delivered wrong data")

    @staticmethod
    def get_id():
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        rc = lib().gs_comm_get_id(buf)
        if rc:
            raise GossipSimError(rc, "gs_comm_get_id failed (RCCL not loadable?)")
        return buf.raw

    def run_partitioned(self, sims, schedule, collect=True):
        """gs_run_partitioned over this process's Simulators (local: one per part,
        in part order; RCCL: this rank's). -> per part {"t_complete", "hops",
        "peer_range"} [M, own peers] (collect) or None."""
        schedule = sims[0]._schedule(schedule)
        M = len(schedule)
        arr = (ctypes.c_void_p * len(sims))(*[s.ctx for s in sims])
        sinks, keep, out = (GsResultSink * len(sims))(), [], []
        for i, sim in enumerate(sims):
            part = i if self.local else self.rank
            u0, u1 = part * sim.peers // self.parts, (part + 1) * sim.peers // self.parts
            sim.part_range = (u0, u1)
            if collect:
                tc = np.zeros(M * (u1 - u0), np.uint64)
                hp = np.zeros(M * (u1 - u0), np.uint8)
                keep += [tc, hp]
                sinks[i].t_complete_ns = _ptr(tc, u64)
                sinks[i].hops = _ptr(hp, u8)
                out.append({"t_complete": tc.reshape(M, u1 - u0), "hops": hp.reshape(M, u1 - u0),
                            "peer_range": (u0, u1)})
        rc = lib().gs_run_partitioned(arr, len(sims), self.h, schedule, M, sinks if collect else None)
        if rc:
            raise GossipSimError(rc, lib().gs_last_error(sims[0].ctx).decode())
        return out if collect else None

    def close(self):
        if self.h:
            lib().gs_comm_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ops_of(transport, nranks):
    """gs_comm_ops over a transport object with allgather(np.uint64[n]) -> [nranks, n]
    and exchange(list of send bytes, list of recv sizes) -> list of recv bytes.
    An exception in the transport becomes a non-zero return (the call fails)."""
    def allgather(_user, mine, n, out):
        try:
            a = np.ctypeslib.as_array(mine, (n,)).copy() if n else np.zeros(0, np.uint64)
            got = np.ascontiguousarray(transport.allgather(a), np.uint64).reshape(-1)
            if got.size != nranks * n:
                return 2
            ctypes.memmove(out, got.ctypes.data, got.nbytes)
            return 0
        except Exception:  # noqa: BLE001  (reported as the call's failure)
            import traceback
            traceback.print_exc()
            return 1

    def exchange(_user, send, send_bytes, recv, recv_bytes):
        try:
            sends = [ctypes.string_at(send[p], send_bytes[p]) if send_bytes[p] else b"" for p in range(nranks)]
            sizes = [int(recv_bytes[p]) for p in range(nranks)]
            got = transport.exchange(sends, sizes)
            for p in range(nranks):
                if len(got[p]) != sizes[p]:
                    return 2
                if sizes[p]:
                    ctypes.memmove(recv[p], bytes(got[p]), sizes[p])
            return 0
        except Exception:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            return 1

    ops = GsCommOps()
    ops._cb = (ALLGATHER_FN(allgather), EXCHANGE_FN(exchange))  # kept alive with the struct
    ops.allgather, ops.exchange = ops._cb
    return ops


class TorchDistTransport:
    """gs_comm_ops over torch.distributed (any backend with all_gather and
    point-to-point send / recv, e.g. gloo on CPU tensors): one rank per process,
    launched by torchrun or multiprocessing, the rendezvous the caller's."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)

    def allgather(self, mine):
        t = self.torch.from_numpy(mine.view(np.int64).copy())
        out = [self.torch.empty_like(t) for _ in range(self.size)]
        self.dist.all_gather(out, t, group=self.group)
        return np.stack([o.numpy().view(np.uint64) for o in out])

    def exchange(self, sends, sizes):
        torch, dist = self.torch, self.dist
        reqs, recvs = [], [b""] * self.size
        bufs = {}
        for p in range(self.size):
            if p == self.rank:
                continue
            if sizes[p]:
                bufs[p] = torch.empty(sizes[p], dtype=torch.uint8)
                reqs.append(dist.irecv(bufs[p], src=p, group=self.group))
            if len(sends[p]):
                reqs.append(dist.isend(torch.frombuffer(bytearray(sends[p]), dtype=torch.uint8), dst=p,
                                       group=self.group))
        for r in reqs:
            r.wait()
        for p, b in bufs.items():
            recvs[p] = b.numpy().tobytes()
        return recvs
