"""ctypes wrapper of the CPU oracle (oracle/gs_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker. The product path
(dst-libp2p-test-node_amd/) never imports this module.

Parity status: link tables pinned against shadow/topogen.py outputs and the
log format pinned against shadow/summary_latency*.awk (tests/golden/); the
gossipsub dissemination and mesh rules are a restatement of the
third-party libp2p-gossipsub 0.49.2 behaviour (not vendored, no reference
tests) — parity unpinned for those, see DESIGN.md §3.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "gs_oracle.c")
LIB = os.path.join(HERE, "_build", "libgs_oracle.so")
MESH_W = 16


class OrParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "peers", "connect_to", "dial_extra", "max_connections", "fragments",
        "muxer", "signed_msgs", "d", "d_lo", "d_hi", "d_lazy", "d_out",
        "gossip_factor_milli")] + [
        ("heartbeat_ns", ctypes.c_uint64), ("backoff_ns", ctypes.c_uint64)] + [
        (n, ctypes.c_uint32) for n in ("flood_publish", "idontwant", "lazy_gossip", "self_log")] + [
        ("seed", ctypes.c_uint64), ("history_gossip", ctypes.c_uint32), ("hb_phase_ns", ctypes.c_uint64)] + [
        (n, ctypes.c_uint32) for n in ("churn_ppm", "churn_down", "churn_horizon", "node", "sub_graft", "hs_rtts")]


class OrStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "messages", "deliveries", "frag_deliveries", "relaxations", "bytes_alg",
        "latency_sum_ms", "latency_max_ms", "gossip_iwant")]


def build(force=False):
    """Compile the oracle with gcc into oracle/_build (git-ignored)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", LIB, SRC])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        u32, u64, u8 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint8
        L.or_rng.restype = u64
        L.or_rng.argtypes = [u64, u32, u32, u32, u32]
        L.or_wire_bytes.restype = u64
        L.or_wire_bytes.argtypes = [u64, u32, u32]
        L.or_wire_packets.argtypes = [u64, u32, u32, P(u64), P(u64)]
        L.or_ctrl_packets.argtypes = [u32, u32, u32, P(u64), P(u64), P(u64)]
        L.or_run_traffic.argtypes = [P(OrParams), P(u64), P(u32), P(u32), P(u8), P(u8), u32, P(u64),
                                     P(u64), P(u64), P(u64), P(u32), P(u32), P(u32), u64, P(u64), P(u8),
                                     P(OrStats), P(u64)]
        L.or_topogen_links.argtypes = [u32, u32, u32, u32, u32, u32, P(u64), P(u64)]
        L.or_dials_per_peer.restype = u32
        L.or_dials_per_peer.argtypes = [P(OrParams)]
        L.or_build_topology.argtypes = [P(OrParams), P(u64), P(u32), P(u8), P(u64)]
        L.or_mesh_converge.argtypes = [P(OrParams), P(u64), P(u32), P(u8), P(u8), u32, P(u64),
                                       u32, P(u32), P(u8), P(u32)]
        L.or_run.argtypes = [P(OrParams), P(u64), P(u32), P(u32), P(u8), P(u8), u32, P(u64),
                             P(u64), P(u64), P(u64), P(u32), P(u32), P(u32), u64, P(u64), P(u8),
                             P(OrStats)]
        L.or_offline.argtypes = [P(OrParams), u32, u64]
        L.or_run_mt.argtypes = L.or_run.argtypes + [ctypes.c_int]
        L.or_mesh_churn.argtypes = [P(OrParams), P(u64), P(u32), P(u8), P(u8), u32, P(u64), u32, u32,
                                    P(u32), P(u8), P(u8)]
        L.or_mesh_churn_sel.argtypes = [P(OrParams), P(u64), P(u32), P(u8), P(u8), u32, P(u64), u32, P(u8),
                                        ctypes.c_int, P(u32), P(u8), P(u8)]
        L.or_run_churn.argtypes = [P(OrParams), P(u64), P(u32), P(u32), P(u8), P(u8), u32, u32, P(u8), u32,
                                   P(u64), P(u64), P(u64), P(u64), P(u32), P(u32), P(u32), u64, P(u64), P(u8),
                                   P(OrStats)]
        L.or_run_churn_traffic.argtypes = L.or_run_churn.argtypes + [P(u64)]
        _lib = L
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def params(**kw):
    """Rust preset defaults (rust-test-node/src/main.rs:36-38,223-241; env.rs:38-67)."""
    d = dict(peers=100, connect_to=10, dial_extra=1, max_connections=0, fragments=1,
             muxer=0, signed_msgs=1, d=6, d_lo=4, d_hi=8, d_lazy=6, d_out=3,
             gossip_factor_milli=250, heartbeat_ns=1_000_000_000, backoff_ns=60_000_000_000,
             flood_publish=1, idontwant=0, lazy_gossip=1, self_log=0, seed=1, history_gossip=3,
             hb_phase_ns=0, churn_ppm=0, churn_down=10, churn_horizon=16, node=0, sub_graft=1, hs_rtts=3)
    d.update(kw)
    return OrParams(**d)


def params_for(node, **kw):
    """The oracle's restatement of each test node's own settings:
    go-test-node/main.go:153-175,374-385 (Dout 2, IDONTWANT 1000 B, StrictNoSign,
    own publish delivered locally) and nim gossipsub-queues/main.nim:242-332,
    396, 429 (CONNECTTO dials, MAXCONNECTIONS 250, Dout = D div 2, Dlazy = D,
    anonymize, SELFTRIGGER)."""
    node = {"rust": 0, "go": 1, "nim": 2}.get(node, node)
    d = dict(node=node)
    if node == 1:
        d.update(d_out=2, idontwant=1000, signed_msgs=0, self_log=1, sub_graft=0)
    elif node == 2:
        D = kw.get("d", 6)
        d.update(dial_extra=0, max_connections=250, d_out=D // 2, d_lazy=D, signed_msgs=0, self_log=1,
                 sub_graft=0)
    d.update(kw)
    return params(**d)


def wire_bytes(payload, muxer=0, signed=1):
    return int(lib().or_wire_bytes(payload, muxer, signed))


def rng(seed, purpose, a, b, c):
    return int(lib().or_rng(seed, purpose, a, b, c))


def topogen_links(stages, bl, bh, ll, lh, mode=0):
    lat = np.zeros(stages * stages, np.uint64)
    bw = np.zeros(stages, np.uint64)
    rc = lib().or_topogen_links(stages, bl, bh, ll, lh, mode, _p(lat, ctypes.c_uint64),
                                _p(bw, ctypes.c_uint64))
    if rc:
        raise ValueError("or_topogen_links rc=%d" % rc)
    return lat.reshape(stages, stages), bw


def build_topology(p):
    N = p.peers
    k = lib().or_dials_per_peer(ctypes.byref(p))
    row_ptr = np.zeros(N + 1, np.uint64)
    col = np.zeros(max(1, 2 * k * N), np.uint32)
    flags = np.zeros(max(1, 2 * k * N), np.uint8)
    nnz = ctypes.c_uint64(0)
    rc = lib().or_build_topology(ctypes.byref(p), _p(row_ptr, ctypes.c_uint64),
                                 _p(col, ctypes.c_uint32), _p(flags, ctypes.c_uint8),
                                 ctypes.byref(nnz))
    if rc:
        raise ValueError("or_build_topology rc=%d" % rc)
    n = nnz.value
    return row_ptr, col[:n].copy(), flags[:n].copy()


def mesh_converge(p, row_ptr, col, flags, stage, lat, max_hb=400, allow_wide=False):
    """allow_wide: a mesh row wider than the ELL (possible before heartbeat 1
    prunes it) returns (flags, None, None, epochs) instead of raising."""
    N = p.peers
    S = lat.shape[0]
    flags = flags.copy()
    mesh = np.zeros(N * MESH_W, np.uint32)
    cnt = np.zeros(N, np.uint8)
    ep = ctypes.c_uint32(0)
    lat = np.ascontiguousarray(lat.reshape(-1), np.uint64)
    stage = np.ascontiguousarray(stage, np.uint8)
    rc = lib().or_mesh_converge(ctypes.byref(p), _p(row_ptr, ctypes.c_uint64),
                                _p(col, ctypes.c_uint32), _p(flags, ctypes.c_uint8),
                                _p(stage, ctypes.c_uint8), S, _p(lat, ctypes.c_uint64), max_hb,
                                _p(mesh, ctypes.c_uint32), _p(cnt, ctypes.c_uint8),
                                ctypes.byref(ep))
    if rc == -5 and allow_wide:
        return flags, None, None, ep.value
    if rc:
        raise ValueError("or_mesh_converge rc=%d" % rc)
    return flags, mesh.reshape(N, MESH_W), cnt, ep.value


def offline(p, u, h):
    return bool(lib().or_offline(ctypes.byref(p), u, h))


def epoch_at(p, t_abs):
    """Heartbeat epoch containing absolute time t (heartbeats at hb_phase + h*hb)."""
    t_abs = int(t_abs)
    return 0 if t_abs < p.hb_phase_ns else (t_abs - p.hb_phase_ns) // p.heartbeat_ns


def mesh_churn(p, row_ptr, col, flags, stage, lat, h_lo, h_hi):
    """Churn snapshots for epochs [h_lo, h_hi]: mesh [E, N, 16], cnt [E, N], offline [E, N]."""
    N, E = p.peers, h_hi - h_lo + 1
    S = lat.shape[0]
    mesh = np.zeros(E * N * MESH_W, np.uint32)
    cnt = np.zeros(E * N, np.uint8)
    off = np.zeros(E * N, np.uint8)
    lat = np.ascontiguousarray(lat.reshape(-1), np.uint64)
    stage = np.ascontiguousarray(stage, np.uint8)
    flags = np.ascontiguousarray(flags, np.uint8)
    rc = lib().or_mesh_churn(ctypes.byref(p), _p(row_ptr, ctypes.c_uint64), _p(col, ctypes.c_uint32),
                             _p(flags, ctypes.c_uint8), _p(stage, ctypes.c_uint8), S, _p(lat, ctypes.c_uint64),
                             h_lo, h_hi, _p(mesh, ctypes.c_uint32), _p(cnt, ctypes.c_uint8),
                             _p(off, ctypes.c_uint8))
    if rc:
        raise ValueError("or_mesh_churn rc=%d" % rc)
    return mesh.reshape(E, N, MESH_W), cnt.reshape(E, N), off.reshape(E, N)


def mesh_churn_ranges(p, row_ptr, col, flags, stage, lat, ranges, threads=0):
    """One churn replay from epoch 0 (or_mesh_churn_sel, OpenMP over peers when
    threads > 1), keeping only the epochs of `ranges` [(h_lo, h_hi), ...]:
    returns {(h_lo, h_hi): (mesh [E, N, 16], cnt [E, N], offline [E, N])}, the
    snapshot tuples mesh_churn would return for each range."""
    N = p.peers
    h_top = max(hi for _, hi in ranges)
    keep = np.zeros(h_top + 1, np.uint8)
    for lo, hi in ranges:
        keep[lo:hi + 1] = 1
    K = int(keep.sum())
    mesh = np.zeros(K * N * MESH_W, np.uint32)
    cnt = np.zeros(K * N, np.uint8)
    off = np.zeros(K * N, np.uint8)
    S = lat.shape[0]
    lat = np.ascontiguousarray(lat.reshape(-1), np.uint64)
    stage = np.ascontiguousarray(stage, np.uint8)
    flags = np.ascontiguousarray(flags, np.uint8)
    rc = lib().or_mesh_churn_sel(ctypes.byref(p), _p(row_ptr, ctypes.c_uint64), _p(col, ctypes.c_uint32),
                                 _p(flags, ctypes.c_uint8), _p(stage, ctypes.c_uint8), S, _p(lat, ctypes.c_uint64),
                                 h_top, _p(keep, ctypes.c_uint8), int(threads), _p(mesh, ctypes.c_uint32),
                                 _p(cnt, ctypes.c_uint8), _p(off, ctypes.c_uint8))
    if rc:
        raise ValueError("or_mesh_churn_sel rc=%d" % rc)
    slot = np.cumsum(keep) - 1  # epoch -> kept slot
    mesh, cnt, off = mesh.reshape(K, N, MESH_W), cnt.reshape(K, N), off.reshape(K, N)
    out = {}
    for lo, hi in ranges:
        a, b = int(slot[lo]), int(slot[hi]) + 1
        out[(lo, hi)] = (mesh[a:b], cnt[a:b], off[a:b])
    return out


def _frags_ptr(sched_frags, M):
    """Per-message chunk counts (0 = p.fragments) -> (array keeping it alive, pointer or None)."""
    if sched_frags is None:
        return None, None
    a = np.ascontiguousarray(np.broadcast_to(np.asarray(sched_frags, np.uint32), (M,)), np.uint32)
    return a, _p(a, ctypes.c_uint32)


def run_churn(p, row_ptr, col, snaps, h_lo, stage, lat, bw_up, bw_dn, sched_t, sched_pub, sched_size,
              sched_frags=None, traffic=None):
    """traffic: optional uint64 [N, TR_COLS] accumulated per-peer counters (or_run_churn_traffic)."""
    N = p.peers
    S = lat.shape[0]
    M = len(sched_t)
    smesh, scnt, soff = snaps
    tc = np.zeros(M * N, np.uint64)
    hops = np.zeros(M * N, np.uint8)
    st = OrStats()
    a64 = lambda x: np.ascontiguousarray(x, np.uint64)
    a32 = lambda x: np.ascontiguousarray(x, np.uint32)
    lat, bw_up, bw_dn, sched_t = a64(lat.reshape(-1)), a64(bw_up), a64(bw_dn), a64(sched_t)
    sched_pub, sched_size = a32(sched_pub), a32(sched_size)
    smesh, scnt, soff = a32(smesh.reshape(-1)), np.ascontiguousarray(scnt.reshape(-1), np.uint8), \
        np.ascontiguousarray(soff.reshape(-1), np.uint8)
    fa, fp = _frags_ptr(sched_frags, M)
    stage = np.ascontiguousarray(stage, np.uint8)
    args = (ctypes.byref(p), _p(row_ptr, ctypes.c_uint64), _p(col, ctypes.c_uint32),
            _p(smesh, ctypes.c_uint32), _p(scnt, ctypes.c_uint8), _p(soff, ctypes.c_uint8),
            h_lo, len(scnt) // N, _p(stage, ctypes.c_uint8), S, _p(lat, ctypes.c_uint64),
            _p(bw_up, ctypes.c_uint64), _p(bw_dn, ctypes.c_uint64), _p(sched_t, ctypes.c_uint64),
            _p(sched_pub, ctypes.c_uint32), _p(sched_size, ctypes.c_uint32), fp, M,
            _p(tc, ctypes.c_uint64), _p(hops, ctypes.c_uint8), ctypes.byref(st))
    if traffic is None:
        rc = lib().or_run_churn(*args)
    else:
        assert traffic.dtype == np.uint64 and traffic.shape == (N, TR_COLS) and traffic.flags.c_contiguous
        rc = lib().or_run_churn_traffic(*args, _p(traffic, ctypes.c_uint64))
    if rc:
        raise ValueError("or_run_churn rc=%d" % rc)
    stats = {n: getattr(st, n) for n, _ in OrStats._fields_}
    return tc.reshape(M, N), hops.reshape(M, N), stats


def wire_packets(payload, muxer=0, signed=1):
    pk, hd = ctypes.c_uint64(), ctypes.c_uint64()
    lib().or_wire_packets(payload, muxer, signed, ctypes.byref(pk), ctypes.byref(hd))
    return pk.value, hd.value


def ctrl_packets(kind, node=0, muxer=0):
    """(bytes, packets, header bytes) of one IHAVE (kind 0) / IWANT (1) RPC or one ACK (2)."""
    b, pk, hd = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib().or_ctrl_packets(kind, node, muxer, ctypes.byref(b), ctypes.byref(pk), ctypes.byref(hd))
    return b.value, pk.value, hd.value


# per-peer traffic columns (gossipsim.h GS_TR_*)
TR_COLS = 12


def run(p, row_ptr, col, mesh, cnt, stage, lat, bw_up, bw_dn, sched_t, sched_pub, sched_size, sched_frags=None,
        traffic=None, threads=0):
    """traffic: optional uint64 [N, TR_COLS] accumulated per-peer counters (or_run_traffic);
    sched_frags: chunks per message (0 = p.fragments); threads > 0: messages in
    parallel on that many host threads (or_run_mt)."""
    N = p.peers
    S = lat.shape[0]
    M = len(sched_t)
    tc = np.zeros(M * N, np.uint64)
    hops = np.zeros(M * N, np.uint8)
    st = OrStats()
    a64 = lambda x: np.ascontiguousarray(x, np.uint64)
    a32 = lambda x: np.ascontiguousarray(x, np.uint32)
    lat, bw_up, bw_dn, sched_t = a64(lat.reshape(-1)), a64(bw_up), a64(bw_dn), a64(sched_t)
    sched_pub, sched_size = a32(sched_pub), a32(sched_size)
    mesh = a32(mesh.reshape(-1))
    stage = np.ascontiguousarray(stage, np.uint8)
    fa, fp = _frags_ptr(sched_frags, M)
    args = (ctypes.byref(p), _p(row_ptr, ctypes.c_uint64), _p(col, ctypes.c_uint32),
            _p(mesh, ctypes.c_uint32), _p(cnt, ctypes.c_uint8), _p(stage, ctypes.c_uint8),
            S, _p(lat, ctypes.c_uint64), _p(bw_up, ctypes.c_uint64),
            _p(bw_dn, ctypes.c_uint64), _p(sched_t, ctypes.c_uint64),
            _p(sched_pub, ctypes.c_uint32), _p(sched_size, ctypes.c_uint32), fp, M,
            _p(tc, ctypes.c_uint64), _p(hops, ctypes.c_uint8), ctypes.byref(st))
    if threads:
        rc = lib().or_run_mt(*args, int(threads))
    elif traffic is None:
        rc = lib().or_run(*args)
    else:
        assert traffic.dtype == np.uint64 and traffic.shape == (N, TR_COLS) and traffic.flags.c_contiguous
        rc = lib().or_run_traffic(*args, _p(traffic, ctypes.c_uint64))
    if rc:
        raise ValueError("or_run rc=%d" % rc)
    stats = {n: getattr(st, n) for n, _ in OrStats._fields_}
    return tc.reshape(M, N), hops.reshape(M, N), stats


def simulate(p, stages=1, links=(50, 50, 50, 50), mode=0, sched=None, max_hb=400, traffic=False):
    """Whole pipeline on the CPU: links -> topology -> mesh -> run (+ per-peer traffic [N, TR_COLS])."""
    bl, bh, ll, lh = links
    lat, bw = topogen_links(stages, bl, bh, ll, lh, mode)
    stage = (np.arange(p.peers) % stages).astype(np.uint8)
    row_ptr, col, flags0 = build_topology(p)
    flags, mesh, cnt, epochs = mesh_converge(p, row_ptr, col, flags0, stage, lat, max_hb)
    t, pub, size = sched[:3]
    frags = sched[3] if len(sched) > 3 else None
    out = dict(lat=lat, bw=bw, stage=stage, row_ptr=row_ptr, col=col, flags=flags, mesh=mesh,
               cnt=cnt, epochs=epochs)
    tr = np.zeros((p.peers, TR_COLS), np.uint64) if traffic else None
    if p.churn_ppm:  # time-varying mesh: snapshots of every epoch the schedule can use
        h_lo = min(epoch_at(p, x) for x in t)
        h_hi = max(epoch_at(p, x) for x in t) + p.churn_horizon
        snaps = mesh_churn(p, row_ptr, col, flags0, stage, lat, h_lo, h_hi)
        tc, hops, stats = run_churn(p, row_ptr, col, snaps, h_lo, stage, lat, bw, bw, t, pub, size, frags,
                                    traffic=tr)
        out.update(snaps=snaps, h_lo=h_lo)
    else:
        tc, hops, stats = run(p, row_ptr, col, mesh, cnt, stage, lat, bw, bw, t, pub, size, frags, traffic=tr)
    if traffic:
        out["traffic"] = tr
    out.update(t_complete=tc, hops=hops, stats=stats)
    return out
