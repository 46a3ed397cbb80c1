"""CPU tests of the oracle (oracle/gs_oracle.c) against the reference's own
artefacts (topogen.py outputs, committed as tests/golden/topogen_*.json) and a
pure-Python restatement of the dissemination rules for small cases."""
import glob
import heapq
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T0 = 946684800_000_000_000 + 500_000_000_000  # Shadow epoch + injector start (topogen.py:130)


def _topogen_args(flags):
    d = {"-n": 100, "-bl": 50, "-bh": 50, "-ll": 100, "-lh": 100, "-st": 1}  # topogen.py:15-20
    for i in range(0, len(flags), 2):
        if flags[i] in d:
            d[flags[i]] = int(flags[i + 1])
    return d


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "topogen_*.json"))))
def test_links_match_topogen_gml(path):
    fx = json.load(open(path))
    a = _topogen_args(fx["flags"])
    S = a["-st"]
    lat, bw = oracle.topogen_links(S, a["-bl"], a["-bh"], a["-ll"], a["-lh"], mode=0)
    for i in range(S):
        up, dn = fx["nodes"][str(i)]
        assert bw[i] == up * 1_000_000 == dn * 1_000_000
    assert fx["nodes"][str(S)] == [100, 100]  # injector node (topogen.py:65)
    seen = 0
    for s, t, l, loss in fx["edges"]:
        assert loss == 0.0
        if s < S and t < S:
            assert lat[s, t] == lat[t, s] == l * 1_000_000
            seen += 1
        else:
            assert l == 1  # injector hub edges (topogen.py:66-69)
    assert seen == S * (S + 1) // 2
    # host -> stage (topogen.py:121-122) and the controller on the hub node
    assert fx["host_stage"] == [i % S for i in range(a["-n"])]
    assert fx["controller"] == S


def test_shortest_path_mode_uses_injector_hub():
    lat, _ = oracle.topogen_links(5, 50, 150, 40, 130, mode=1)
    assert (lat == 2_000_000).all()  # every pair is 1 ms + 1 ms through the hub


def test_wire_bytes_known_answers():
    # signed RPC: from(40) + data(1+2+15000) + seqno(10) + topic(6) + sig(66) = 15125;
    # RPC field 1+2+15125 = 15128; length prefix 2 -> frame 15130; yamux +12 -> 15142;
    # noise +18 -> 15160; TCP/IP 11 segments x 40 -> 15600
    assert oracle.wire_bytes(15000, 0, 1) == 15600
    # fragment of config #2: 1875 B payload
    frame = 1875 + 2 + 1 + 40 + 10 + 6 + 66  # data field + other fields
    frame = 1 + 2 + frame  # RPC publish field
    frame = 2 + frame  # length prefix
    assert oracle.wire_bytes(1875, 0, 1) == frame + 12 + 18 + 2 * 40
    # QUIC: 65 B per 1415 B packet
    assert oracle.wire_bytes(15000, 1, 1) == 15130 + 11 * 65
    # unsigned (nim anonymize): data + topic only
    assert oracle.wire_bytes(100, 0, 0) == (1 + 1 + (1 + 1 + 100) + 6) + 1 + 12 + 18 + 40


@pytest.mark.parametrize("name", ["uniform_n300", "hetero_n400_f4", "nim_n200_cap"])
def test_oracle_regression_fixture(name):
    """The oracle still reproduces its committed outputs bit for bit."""
    meta = json.load(open(os.path.join(GOLDEN, "oracle_%s.json" % name)))
    fx = np.load(os.path.join(GOLDEN, "oracle_%s.npz" % name))
    p = oracle.params(**meta["params"])
    r = oracle.simulate(p, meta["stages"], tuple(meta["links"]),
                        sched=(fx["sched_t"], fx["sched_pub"], np.full(meta["n_msgs"], meta["msg_size"])))
    for k in ("row_ptr", "col", "flags", "mesh", "cnt", "t_complete", "hops"):
        np.testing.assert_array_equal(r[k], fx[k], err_msg=k)
    assert r["stats"] == meta["stats"]
    assert r["epochs"] == meta["epochs"]


def _sim(N=300, seed=7, S=3, links=(30, 90, 20, 80), **kw):
    p = oracle.params(peers=N, seed=seed, **kw)
    M = 4
    t = T0 + np.arange(M, dtype=np.uint64) * 1_000_000_000
    pub = (np.arange(M) * 37 + 5) % N
    return p, oracle.simulate(p, S, links, sched=(t, pub, np.full(M, 15000))), (t, pub)


def test_topology_invariants():
    p, r, _ = _sim(N=500, max_connections=0)
    row, col, flags = r["row_ptr"].astype(np.int64), r["col"], r["flags"]
    N = p.peers
    k = oracle.lib().or_dials_per_peer(p)
    assert k == 11  # CONNECTTO + 1 (main.rs:337, defect D4)
    edges = set()
    for u in range(N):
        c = col[row[u]:row[u + 1]]
        assert (np.diff(c.astype(np.int64)) > 0).all() and u not in c
        assert (flags[row[u]:row[u + 1]] & 1).sum() == k  # u dialed exactly k peers
        edges.update((u, int(w)) for w in c)
    assert all((w, u) in edges for (u, w) in edges)


def test_mesh_invariants():
    p, r, _ = _sim(N=600)
    row, col, flags, mesh, cnt = r["row_ptr"].astype(np.int64), r["col"], r["flags"], r["mesh"], r["cnt"]
    N = p.peers
    ms = [set(int(x) for x in mesh[u, :cnt[u]]) for u in range(N)]
    for u in range(N):
        nb = set(int(w) for w in col[row[u]:row[u + 1]])
        assert ms[u] <= nb
        assert p.d_lo <= len(ms[u]) <= p.d_hi
        for w in ms[u]:
            assert u in ms[w]  # GRAFT/PRUNE keep the mesh symmetric
        in_mesh = set(int(col[e]) for e in range(row[u], row[u + 1]) if flags[e] & 2)
        assert in_mesh == ms[u]
    assert r["epochs"] < 400


def _py_subscription_epoch(p, row, col, out, stage, lat):
    """Pure-Python restatement of the subscription epoch 0 (DESIGN.md §2.3;
    libp2p-gossipsub handle_received_subscriptions / handle_graft, upstream,
    reached through the 20 s pump of rust-test-node/src/main.rs:357-379): every
    peer grafts its first D_lo connections in subscription-arrival order
    (3 rtt + lat(w->u), id); receivers take the GRAFTs in arrival order
    (4 rtt, id) and refuse beyond D_hi unless they dialed the grafter."""
    N, HS = p.peers, 3
    rtt = lambda a, b: int(lat[a, b]) + int(lat[b, a])
    nb = [[int(w) for w in col[row[u]:row[u + 1]]] for u in range(N)]
    prop = [set() for _ in range(N)]
    for u in range(N):
        order = sorted(nb[u], key=lambda w: (HS * rtt(stage[u], stage[w]) + int(lat[stage[w], stage[u]]), w))
        prop[u] = set(order[:p.d_lo])
    mesh = [set() for _ in range(N)]
    accepted = set()
    for w in range(N):
        c = len(prop[w])
        for u in sorted((u for u in nb[w] if w in prop[u]), key=lambda u: ((HS + 1) * rtt(stage[u], stage[w]), u)):
            if u in prop[w]:
                accepted.add((u, w))
                continue
            if c >= p.d_hi and (w, u) not in out:
                continue
            accepted.add((u, w))
            mesh[w].add(u)
            c += 1
    for u in range(N):
        for w in prop[u]:
            if (u, w) in accepted:
                mesh[u].add(w)
    return mesh


@pytest.mark.parametrize("S,links", [(5, (50, 150, 40, 130)), (3, (30, 90, 20, 80)), (5, (20, 200, 10, 90))])
def test_subscription_epoch_is_handshake_ordered(S, links):
    """A5 (i): the mesh before heartbeat 1 equals the pure-Python restatement,
    is symmetric, and is latency-ordered on heterogeneous links: its links are
    markedly shorter than the connections they were chosen from. (GRAFTs from
    peers a receiver dialed are always accepted, so a popular low-latency peer
    can hold more than GS_MESH_W links before heartbeat 1 prunes it to D: the
    mesh is read from the CSR flags.)"""
    p = oracle.params(peers=400, seed=13)
    lat, _ = oracle.topogen_links(S, *links)
    stage = (np.arange(p.peers) % S).astype(np.uint8)
    row, col, flags0 = oracle.build_topology(p)
    row = row.astype(np.int64)
    flags, _, _, ep = oracle.mesh_converge(p, row.astype(np.uint64), col, flags0, stage, lat, max_hb=0,
                                           allow_wide=True)
    assert ep == 0
    out = set((u, int(col[e])) for u in range(p.peers) for e in range(row[u], row[u + 1]) if flags0[e] & 1)
    ref = _py_subscription_epoch(p, row, col, out, stage, lat)
    got = [set(int(col[e]) for e in range(row[u], row[u + 1]) if flags[e] & 2) for u in range(p.peers)]
    assert got == ref
    assert all(u in got[w] for u in range(p.peers) for w in got[u])
    lat_mesh = np.mean([lat[stage[u], stage[w]] for u in range(p.peers) for w in got[u]])
    lat_conn = np.mean([lat[stage[u], stage[col[e]]] for u in range(p.peers) for e in range(row[u], row[u + 1])])
    assert lat_mesh < 0.9 * lat_conn
    # without it (go / nim presets) the mesh before heartbeat 1 is empty
    p0 = oracle.params(peers=400, seed=13, sub_graft=0)
    _, _, cnt0, _ = oracle.mesh_converge(p0, row.astype(np.uint64), col, flags0, stage, lat, max_hb=0)
    assert not cnt0.any()
    # heartbeat 1 prunes every row back under D_hi (the converged mesh fits the ELL)
    _, mesh1, cnt1, _ = oracle.mesh_converge(p, row.astype(np.uint64), col, flags0, stage, lat, max_hb=400)
    assert cnt1.max() <= p.d_hi


def _py_gossip_targets(p, r, v, h, ch=None):
    row, col = r["row_ptr"].astype(np.int64), r["col"]
    mesh, cnt = (r["mesh"], r["cnt"]) if ch is None else ch.snap(h)
    ms = set(int(x) for x in mesh[v, :cnt[v]])
    cand = sorted((oracle.rng(p.seed, 6, v, h & 0xFFFFFFFF, int(w)), int(w))
                  for w in col[row[v]:row[v + 1]] if int(w) not in ms and not (ch and ch.off(h, int(w))))
    rr = max(p.d_lazy, len(cand) * p.gossip_factor_milli // 1000)
    return [w for _, w in cand[:min(rr, len(cand))]]


class _Churn:
    """Epoch lookups over the oracle's snapshots for one message."""

    def __init__(self, p, r, t_pub):
        self.p, self.mesh, self.cnt, self.offl = p, *r["snaps"]
        self.h_lo = r["h_lo"]
        self.cap = self.epoch(t_pub) + p.churn_horizon

    def epoch(self, tabs):
        return 0 if tabs < self.p.hb_phase_ns else (tabs - self.p.hb_phase_ns) // self.p.heartbeat_ns

    def dead(self, h):
        return h > self.cap

    def snap(self, h):
        return self.mesh[h - self.h_lo], self.cnt[h - self.h_lo]

    def off(self, h, u):
        return bool(self.offl[h - self.h_lo, u])

    def lost(self, tabs, w):  # delivery at absolute time tabs
        h = self.epoch(tabs)
        return self.dead(h) or self.off(h, w)


def _py_disseminate(p, r, t_pub, pub, size):
    """Pure-Python event simulation of DESIGN.md §2.5-2.8 (small N only)."""
    N, F = p.peers, p.fragments
    row, col = r["row_ptr"].astype(np.int64), r["col"]
    mesh, cnt, stage, lat, bw = r["mesh"], r["cnt"], r["stage"], r["lat"], r["bw"]
    ch = _Churn(p, r, t_pub) if p.churn_ppm else None
    if ch and ch.off(ch.epoch(t_pub), pub):  # an offline publisher publishes nothing
        return np.full(N, np.iinfo(np.uint64).max, np.uint64), np.full(N, 255, np.uint8), 0
    payload = size // F
    wire = oracle.wire_bytes(payload, p.muxer, p.signed_msgs)
    ser = [(-(-wire * 8_000_000_000 // int(b))) for b in bw]
    best = {}
    busy = [0] * N
    heap = []  # (time, type, key, dst, frag): arrivals (0) before IHAVEs (1) at equal time
    iwant = [0]

    def gossip(v, f, tv, hv):
        tabs = t_pub + tv
        h0 = 0 if tabs <= p.hb_phase_ns else -(-(tabs - p.hb_phase_ns) // p.heartbeat_ns)
        sv = stage[v]
        for k in range(p.history_gossip):
            T = p.hb_phase_ns + (h0 + k) * p.heartbeat_ns - t_pub
            if ch and (ch.dead(h0 + k) or ch.off(h0 + k, v)):
                continue
            for w in _py_gossip_targets(p, r, v, h0 + k, ch):
                sw = stage[w]
                ti = T + int(lat[sv, sw])
                A = ti + int(lat[sw, sv]) + ser[sv] + int(lat[sv, sw]) + max(0, ser[sw] - ser[sv])
                if ch and (ch.lost(t_pub + ti, w) or ch.lost(t_pub + A, w)):
                    continue
                heapq.heappush(heap, (ti, 1, (A, hv + 1, v), w, f))

    for f in range(F):
        best[(pub, f)] = (0, 0, pub)
        if p.lazy_gossip:
            gossip(pub, f, 0, 0)
    tg = [int(x) for x in col[row[pub]:row[pub + 1]] if not (ch and ch.off(ch.epoch(t_pub), int(x)))]
    sp = stage[pub]
    for f in range(F):
        for j, w in enumerate(tg):
            arr = (f * len(tg) + j + 1) * ser[sp] + int(lat[sp, stage[w]]) + max(0, ser[stage[w]] - ser[sp])
            if ch and ch.lost(t_pub + arr, w):
                continue
            k = (arr, 1, pub)
            if k < best.get((w, f), (1 << 80,)):
                best[(w, f)] = k
                heapq.heappush(heap, (arr, 0, k, w, f))
    done = set([(pub, f) for f in range(F)])
    while heap:
        _, typ, k, u, f = heapq.heappop(heap)
        if typ == 1:
            if (u, f) in done:
                continue
            iwant[0] += 1
            if k < best.get((u, f), (1 << 80,)):
                best[(u, f)] = k
                heapq.heappush(heap, (k[0], 0, k, u, f))
            continue
        if (u, f) in done or best[(u, f)] != k:
            continue
        done.add((u, f))
        t, h, src = k
        su = stage[u]
        mrow, mcnt = mesh, cnt
        if ch:
            if ch.dead(ch.epoch(t_pub + t)):
                continue  # received past the message's lifetime: not forwarded
            mrow, mcnt = ch.snap(ch.epoch(t_pub + t))
        if p.lazy_gossip:
            gossip(u, f, t, h)
        targets = [int(w) for w in mrow[u, :mcnt[u]] if w != src and w != pub]
        start = max(t, busy[u]) if F > 1 else t
        busy[u] = start + len(targets) * ser[su]
        for j, w in enumerate(targets):
            arr = start + (j + 1) * ser[su] + int(lat[su, stage[w]]) + max(0, ser[stage[w]] - ser[su])
            if ch and ch.lost(t_pub + arr, w):
                continue
            nk = (arr, h + 1, u)
            if nk < best.get((w, f), (1 << 80,)):
                best[(w, f)] = nk
                heapq.heappush(heap, (arr, 0, nk, w, f))
    tc = np.full(N, np.iinfo(np.uint64).max, np.uint64)
    hops = np.full(N, 255, np.uint8)
    for u in range(N):
        if u == pub:
            tc[u], hops[u] = t_pub, 0
            continue
        ks = [best.get((u, f)) for f in range(F)]
        if any(x is None for x in ks):
            continue
        mk = max(ks)
        tc[u] = t_pub + mk[0]
        hops[u] = mk[1]
    return tc, hops, iwant[0]


@pytest.mark.parametrize("frags,gossip,churn", [(1, 0, 0), (3, 0, 0), (1, 1, 0), (2, 1, 0), (1, 0, 1), (2, 1, 1)])
def test_oracle_matches_pure_python_restatement(frags, gossip, churn):
    # slow links + a heartbeat phase inside the dissemination window so IWANTs happen
    kw = dict(lazy_gossip=gossip, hb_phase_ns=37_000_000, heartbeat_ns=100_000_000) if gossip else {}
    if churn:  # 3 % departures per 100 ms heartbeat, 8-heartbeat outages, heartbeats from T0 - 2 s
        kw.update(churn_ppm=30000, churn_down=8, churn_horizon=12, heartbeat_ns=100_000_000,
                  hb_phase_ns=T0 - 2_000_000_000 + 37_000_000)
    p, r, (t, pub) = _sim(N=150, fragments=frags, links=(5, 20, 20, 80), **kw)
    iw = 0
    for m in range(len(t)):
        tc, hops, nw = _py_disseminate(p, r, int(t[m]), int(pub[m]), 15000)
        iw += nw
        np.testing.assert_array_equal(r["t_complete"][m], tc)
        np.testing.assert_array_equal(r["hops"][m], hops)
    assert r["stats"]["gossip_iwant"] == iw
    if gossip:
        assert iw > 0


def test_fragment_collision_defect_d8():
    # payload 10 B with 4 fragments: fragments identical -> dedup -> never complete
    p = oracle.params(peers=60, fragments=4)
    r = oracle.simulate(p, 1, (50, 50, 50, 50), sched=(np.array([T0], np.uint64), np.array([3]), np.array([40])))
    assert r["stats"]["deliveries"] == 0
    assert r["stats"]["frag_deliveries"] == 59  # fragment 0 still spreads
    with pytest.raises(ValueError):  # payload < 8 B: main.rs:110 would panic
        oracle.simulate(p, 1, (50, 50, 50, 50), sched=(np.array([T0], np.uint64), np.array([3]), np.array([28])))


@pytest.mark.parametrize("node,bad,good", [("rust", 28, 40), ("go", 8, 12), ("nim", 64, 68)])
def test_fragment_layout_per_node(node, bad, good):
    """F=4: rust rejects payloads under 8 B and merges fragments of <= 10 B
    (D8); go's 8-byte stamp + msg_size/F layout fails only below 3 B of body
    (payload[10], main.go:70-74); nim's 16-byte header needs msg_size/F >= 17
    (nowBytes[16], main.nim:165-175). Layouts that accept a size never merge."""
    p = oracle.params_for(node, peers=60, fragments=4)
    one = lambda size: oracle.simulate(p, 1, (50, 50, 50, 50),
                                       sched=(np.array([T0], np.uint64), np.array([3]), np.array([size])))
    with pytest.raises(ValueError):
        one(bad)
    r = one(good)
    assert r["stats"]["deliveries"] == (0 if node == "rust" else 59)  # the publisher is not counted
    assert r["stats"]["frag_deliveries"] == (59 if node == "rust" else 4 * 59)


@pytest.mark.parametrize("kw", [dict(), dict(fragments=3), dict(flood_publish=0), dict(idontwant=1000)])
def test_traffic_identities(kw):
    """Eager forwarding only: every send is one relaxation and, without churn,
    one receipt: sum(tx) = sum(rx) = R x wire bytes; a non-publisher's sends
    = its forwards; every receipt of k packets returns ceil(k/2) ACKs."""
    p = oracle.params(peers=300, seed=7, lazy_gossip=0, **kw)
    t = np.uint64(T0) + np.arange(4, dtype=np.uint64) * np.uint64(10 ** 9)
    r = oracle.simulate(p, 5, (50, 150, 40, 130), sched=(t, np.array([3, 50, 120, 299]), np.full(4, 15000)),
                        traffic=True)
    tr, st = r["traffic"], r["stats"]
    W = oracle.wire_bytes(15000 // p.fragments, p.muxer, p.signed_msgs)
    pk, hd = oracle.wire_packets(15000 // p.fragments, p.muxer, p.signed_msgs)
    assert tr[:, 0].sum() == tr[:, 1].sum() == st["relaxations"] * W
    assert tr[:, 2].sum() == st["relaxations"] * pk and tr[:, 4].sum() == st["relaxations"] * hd
    assert (tr[:, 0] % W == 0).all() and (tr[:, 1] >= W).all()  # everyone receives at least once
    assert tr[:, 6].sum() == st["deliveries"] and tr[:, 7].sum() == st["messages"] == 4
    got = (r["t_complete"] != np.iinfo(np.uint64).max).sum(axis=0) - np.bincount([3, 50, 120, 299], minlength=300)
    np.testing.assert_array_equal(tr[:, 6], got)
    ack = oracle.ctrl_packets(2, p.node, p.muxer)[0]
    np.testing.assert_array_equal(tr[:, 8], tr[:, 3] // pk * ((pk + 1) // 2))  # ACKs sent per packets received
    assert tr[:, 8].sum() == tr[:, 9].sum() and (tr[:, 10] == tr[:, 8] * ack).all() and (tr[:, 11] == tr[:, 9] * ack).all()
    np.testing.assert_array_equal(tr[:, 9], tr[:, 2] // pk * ((pk + 1) // 2))  # ACKs back per send


def test_control_rpc_sizes():
    """IHAVE / IWANT RPCs with one 20-byte (rust / nim) or 32-byte (go) id:
    protobuf sizes + yamux 12 + noise 18 + one TCP/IPv4 header (QUIC 65)."""
    ih = 1 + 1 + (1 + 1 + (1 + 1 + 4) + (1 + 1 + 20))  # RPC.control{ihave{topic, id}}
    iw = 1 + 1 + (1 + 1 + (1 + 1 + 20))              # RPC.control{iwant{id}}
    assert oracle.ctrl_packets(0, 0, 0) == (1 + ih + 12 + 18 + 40, 1, 40)
    assert oracle.ctrl_packets(1, 0, 0) == (1 + iw + 12 + 18 + 40, 1, 40)
    assert oracle.ctrl_packets(1, 1, 0)[0] == oracle.ctrl_packets(1, 0, 0)[0] + 12
    assert oracle.ctrl_packets(0, 0, 1) == (1 + ih + 65, 1, 65)
    assert oracle.ctrl_packets(2, 0, 0) == (40, 1, 40) and oracle.ctrl_packets(2, 2, 1) == (65, 1, 65)


@pytest.mark.parametrize("case", ["noop", "iwant", "churn"])
def test_traffic_with_gossip_and_churn(case):
    """Lazy gossip adds IHAVE RPCs (every target, every history heartbeat) and,
    for targets that had not seen the message, IWANT RPCs + answers; churn
    loses sends (counted at the sender only) and their ACKs."""
    kw = dict(peers=400, seed=17, hb_phase_ns=T0 % 1_000_000_000)  # heartbeat at the publish instant
    if case == "noop":  # first gossip heartbeat 2.997 s after every publish: all IHAVEs land late
        kw.update(heartbeat_ns=3_000_000_000, hb_phase_ns=T0 - 3_000_000)
    if case == "churn":
        kw.update(churn_ppm=30000, hb_phase_ns=T0 - 4_000_000_000, heartbeat_ns=200_000_000, churn_horizon=8)
    p = oracle.params(**kw)
    t = np.uint64(T0) + np.arange(5, dtype=np.uint64) * np.uint64(3 * 10 ** 9)
    sched = (t, np.array([3, 50, 120, 299, 7]), np.full(5, 15000))
    r = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched, traffic=True)
    tr, st = r["traffic"].astype(np.int64), r["stats"]
    W = oracle.wire_bytes(15000, 0, 1)
    ihw = oracle.ctrl_packets(0)[0]
    iww = oracle.ctrl_packets(1)[0]
    ack = oracle.ctrl_packets(2)[0]
    # tx = R x W (eager sends + IWANT answers) + IHAVEs + IWANTs; R counts only answers that arrive
    extra = tr[:, 0].sum() - st["relaxations"] * W - st["gossip_iwant"] * iww
    if case == "noop":
        assert st["gossip_iwant"] == 0 and extra > 0 and extra % ihw == 0
        e = oracle.simulate(oracle.params(lazy_gossip=0, **kw), 5, (50, 150, 40, 130), sched=sched, traffic=True)
        d = tr - e["traffic"].astype(np.int64)  # gossip adds IHAVE traffic and nothing else
        assert (d[:, 0] % ihw == 0).all() and (d[:, 6:8] == 0).all() and d[:, 0].sum() == d[:, 1].sum()
    if case == "iwant":
        assert st["gossip_iwant"] > 0 and extra > 0 and extra % ihw == 0
    if case == "churn":
        assert tr[:, 0].sum() > tr[:, 1].sum()  # lost sends: tx without rx
    else:
        assert tr[:, 0].sum() == tr[:, 1].sum() and tr[:, 2].sum() == tr[:, 3].sum()
    assert tr[:, 8].sum() == tr[:, 9].sum() and (tr[:, 10] == tr[:, 8] * ack).all()
    assert tr[:, 6].sum() == st["deliveries"]


def test_stats_identities():
    p, r, _ = _sim(N=400, fragments=2)
    st = r["stats"]
    assert st["bytes_alg"] == 16 * st["frag_deliveries"] + 12 * st["relaxations"] + 8 * st["deliveries"]
    delivered = (r["t_complete"] != np.iinfo(np.uint64).max).sum() - st["messages"]
    assert st["deliveries"] == delivered
    assert st["frag_deliveries"] == st["deliveries"] * 2


def _py_offline(p, u, h):
    """a departure drawn at one of the epochs h-down+1..h."""
    return h > 0 and any((oracle.rng(p.seed, 7, u, h - k, 0) * 1_000_000) >> 64 < p.churn_ppm
                         for k in range(min(p.churn_down, h)))


def test_churn_snapshots_invariants():
    """Churn (config #3 semantics): the offline draw, empty rows for offline
    peers, no offline peer in any row, a symmetric mesh in every epoch, the
    expected offline fraction, and offline publishers publishing nothing."""
    ph = T0 - 3_000_000_000
    p, r, (t, pub) = _sim(N=400, seed=9, churn_ppm=20000, churn_down=10, churn_horizon=6,
                          heartbeat_ns=100_000_000, hb_phase_ns=ph)
    sm, sc, so = r["snaps"]
    h_lo = r["h_lo"]
    N = p.peers
    for e in range(0, len(sc), 7):
        for u in range(0, N, 13):
            assert bool(so[e, u]) == _py_offline(p, u, h_lo + e)
    for e in range(len(sc)):
        rows = [set(int(x) for x in sm[e, u, :sc[e, u]]) for u in range(N)]
        off = so[e].astype(bool)
        assert all(len(rows[u]) == 0 for u in np.flatnonzero(off))
        for u in range(N):
            assert not any(off[w] for w in rows[u])
            assert all(u in rows[w] for w in rows[u])
    q = 1 - (1 - p.churn_ppm / 1e6) ** p.churn_down
    assert abs(so[1:].mean() - q) < 0.05
    for m in range(len(t)):
        e = (int(t[m]) - ph) // p.heartbeat_ns - h_lo
        if so[e, pub[m]]:
            assert (r["t_complete"][m] == np.iinfo(np.uint64).max).all()
        else:
            assert r["t_complete"][m, pub[m]] == t[m]


@pytest.mark.parametrize("name,sub,epochs", [("uniform_n300", 1, 65), ("uniform_n300", 0, 7),
                                             ("hetero_n400_f4", 1, 6), ("hetero_n400_f4", 0, 67)])
def test_convergence_epochs_follow_the_prune_backoff(name, sub, epochs):
    """Why the committed fixtures' convergence epochs moved when subscription
    grafting was switched on (7 -> 65 uniform, 67 -> 6 heterogeneous): on
    uniform links every subscription arrives at the same instant, so each peer
    grafts its D_lo lowest-id connections; the low ids collect more GRAFTs than
    D_hi, reject the peers they did not dial, and each rejection is a PRUNE with
    the 60-heartbeat back-off (main.rs:229) — the mesh settles only after the
    back-offs expire (> 60 epochs). On heterogeneous links the handshake order
    spreads the grafts by latency and nothing waits for a back-off, while the
    random heartbeat grafts of the other start do trip one."""
    import json
    meta = json.load(open(os.path.join(GOLDEN, "oracle_%s.json" % name)))
    kw = dict(meta["params"], sub_graft=sub)
    p = oracle.params(**kw)
    S = meta["stages"]
    lat, _ = oracle.topogen_links(S, *meta["links"])
    stage = (np.arange(p.peers) % S).astype(np.uint8)
    row, col, flags0 = oracle.build_topology(p)
    _, _, _, ep = oracle.mesh_converge(p, row, col, flags0, stage, lat)
    assert ep == epochs
    backoff = p.backoff_ns // p.heartbeat_ns
    assert (ep > backoff) == (epochs > 60)
    if sub and S == 1:  # the epoch-0 grafts all go to the lowest ids
        row = row.astype(np.int64)
        out = set((u, int(col[e])) for u in range(p.peers) for e in range(row[u], row[u + 1]) if flags0[e] & 1)
        mesh0 = _py_subscription_epoch(p, row, col, out, stage, lat)
        assert max(len(m) for m in mesh0[:10]) > p.d_hi  # popular low ids hold more than D_hi before heartbeat 1
