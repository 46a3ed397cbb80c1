"""CPU tests of the product's host side: the C-ABI library loads and exports every
symbol include/gossipsim.h declares, and its host-only helpers (wire bytes,
topogen links, run.sh schedule, env surface, arrival-log writer) agree with the
oracle and the reference's golden artefacts. No device compute is called."""
import ctypes
import glob
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import gossipsim
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
HEADER = os.path.join(ROOT, "include", "gossipsim.h")
REF_SHADOW = "/root/reference/shadow"


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gs_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = gossipsim.lib()
    syms = declared_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(gossipsim.SIGNATURES)


def test_abi_struct_layouts_match_header(tmp_path):
    """The ctypes mirror of the ABI structs (gossipsim.py) has the layout the
    header gives a C compiler: sizes and every field offset of gs_result_sink
    (incl. ABI 7's `want`), gs_config, gs_publish, gs_stats, gs_msg_summary;
    GS_ABI_VERSION and the GS_WANT_* bits."""
    import ctypes
    import subprocess
    structs = {"gs_result_sink": gossipsim.GsResultSink, "gs_config": gossipsim.GsConfig,
               "gs_publish": gossipsim.GsPublish, "gs_stats": gossipsim.GsStats,
               "gs_msg_summary": gossipsim.GsMsgSummary}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gossipsim.h"', "int main(void) {",
             '  printf("abi %u\\n", GS_ABI_VERSION);',
             '  printf("want %u,%u\\n", (unsigned)GS_WANT_T_COMPLETE, (unsigned)GS_WANT_HOPS);']
    for name, cls in structs.items():
        lines.append('  printf("%s size %%zu\\n", sizeof(%s));' % (name, name))
        for f, _ in cls._fields_:
            lines.append('  printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (name, f, name, f))
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)])
    got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)]).decode().splitlines())
    assert int(got["abi"]) == gossipsim.ABI_VERSION == 10
    assert got["want"] == "%d,%d" % (gossipsim.WANT_T_COMPLETE, gossipsim.WANT_HOPS)
    for name, cls in structs.items():
        assert int(got["%s size" % name]) == ctypes.sizeof(cls), name
        for f, _ in cls._fields_:
            assert int(got["%s.%s" % (name, f)]) == getattr(cls, f).offset, (name, f)
    assert "want" in [f for f, _ in gossipsim.GsResultSink._fields_]


def test_no_gpu_means_loud_failure():
    """Without a device the product raises; there is no CPU fallback path."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(gossipsim.GossipSimError) as e:
        gossipsim.Simulator(peers=50)
    assert e.value.status == -3  # GS_EDEVICE


@pytest.mark.parametrize("muxer", [0, 1, 2])
@pytest.mark.parametrize("signed", [0, 1])
def test_wire_bytes_match_oracle(muxer, signed):
    for payload in [8, 11, 100, 1000, 1460, 1875, 15000, 16380, 65519, 70000, 1 << 20]:
        assert gossipsim.wire_bytes(payload, muxer, signed) == oracle.wire_bytes(payload, muxer, signed)


@pytest.mark.parametrize("muxer", [0, 1, 2])
@pytest.mark.parametrize("signed", [0, 1])
def test_wire_packets_match_oracle(muxer, signed):
    for payload in [8, 100, 1300, 1460, 1875, 2900, 15000, 65519, 1 << 20]:
        pk, hd = gossipsim.wire_packets(payload, muxer, signed)
        assert (pk, hd) == oracle.wire_packets(payload, muxer, signed)
        assert hd == pk * (65 if muxer == 1 else 40) and pk >= 1


def test_control_packets_match_oracle():
    for node in ("rust", "go", "nim"):
        for muxer in ("yamux", "quic", "mplex"):
            for kind in ("ihave", "iwant", "ack"):
                got = gossipsim.control_packets(kind, node, muxer)
                assert got == oracle.ctrl_packets(gossipsim.CTRL_KINDS[kind], gossipsim.NODES[node],
                                                  gossipsim.MUXERS[muxer])


def _shadow_log(tmp_path):
    """A config #3-style report (heterogeneous links, lazy gossip with IWANTs,
    churn) from the oracle's per-peer traffic."""
    p = oracle.params(peers=300, seed=5, fragments=2, churn_ppm=20000, heartbeat_ns=200_000_000,
                      hb_phase_ns=gossipsim.T0_NS - 2_000_000_000, churn_horizon=10)
    t = np.uint64(gossipsim.T0_NS) + np.arange(3, dtype=np.uint64) * np.uint64(10 ** 9)
    r = oracle.simulate(p, 3, (20, 80, 30, 60), sched=(t, np.array([1, 40, 79]), np.full(3, 15000)), traffic=True)
    assert r["stats"]["gossip_iwant"] > 0
    out = str(tmp_path / "shadowlog")
    gossipsim.write_shadow_heartbeat(out, r["traffic"], sim_seconds=900)
    return r["traffic"], out


def test_shadow_heartbeat_lines(tmp_path):
    tr, out = _shadow_log(tmp_path)
    lines = open(out).read().splitlines()
    assert len(lines) == tr.shape[0]
    for u, ln in enumerate(lines):
        f = ln.split()
        assert f[4] == "[pod-%d]" % u and f[8] == "[node]"
        arr = [int(x) for x in re.split(",|;", f[9])]
        assert arr[1] == tr[u, 1] + tr[u, 11] and arr[2] == tr[u, 0] + tr[u, 10]
        ri, ro = 6 + 24, 6 + 36  # remote in / out groups (0-based; awk's arr[idx] is 1-based)
        assert arr[ri:ri + 9] == [tr[u, 3] + tr[u, 9], tr[u, 1] + tr[u, 11], tr[u, 9], tr[u, 11], 0, 0,
                                  tr[u, 3], tr[u, 5], tr[u, 1] - tr[u, 5]]
        assert arr[ro:ro + 9] == [tr[u, 2] + tr[u, 8], tr[u, 0] + tr[u, 10], tr[u, 8], tr[u, 10], 0, 0,
                                  tr[u, 2], tr[u, 4], tr[u, 0] - tr[u, 4]]


@pytest.mark.skipif(not os.path.isdir(REF_SHADOW) or not shutil.which("awk"),
                    reason="reference awk scripts only in the build container")
def test_shadow_heartbeat_round_trips_through_reference_awk(tmp_path):
    tr, out = _shadow_log(tmp_path)
    got = subprocess.check_output(["awk", "-f", os.path.join(REF_SHADOW, "summary_shadowlog.awk"), out]).decode()
    s = lambda c: int(tr[:, c].sum())
    m = re.search(r"Total Bytes Received :\s+(\d+)\s+Total Bytes Transferred :\s+(\d+)", got)
    assert m and int(m.group(1)) == s(1) + s(11) and int(m.group(2)) == s(0) + s(10)
    num = r"\s+(\d+)\s+"
    pat = ("Remote %s pkt:" + num + "Bytes :" + num + "ctrlPkt:" + num + "ctrlHdrBytes:" + num + "DataPkt:" + num +
           "DataHdrBytes:" + num + r"DataBytes\s+(\d+)")
    m = re.search(pat % "IN", got)
    assert m and [int(x) for x in m.groups()] == [s(3) + s(9), s(1) + s(11), s(9), s(11), s(3), s(5), s(1) - s(5)]
    m = re.search(pat.replace("Bytes :" + num, r"Bytes :\s+(\d*)\s+") % "OUT", got)  # the awk prints an unset name
    assert m and [int(x) for x in m.groups()[2:]] == [s(8), s(10), s(2), s(4), s(0) - s(4)]
    assert s(0) > s(1)  # churn: lost sends


def test_node_metrics_openmetrics(tmp_path):
    """rust-test-node's metric names (metrics.rs:60-129) per peer from the simulator's counters."""
    p = oracle.params(peers=120, seed=6)
    t = np.uint64(gossipsim.T0_NS) + np.arange(5, dtype=np.uint64) * np.uint64(10 ** 9)
    pubs = np.array([0, 7, 7, 60, 119])
    r = oracle.simulate(p, 5, (50, 150, 40, 130), sched=(t, pubs, np.full(5, 15000)), traffic=True)
    cfg = gossipsim.PeerConfig(peers=120)
    out = str(tmp_path / "metrics.txt")
    gossipsim.write_node_metrics(cfg, out, r["row_ptr"], r["cnt"], r["traffic"])
    text = open(out).read()
    assert text.endswith("# EOF\n")
    vals = {}
    for ln in text.splitlines():
        m = re.match(r'(\w+)\{(?:topic="test",)?peer="pod-(\d+)"\} (\d+)$', ln)
        if m:
            vals.setdefault(m.group(1), {})[int(m.group(2))] = int(m.group(3))
    deg = np.diff(r["row_ptr"].astype(np.int64))
    assert [vals["libp2p_peers"][u] for u in range(120)] == deg.tolist()
    assert [vals["libp2p_gossipsub_peers_per_topic_mesh"][u] for u in range(120)] == r["cnt"].tolist()
    recv = (r["t_complete"] != np.iinfo(np.uint64).max).sum(axis=0) - np.bincount(pubs, minlength=120)
    assert [vals["libp2p_gossipsub_received_total"][u] for u in range(120)] == recv.tolist()
    assert vals["libp2p_pubsub_messages_published_total"][7] == 2 and sum(
        vals["libp2p_pubsub_messages_published_total"].values()) == 5
    assert all(vals["libp2p_gossipsub_healthy_peers_topics"][u] == (r["cnt"][u] >= 4) for u in range(120))
    assert "# TYPE libp2p_gossipsub_received counter" in text


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "topogen_*.json"))))
@pytest.mark.parametrize("shortest", [False, True])
def test_topogen_links_match_oracle_and_fixture(path, shortest):
    fx = json.load(open(path))
    a = {"-bl": 50, "-bh": 50, "-ll": 100, "-lh": 100, "-st": 1}
    for i in range(0, len(fx["flags"]), 2):
        if fx["flags"][i] in a:
            a[fx["flags"][i]] = int(fx["flags"][i + 1])
    S = a["-st"]
    lat, bw = gossipsim.topogen_links(S, a["-bl"], a["-bh"], a["-ll"], a["-lh"], shortest)
    olat, obw = oracle.topogen_links(S, a["-bl"], a["-bh"], a["-ll"], a["-lh"], 1 if shortest else 0)
    np.testing.assert_array_equal(lat, olat)
    np.testing.assert_array_equal(bw, obw)
    if not shortest:
        for s, t, l, _ in fx["edges"]:
            if s < S and t < S:
                assert lat[s, t] == l * 1_000_000


@pytest.mark.parametrize("name,S,links", [("runsh_example", 5, (50, 150, 40, 130)),
                                          ("seven_stages", 7, (10, 1000, 5, 300))])
@pytest.mark.parametrize("shortest", [False, True])
def test_gml_and_shadow_yaml_ingest(name, S, links, shortest):
    """topogen's own GML / shadow.yaml (tests/golden, made by running shadow/topogen.py)
    read back == the topogen arithmetic restated in gs_topogen_links."""
    lat, up, dn = gossipsim.links_from_gml(os.path.join(GOLDEN, "topogen_%s.gml" % name), shortest)
    tlat, tbw = gossipsim.topogen_links(S, *links, shortest)
    assert lat.shape == (S + 1, S + 1)  # + topogen's injector node
    np.testing.assert_array_equal(lat[:S, :S], tlat)
    np.testing.assert_array_equal(up[:S], tbw)
    np.testing.assert_array_equal(dn[:S], tbw)
    assert up[S] == dn[S] == 100_000_000  # the injector node: 100 Mbit (topogen.py:64-69)
    if not shortest:
        assert (lat[S, :S] == 1_000_000).all()
    fx = json.load(open(os.path.join(GOLDEN, "topogen_%s.json" % name)))
    st = gossipsim.shadow_hosts(os.path.join(GOLDEN, "topogen_%s.yaml" % name), len(fx["host_stage"]))
    np.testing.assert_array_equal(st, fx["host_stage"])
    np.testing.assert_array_equal(st, np.arange(len(st)) % S)  # topogen.py:121-122
    with pytest.raises(gossipsim.GossipSimError, match="GS_EINVAL"):  # more peers than hosts
        gossipsim.shadow_hosts(os.path.join(GOLDEN, "topogen_%s.yaml" % name), len(st) + 5)


def test_gml_rejects_packet_loss(tmp_path):
    g = open(os.path.join(GOLDEN, "topogen_runsh_example.gml")).read().replace("packet_loss 0.0", "packet_loss 0.01", 1)
    (tmp_path / "lossy.gml").write_text(g)
    with pytest.raises(gossipsim.GossipSimError, match="GS_EUNSUPPORTED"):
        gossipsim.links_from_gml(str(tmp_path / "lossy.gml"))


def test_schedule_runsh():
    # run.sh:34-36: publisher_id, rotation, inter_message_delay (ms)
    sch = gossipsim.schedule_runsh(5, 100, 98, 1, 10, 1_000_000_000, 15000)
    assert [s.publisher for s in sch] == [98, 99, 0, 1, 2]
    assert [s.t_pub_ns for s in sch] == [10 + i * 1_000_000_000 for i in range(5)]
    sch = gossipsim.schedule_runsh(3, 100, 4, 0, 0, 4_000_000_000, 15000)
    assert [s.publisher for s in sch] == [4, 4, 4] and sch[2].t_pub_ns == 8_000_000_000


def _emit_awk_fixture(tmp_path):
    arrivals = json.load(open(os.path.join(GOLDEN, "awk_arrivals.json")))
    txs = sorted(set(a[1] for a in arrivals))
    peers = 13
    sched = (gossipsim.GsPublish * len(txs))()
    tc = np.full((len(txs), peers), np.iinfo(np.uint64).max, np.uint64)
    for i, tx in enumerate(txs):
        sched[i] = gossipsim.GsPublish(tx, 0, 15000)  # publisher 0 never logs (rust preset)
        tc[i, 0] = tx
    for peer, tx, ms in arrivals:
        tc[txs.index(tx), peer] = tx + ms * 1_000_000 + 123_456  # sub-ms part is truncated
    out = str(tmp_path / "latencies")
    rc = gossipsim.lib().gs_write_latency_log(out.encode(), sched, len(txs), peers,
                                              tc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 0)
    assert rc == 0
    return out


def test_latency_log_matches_reference_grep_format(tmp_path):
    out = _emit_awk_fixture(tmp_path)
    assert open(out).read() == open(os.path.join(GOLDEN, "awk_latencies.txt")).read()


@pytest.mark.skipif(not os.path.isdir(REF_SHADOW) or not shutil.which("awk"),
                    reason="reference awk scripts only in the build container")
@pytest.mark.parametrize("script", ["summary_latency", "summary_latency_large"])
def test_latency_log_round_trips_through_reference_awk(tmp_path, script):
    out = _emit_awk_fixture(tmp_path)
    got = subprocess.check_output(["awk", "-f", os.path.join(REF_SHADOW, script + ".awk"), out]).decode()
    want = open(os.path.join(GOLDEN, "awk_latencies__%s.txt" % script)).read()
    assert got == want


def test_config_from_env_defaults_and_errors(monkeypatch):
    for k in ("PEERS", "CONNECTTO", "FRAGMENTS", "MUXER", "MAXCONNECTIONS", "GOSSIPSUB_D"):
        monkeypatch.delenv(k, raising=False)
    c = gossipsim.PeerConfig.from_env()
    assert (c.peers, c.connect_to, c.fragments, c.muxer) == (100, 10, 1, 0)  # env.rs:38-67
    assert (c.d, c.d_lo, c.d_hi, c.d_out, c.d_lazy) == (6, 4, 8, 3, 6)      # main.rs:36-38,234-235
    monkeypatch.setenv("PEERS", "2000")
    monkeypatch.setenv("MUXER", "QUIC")
    monkeypatch.setenv("FRAGMENTS", "8")
    monkeypatch.setenv("GOSSIPSUB_D_HIGH", "12")
    monkeypatch.setenv("GOSSIPSUB_GOSSIP_FACTOR", "0.5")
    c = gossipsim.PeerConfig.from_env()
    assert (c.peers, c.muxer, c.fragments, c.d_hi, c.gossip_factor_milli) == (2000, 1, 8, 12, 500)
    monkeypatch.setenv("PEERS", "notanumber")  # parse().unwrap_or(100) (env.rs:38-41)
    assert gossipsim.PeerConfig.from_env().peers == 100
    monkeypatch.setenv("MUXER", "tcp")
    with pytest.raises(gossipsim.GossipSimError, match="Unknown muxer type: tcp"):
        gossipsim.PeerConfig.from_env()
    monkeypatch.setenv("MUXER", "yamux")
    monkeypatch.setenv("PEERS", "10")
    monkeypatch.setenv("CONNECTTO", "10")
    with pytest.raises(gossipsim.GossipSimError, match="Not enough peers"):
        gossipsim.PeerConfig.from_env()


@pytest.mark.parametrize("node", ["rust", "go", "nim"])
def test_node_presets_match_oracle_restatement(node):
    """gs_config_preset == the oracle's own reading of each node's settings."""
    c = gossipsim.PeerConfig(node=node)
    p = oracle.params_for(node)
    for name, _ in oracle.OrParams._fields_:
        assert getattr(c, name) == getattr(p, name), name


def test_gs_node_env_selects_preset(monkeypatch):
    for k in ("PEERS", "CONNECTTO", "MAXCONNECTIONS", "SELFTRIGGER", "MUXER", "GOSSIPSUB_D_OUT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("GS_NODE", "nim")
    c = gossipsim.PeerConfig.from_env()
    assert (c.node, c.dial_extra, c.max_connections, c.d_out, c.self_log, c.signed_msgs) == (2, 0, 250, 3, 1, 0)
    monkeypatch.setenv("MAXCONNECTIONS", "40")  # env still overrides the preset (main.nim:429)
    monkeypatch.setenv("SELFTRIGGER", "false")  # main.nim:245
    c = gossipsim.PeerConfig.from_env()
    assert (c.max_connections, c.self_log) == (40, 0)
    monkeypatch.setenv("GS_NODE", "GO")
    c = gossipsim.PeerConfig.from_env()
    assert (c.node, c.d_out, c.idontwant, c.signed_msgs) == (1, 2, 1000, 0)
    monkeypatch.setenv("GS_NODE", "java")
    with pytest.raises(gossipsim.GossipSimError, match="Unknown node type: java"):
        gossipsim.PeerConfig.from_env()


def _node_log(tmp_path, node, self_log):
    cfg = gossipsim.PeerConfig(node=node, peers=4, self_log=self_log, seed=9)
    tx = [1_700_000_000_000_000_000, 1_700_000_001_000_000_000]
    sched = (gossipsim.GsPublish * 2)(gossipsim.GsPublish(tx[0], 0, 15000), gossipsim.GsPublish(tx[1], 2, 15000))
    tc = np.array([[tx[0], tx[0] + 120_400_000, gossipsim.UNDELIVERED, tx[0] + 95_000_001],
                   [tx[1] + 310_999_999, tx[1] + 5_000_000, tx[1], tx[1] + 230_000_000]], np.uint64)
    out = str(tmp_path / ("latencies_" + node))
    rc = gossipsim.lib().gs_write_node_log(ctypes.byref(cfg.c), out.encode(), sched, 2,
                                           tc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert rc == 0
    return [l.split(":", 2) for l in open(out).read().splitlines()], tx


def test_node_log_lines(tmp_path):
    rows, tx = _node_log(tmp_path, "rust", 0)
    assert [r[2] for r in rows] == ["%d milliseconds: 310" % tx[1], "%d milliseconds: 120" % tx[0],
                                    "%d milliseconds: 5" % tx[1], "%d milliseconds: 95" % tx[0],
                                    "%d milliseconds: 230" % tx[1]]
    rows_go, _ = _node_log(tmp_path, "go", 1)  # go: same line, own publish delivered locally
    assert len(rows_go) == len(rows) + 2
    nim, _ = _node_log(tmp_path, "nim", 1)     # nim: "<msgId> milliseconds: <ms>" (main.nim:150)
    ids = {}
    for path, _, text in nim:
        mid, rest = text.split(" ", 1)
        assert int(mid) < 2 ** 63 and int(mid) not in tx
        ids.setdefault(rest.split()[-1], set()).add(mid)
    assert len({m for s in ids.values() for m in s}) == 2  # one id per message


@pytest.mark.skipif(not os.path.isdir(REF_SHADOW) or not shutil.which("awk"),
                    reason="reference awk scripts only in the build container")
def test_nim_log_round_trips_through_reference_awk(tmp_path):
    _node_log(tmp_path, "nim", 1)
    got = subprocess.check_output(["awk", "-f", os.path.join(REF_SHADOW, "summary_latency.awk"),
                                   str(tmp_path / "latencies_nim")]).decode()
    assert re.search(r"Total Messages Published :\s+2\b", got) and re.search(r"Total Nodes :\s+3\b", got)
    assert re.search(r"MAX :\s+310\b", got)


def test_shard_messages_partition():
    """Message sharding used by bench.py: disjoint, covering, publisher rule of run.sh."""
    N, B, world, steps = 1000, 8, 4, 3
    seen = []
    for step in range(steps):
        for rank in range(world):
            t, pub, size = gossipsim.shard_messages(step, rank, world, B, N, 15000)
            assert len(t) == B
            seen.extend(zip(t.tolist(), pub.tolist()))
    assert len(set(seen)) == steps * world * B
    idx = sorted((t - gossipsim.T0_NS) // gossipsim.DELAY_NS for t, _ in seen)
    assert idx == list(range(steps * world * B))
    for t, p in seen:
        assert p == (6 + (t - gossipsim.T0_NS) // gossipsim.DELAY_NS) % N


def test_shadow_injector_from_topogen_yaml():
    """The controller host topogen writes (topogen.py:125-136): traffic_sync.py's
    -s / -m / -d / -n args and its start_time, from the committed topogen output."""
    inj = gossipsim.shadow_injector(os.path.join(GOLDEN, "topogen_runsh_example.yaml"))
    assert inj == dict(start_ns=500_000_000_000, delay_ns=1_000_000_000, msg_size=15000, messages=10, peers=100)
    with pytest.raises(gossipsim.GossipSimError):
        gossipsim.shadow_injector(os.path.join(GOLDEN, "topogen_runsh_example.gml"))


def test_read_schedule_file(tmp_path):
    path = tmp_path / "sched.txt"
    path.write_text("# t_pub_ns publisher msg_size [frags]\n"
                    "946685300003000000 6 15000\n\n"
                    "946685301003000000 7 15000 3   # three chunks\n"
                    "946685302003000000 8 4000 0\n")
    rows = gossipsim.read_schedule(str(path))
    got = [(r.t_pub_ns, r.publisher, r.msg_size, r.frags) for r in rows]
    assert got == [(946685300003000000, 6, 15000, 0), (946685301003000000, 7, 15000, 3),
                   (946685302003000000, 8, 4000, 0)]
    bad = tmp_path / "bad.txt"
    bad.write_text("946685300003000000 6\n")
    with pytest.raises(gossipsim.GossipSimError, match="GS_EINVAL"):
        gossipsim.read_schedule(str(bad))


def _oracle_run_for_log(N=400, M=12, seed=17, node="rust"):
    p = oracle.params_for(node, peers=N, seed=seed)
    t = np.uint64(gossipsim.T0_NS) + np.arange(M, dtype=np.uint64) * np.uint64(gossipsim.DELAY_NS)
    pub = ((6 + np.arange(M)) % N).astype(np.uint32)
    r = oracle.simulate(p, 5, (50, 150, 40, 130), sched=(t, pub, np.full(M, 15000)))
    sched = gossipsim.schedule_runsh(M, N, 6, 1, gossipsim.T0_NS, gossipsim.DELAY_NS, 15000)
    cfg = gossipsim.PeerConfig(node=node, peers=N, seed=seed)
    return cfg, sched, r["t_complete"]


@pytest.mark.parametrize("node", ["rust", "nim"])
def test_streaming_log_equals_grouped_writer(tmp_path, node):
    """gs_log_* (blocks of message-major results, as gs_result_sink.on_block
    hands them over) writes exactly the lines of the grouped writer; only the
    order differs (block by block instead of peer by peer)."""
    cfg, sched, tc = _oracle_run_for_log(node=node)
    grouped = str(tmp_path / "grouped")
    rc = gossipsim.lib().gs_write_node_log(ctypes.byref(cfg.c), grouped.encode(), sched, len(sched),
                                           tc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert rc == 0
    log = gossipsim.LogStream(cfg, str(tmp_path / "stream"))
    for q0 in range(0, len(sched), 5):
        log.write(sched[q0:q0 + 5], tc[q0:q0 + 5])
    log.close()
    a = open(grouped).read().splitlines()
    b = open(str(tmp_path / "stream")).read().splitlines()
    assert sorted(a) == sorted(b) and len(a) > 0


@pytest.mark.skipif(not os.path.isdir(REF_SHADOW) or not shutil.which("awk"),
                    reason="reference awk scripts only in the build container")
def test_streaming_log_round_trips_through_summary_latency_large(tmp_path):
    """The streamed log through the reference's summary_latency_large.awk: its
    per-message "MAX delay" lines equal the per-message maxima of the results
    (the max_ms of gs_msg_summary), and its message count is the schedule's."""
    cfg, sched, tc = _oracle_run_for_log()
    log = gossipsim.LogStream(cfg, str(tmp_path / "lat"))
    for q0 in range(0, len(sched), 4):
        log.write(sched[q0:q0 + 4], tc[q0:q0 + 4])
    log.close()
    got = subprocess.check_output(["awk", "-f", os.path.join(REF_SHADOW, "summary_latency_large.awk"),
                                   str(tmp_path / "lat")]).decode()
    mx = {}
    for line in got.splitlines():
        m = re.match(r"MAX delay for\s+(\d+)\s+is\s+(\d+)", line)
        if m:
            mx[int(m.group(1))] = int(m.group(2))
    want = {}
    for q, row in enumerate(sched):
        ok = tc[q] != np.iinfo(np.uint64).max
        ok[row.publisher] = False
        want[row.t_pub_ns] = int(((tc[q][ok] - np.uint64(row.t_pub_ns)) // np.uint64(1_000_000)).max())
    assert mx == want
    assert "Total Messages Published :  %d" % len(sched) in got


def test_load_state_rejects_foreign_files(tmp_path):
    """gs_load_state refuses a file that is not a state file of this ABI before
    it touches a device (GS_EINVAL; CPU only: no context is created)."""
    import ctypes
    import struct
    lib = gossipsim.lib()
    out = ctypes.c_void_p()
    bad = tmp_path / "bad"
    bad.write_bytes(b"NOTSTATE" + bytes(64))
    assert lib.gs_load_state(str(bad).encode(), 0, ctypes.byref(out)) == gossipsim.GS_EINVAL
    old = tmp_path / "old"
    old.write_bytes(b"GSIMST01" + struct.pack("<I", gossipsim.ABI_VERSION - 1) + bytes(256))
    assert lib.gs_load_state(str(old).encode(), 0, ctypes.byref(out)) == gossipsim.GS_EINVAL
    short = tmp_path / "short"
    short.write_bytes(b"GSIMST01" + struct.pack("<I", gossipsim.ABI_VERSION) + bytes(8))
    assert lib.gs_load_state(str(short).encode(), 0, ctypes.byref(out)) == gossipsim.GS_EINVAL
    assert lib.gs_load_state(str(tmp_path / "missing").encode(), 0, ctypes.byref(out)) == gossipsim.GS_EINVAL
    assert not out.value


LAYOUT_CHECK = r"""
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gs_layout.h"
using namespace gs;
static uint64_t code(uint64_t m, uint64_t u) { return (m << 32) | u; }
int main() {
  const uint32_t Ns[] = {7, 97, 1000, 4099};
  const uint32_t Bs[] = {1, 2, 3, 5, 16, 17, 1024};
  unsigned long long checks = 0;
  for (uint32_t P = 1; P <= 8; P++)
    for (uint32_t N : Ns)
      for (uint32_t B : Bs) {
        if (P > N) continue;
        const PartLayout L{P, N, B};
        // peers and messages: contiguous covers
        if (L.u0(0) != 0 || L.u0(P) != N || L.m0(0) != 0 || L.m0(P) != B) { puts("cover"); return 1; }
        for (uint32_t p = 0; p < P; p++)
          if (L.u0(p + 1) < L.u0(p) || L.m0(p + 1) < L.m0(p) || L.mn(p) > L.mmax()) { puts("order"); return 1; }
        // message-sharded all-to-all, RCCL form: pack per destination, one send / recv per pair
        std::vector<std::vector<uint64_t>> res(P), send(P), recv(P), loop(P);
        for (uint32_t s = 0; s < P; s++) {
          res[s].resize((size_t)L.mn(s) * N);
          for (uint32_t i = 0; i < L.mn(s); i++)
            for (uint32_t u = 0; u < N; u++) res[s][(size_t)i * N + u] = code(L.m0(s) + i, u);
          send[s].assign((size_t)L.mn(s) * N, ~0ull);
          uint64_t packed = 0;
          for (uint32_t d = 0; d < P; d++) {
            if (L.ms_send_off(s, d) != packed) { puts("send tiling"); return 1; }
            for (uint32_t i = 0; i < L.mn(s); i++)
              for (uint32_t j = 0; j < L.un(d); j++)
                send[s][L.ms_send_off(s, d) + (size_t)i * L.un(d) + j] = res[s][(size_t)i * N + L.u0(d) + j];
            packed += L.ms_count(s, d);
          }
          if (packed != (uint64_t)L.mn(s) * N) { puts("send size"); return 1; }
        }
        for (uint32_t d = 0; d < P; d++) {
          recv[d].assign((size_t)B * L.un(d), ~0ull);
          loop[d].assign((size_t)B * L.un(d), ~0ull);
          uint64_t got = 0;
          for (uint32_t s = 0; s < P; s++) {
            if (L.ms_recv_off(s, d) != got) { puts("recv tiling"); return 1; }
            for (uint64_t k = 0; k < L.ms_count(s, d); k++)
              recv[d][L.ms_recv_off(s, d) + k] = send[s][L.ms_send_off(s, d) + k];
            // loop-back form: a 2-D copy straight from s's rows
            for (uint32_t i = 0; i < L.mn(s); i++)
              for (uint32_t j = 0; j < L.un(d); j++)
                loop[d][L.ms_recv_off(s, d) + (size_t)i * L.un(d) + j] = res[s][(size_t)i * N + L.u0(d) + j];
            got += L.ms_count(s, d);
          }
          if (got != (uint64_t)B * L.un(d)) { puts("recv size"); return 1; }
          for (uint32_t m = 0; m < B; m++)
            for (uint32_t j = 0; j < L.un(d); j++) {
              const uint64_t want = code(m, L.u0(d) + j);
              if (recv[d][(size_t)m * L.un(d) + j] != want || loop[d][(size_t)m * L.un(d) + j] != want) {
                printf("ms P=%u N=%u B=%u d=%u m=%u j=%u\n", P, N, B, d, m, j);
                return 1;
              }
              checks++;
            }
        }
        // list-pass record exchange: part p's records at base[p] of every gathered buffer
        std::vector<uint64_t> cnt(P), base(P + 1);
        for (uint32_t p = 0; p < P; p++) cnt[p] = (p * 7919u + N + B) % 13;
        const uint64_t tot = lp_bases(cnt.data(), P, base.data());
        std::vector<uint64_t> all(tot, ~0ull);
        for (uint32_t p = 0; p < P; p++)
          for (uint64_t k = 0; k < cnt[p]; k++) all[base[p] + k] = code(p, k);
        uint64_t q = 0;
        for (uint32_t p = 0; p < P; p++)
          for (uint64_t k = 0; k < cnt[p]; k++, q++)
            if (all[q] != code(p, k)) { puts("records"); return 1; }
      }
  printf("ok %llu\n", checks);
  return 0;
}
"""

ROUTE_CHECK = r"""
#include <cstdio>
#include <vector>
#include <random>
#include "gs_layout.h"
using namespace gs;
// The routed list-pass exchange simulated on the CPU: random mesh rows (<= 16
// entries, ids of any part), each row's records with random inclusion masks;
// sender p packs, per destination q, the records with a receiver in q (q = p:
// all) with per-peer offsets relative to the segment; receiver q lays the
// segments out by lp_route_bases and adds base[p] to p's offsets. Every
// receiver must then read, for each mesh neighbour, exactly the neighbour's
// records that include it, in emission order (what k_lpull<.., PART> reads).
int main() {
  std::mt19937_64 rng(7);
  unsigned long long checks = 0;
  const uint32_t Ns[] = {5, 37, 1000, 3001};
  for (uint32_t P = 1; P <= 16; P++)
    for (uint32_t N : Ns) {
      if (P > N) continue;
      const PartLayout L{P, N, 1};
      for (uint32_t p = 0; p < P; p++)
        for (uint32_t x = L.u0(p); x < L.u0(p + 1); x++)
          if (L.part_of(x) != p) { printf("part_of P=%u N=%u x=%u\n", P, N, x); return 1; }
      std::vector<std::vector<uint32_t>> mesh(N);
      std::vector<std::vector<uint32_t>> recs(N);  // record = emission index << 16 | inclusion mask
      for (uint32_t u = 0; u < N; u++) {
        const uint32_t d = (uint32_t)(rng() % 17);
        for (uint32_t k = 0; k < d; k++) mesh[u].push_back((uint32_t)(rng() % N));
        const uint32_t n = (uint32_t)(rng() % 9);
        for (uint32_t i = 0; i < n; i++) recs[u].push_back((i << 16) | (uint32_t)(rng() & ((1u << d) - 1)));
      }
      // sender side
      std::vector<std::vector<std::vector<uint32_t>>> seg(P, std::vector<std::vector<uint32_t>>(P));
      std::vector<std::vector<uint64_t>> roff(P, std::vector<uint64_t>(N)), rcg(P, std::vector<uint64_t>(N));
      std::vector<uint64_t> route((size_t)P * P);
      for (uint32_t p = 0; p < P; p++)
        for (uint32_t q = 0; q < P; q++) {
          uint32_t mq = 0;
          for (uint32_t u = L.u0(p); u < L.u0(p + 1); u++) {
            mq = 0;
            for (uint32_t k = 0; k < mesh[u].size(); k++) mq |= L.part_of(mesh[u][k]) == q ? 1u << k : 0u;
            roff[q][u] = seg[p][q].size();  // (tables per destination; u is p's own peer)
            for (uint32_t r : recs[u])
              if (q == p || (r & 0xFFFFu & mq)) seg[p][q].push_back(r);
            rcg[q][u] = seg[p][q].size() - roff[q][u];
          }
          route[(size_t)p * P + q] = seg[p][q].size();
        }
      // receiver side
      for (uint32_t q = 0; q < P; q++) {
        std::vector<uint64_t> base(P);
        const uint64_t tot = lp_route_bases(route.data(), P, q, base.data());
        std::vector<uint32_t> buf(tot, ~0u);
        std::vector<uint64_t> groff(N), grcg(N);
        for (uint32_t p = 0; p < P; p++) {
          for (size_t k = 0; k < seg[p][q].size(); k++) buf[base[p] + k] = seg[p][q][k];
          for (uint32_t u = L.u0(p); u < L.u0(p + 1); u++) {
            groff[u] = roff[q][u] + base[p];
            grcg[u] = rcg[q][u];
          }
        }
        for (uint32_t x : buf)
          if (x == ~0u) { puts("hole"); return 1; }
        for (uint32_t w = L.u0(q); w < L.u0(q + 1); w++)  // every own receiver w and neighbour entry
          for (uint32_t v = 0; v < N; v++)
            for (uint32_t k = 0; k < mesh[v].size(); k++) {
              if (mesh[v][k] != w) continue;
              std::vector<uint32_t> want, got;
              for (uint32_t r : recs[v])
                if ((r >> k) & 1u) want.push_back(r);
              for (uint64_t i = 0; i < grcg[v]; i++)
                if ((buf[groff[v] + i] >> k) & 1u) got.push_back(buf[groff[v] + i]);
              if (want != got) { printf("route P=%u N=%u q=%u w=%u v=%u\n", P, N, q, w, v); return 1; }
              checks++;
            }
      }
    }
  printf("ok %llu\n", checks);
  return 0;
}
"""


def test_partition_routed_record_exchange(tmp_path):
    """The routed list-pass record exchange (csrc/gs_layout.h part_of /
    lp_route_bases, packed by k_lpack_route): for P = 1..16 with uneven peer
    splits, a part receives from every other part only the records with a
    receiver it owns, laid out after its own records, and every receiver reads
    through the offset tables exactly its neighbours' records that include it,
    in order (SURVEY.md §8e's per-destination exchange)."""
    src = tmp_path / "route.cpp"
    src.write_text(ROUTE_CHECK)
    exe = tmp_path / "route"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "dst-libp2p-test-node_amd", "csrc"),
                           str(src), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    assert out.stdout.startswith("ok ") and int(out.stdout.split()[1]) > 10000


def test_partition_layout_exchanges(tmp_path):
    """gs_run_partitioned's block arithmetic (csrc/gs_layout.h, used by both
    the loop-back and the RCCL branches of gs_comm.hip): for P = 1..8 with
    uneven peer splits and batches smaller than P, the message-sharded
    all-to-all (pack per destination, one send / recv per pair, and the
    loop-back 2-D copies) hands every part exactly its peers' rows of every
    message, and the list pass's packed records tile the gathered buffer.
    RCCL with more than one rank never ran here (one GPU per box); this pins
    its offsets on the CPU."""
    src = tmp_path / "layout.cpp"
    src.write_text(LAYOUT_CHECK)
    exe = tmp_path / "layout"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "dst-libp2p-test-node_amd", "csrc"),
                           str(src), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert out.stdout.startswith("ok ") and int(out.stdout.split()[1]) > 100000


def test_uplink_fifo_closed_form(tmp_path):
    """uplink_start's prefix-sum form of the fragment FIFO (gs_relax_kernel.h)
    equals the sequential (key, fragment) fold it replaced, on 2M random
    groups of 2-16 fragments with ties, missing fragments and busy uplinks."""
    exe = tmp_path / "fifo_check"
    subprocess.run(["g++", "-O2", "-o", str(exe), os.path.join(ROOT, "scripts", "fifo_check.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout
