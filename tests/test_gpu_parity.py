"""GPU parity: libgossipsim (HIP, through the C ABI) vs the CPU oracle.

Bit-exact on every integer output: CSR (row_ptr, col, outbound bits), mesh,
per-(message, peer) completion time in ns, hop count, and the counters
(FD, R, deliveries, latency sums). Small sizes compare against the committed
fixtures and fresh oracle runs; large sizes check size-independent properties
plus a sample of messages against the oracle."""
import json
import os

import numpy as np
import pytest

import gossipsim
import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T0 = gossipsim.T0_NS
UND = np.iinfo(np.uint64).max


def _knobs(p):
    return {n: getattr(p, n) for n, _ in oracle.OrParams._fields_}


def gpu_sim(p, S, links, mode=0, batch=64, max_hb=400):
    kw = _knobs(p)
    kw["batch"] = batch
    sim = gossipsim.Simulator(**kw)
    sim.set_topogen_links(S, *links, shortest=bool(mode))
    sim.connect_gossipsub_peers()
    ep = sim.mesh_converge(max_hb)
    return sim, ep


def compare(p, S, links, sched, mode=0, batch=64, ref=None):
    sim, ep = gpu_sim(p, S, links, mode, batch)
    if ref is None:
        ref = oracle.simulate(p, S, links, mode=mode, sched=sched)
    row, col, flags = sim.csr()
    np.testing.assert_array_equal(row, ref["row_ptr"], err_msg="row_ptr")
    np.testing.assert_array_equal(col, ref["col"], err_msg="col")
    mesh, cnt = sim.mesh()
    np.testing.assert_array_equal(cnt, ref["cnt"], err_msg="mesh count")
    np.testing.assert_array_equal(mesh, ref["mesh"], err_msg="mesh")
    np.testing.assert_array_equal(flags, ref["flags"], err_msg="flags")
    assert ep == ref["epochs"]
    res = sim.run(sched)
    np.testing.assert_array_equal(res["t_complete"], ref["t_complete"], err_msg="t_complete")
    np.testing.assert_array_equal(res["hops"], ref["hops"], err_msg="hops")
    st = sim.stats()
    for k in ("deliveries", "frag_deliveries", "relaxations", "bytes_alg", "latency_sum_ms",
              "latency_max_ms", "messages", "gossip_iwant"):
        assert st[k] == ref["stats"][k], k
    return sim, res


def _sched(M, N, size=15000, pub0=6):
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
    return t, (pub0 + np.arange(M)) % N, np.full(M, size)


@pytest.mark.parametrize("name", ["uniform_n300", "hetero_n400_f4", "nim_n200_cap"])
def test_against_committed_oracle_fixtures(name):
    meta = json.load(open(os.path.join(GOLDEN, "oracle_%s.json" % name)))
    fx = np.load(os.path.join(GOLDEN, "oracle_%s.npz" % name))
    p = oracle.params(**meta["params"])
    ref = dict(row_ptr=fx["row_ptr"], col=fx["col"], flags=fx["flags"], mesh=fx["mesh"], cnt=fx["cnt"],
               t_complete=fx["t_complete"], hops=fx["hops"], epochs=int(fx["epochs"][0]), stats=meta["stats"])
    sched = (fx["sched_t"], fx["sched_pub"], np.full(meta["n_msgs"], meta["msg_size"]))
    compare(p, meta["stages"], tuple(meta["links"]), sched, ref=ref)


def test_config1_1k_peers_100_publishes():
    """Config #1: 1k peers, D=6, 100 publishes (publisher 6+i), uniform 50 ms / 50 Mbit."""
    for seed in (1, 2, 3):
        p = oracle.params(peers=1000, seed=seed)
        compare(p, 1, (50, 50, 50, 50), _sched(100, 1000), batch=100)


@pytest.mark.parametrize("frags", [2, 3, 8])
def test_fragments_uplink_fifo(frags):
    p = oracle.params(peers=700, seed=11, fragments=frags)
    compare(p, 5, (50, 150, 40, 130), _sched(12, 700), batch=5)


def test_multi_batch_uneven_and_varying_sizes():
    p = oracle.params(peers=900, seed=5)
    t, pub, size = _sched(23, 900)
    size = size.copy()
    size[7:15] = 3000  # size change splits batches
    compare(p, 3, (20, 200, 10, 90), (t, pub, size), batch=6)


def test_knob_variants():
    cases = [
        (dict(peers=500, seed=3, muxer=1, signed_msgs=0), 2, (10, 100, 5, 50), 0),
        (dict(peers=500, seed=4, flood_publish=0), 1, (50, 50, 50, 50), 0),
        (dict(peers=500, seed=6, idontwant=1000), 5, (50, 150, 40, 130), 0),
        (dict(peers=400, seed=8, dial_extra=0, max_connections=13, connect_to=8), 4, (50, 150, 40, 130), 0),
        (dict(peers=400, seed=9, d=8, d_lo=6, d_hi=12, d_out=2), 1, (100, 100, 30, 30), 0),
        (dict(peers=300, seed=10), 5, (50, 150, 40, 130), 1),  # Shadow shortest-path links
        (dict(peers=64, seed=12, connect_to=3), 1, (50, 50, 50, 50), 0),
    ]
    for kw, S, links, mode in cases:
        p = oracle.params(**kw)
        compare(p, S, links, _sched(9, p.peers), mode=mode, batch=4)


@pytest.mark.parametrize("frags", [1, 2, 3])
def test_lazy_gossip_ihave_iwant(frags):
    """A6: IHAVE/IWANT relaxations, heartbeats landing inside the dissemination
    window (fast heartbeat + phase) so that IWANTs actually happen."""
    p = oracle.params(peers=1500, seed=41, fragments=frags, lazy_gossip=1,
                      heartbeat_ns=100_000_000, hb_phase_ns=37_000_000)
    sim, res = compare(p, 3, (5, 20, 20, 80), _sched(20, 1500), batch=8)
    st = sim.stats()
    ref = oracle.simulate(p, 3, (5, 20, 20, 80), sched=_sched(20, 1500))
    assert st["gossip_iwant"] == ref["stats"]["gossip_iwant"] > 0


@pytest.mark.parametrize("factor,d_lazy", [(1000, 6), (500, 12)])
def test_lazy_gossip_wide_fanout(factor, d_lazy):
    """Gossip fan-out beyond the 8 targets k_gossip keeps in registers: the
    rescan path for the next smallest (rng, id) pair must pick the oracle's
    targets (gossip_factor 1.0 sends IHAVE to every non-mesh connection)."""
    p = oracle.params(peers=1200, seed=43, lazy_gossip=1, gossip_factor_milli=factor, d_lazy=d_lazy,
                      heartbeat_ns=100_000_000, hb_phase_ns=37_000_000)
    sim, _ = compare(p, 3, (5, 20, 20, 80), _sched(16, 1200), batch=8)
    assert sim.stats()["gossip_iwant"] > 0


def test_lazy_gossip_default_heartbeat():
    p = oracle.params(peers=3000, seed=42, lazy_gossip=1)
    compare(p, 5, (50, 150, 40, 130), _sched(30, 3000), batch=16)


@pytest.mark.parametrize("node", ["go", "nim"])
def test_node_presets(node):
    """go-test-node / nim gossipsub-queues settings and fragment layouts
    (gs_config_preset; go's IDONTWANT threshold puts 15 KB messages on the
    IDONTWANT path) bit-exact against the oracle, incl. the smallest valid
    fragments and the node's own publish failure."""
    p = oracle.params_for(node, peers=800, seed=61, fragments=3)
    compare(p, 5, (50, 150, 40, 130), _sched(10, 800), batch=4)
    small = 9 if node == "go" else 51  # msg_size / F = 3 (go) or 17 (nim): the first valid size
    compare(p, 5, (50, 150, 40, 130), _sched(6, 800, size=small), batch=3)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130))
    with pytest.raises(gossipsim.GossipSimError, match="GS_EINVAL"):
        sim.run(_sched(1, 800, size=small - 3))


@pytest.mark.parametrize("B,M", [(64, 70), (512, 512), (1024, 1024)])
def test_idontwant_on_list_pass(monkeypatch, B, M):
    """IDONTWANT (go preset: threshold 1000 B, go-test-node/main.go:165) on the
    list pass: single-fragment batches keep their final keys dense, the emit
    step tests every mesh neighbour's key and the records carry the exclusion
    mask (rows of 64, 512 and 1024 lanes); bit-exact against the oracle, and
    IDONTWANT really suppresses sends."""
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    p = oracle.params_for("go", peers=2000, seed=62, lazy_gossip=0)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(M, 2000), batch=B)
    st = sim.stats()
    assert st["list_pull_batches"] >= 1
    p0 = oracle.params_for("go", peers=2000, seed=62, lazy_gossip=0, idontwant=0)
    ref0 = oracle.simulate(p0, 5, (50, 150, 40, 130), sched=_sched(M, 2000))
    assert st["relaxations"] < ref0["stats"]["relaxations"]


def test_idontwant_list_overflow_and_gossip(monkeypatch):
    """An IDONTWANT batch whose candidate lists overflow re-runs on the push
    path (k_pull has no IDONTWANT); with the go preset's lazy gossip the
    batch's eager result stands when gossip is proven a no-op. Both bit-exact."""
    monkeypatch.setenv("GS_LPULL_CAP", "2")
    p = oracle.params_for("go", peers=1500, seed=63, lazy_gossip=0)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(200, 1500), batch=200)
    assert sim.stats()["list_pull_batches"] == 0
    monkeypatch.delenv("GS_LPULL_CAP")
    p = oracle.params_for("go", peers=1500, seed=64)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(100, 1500), batch=100)
    assert sim.stats()["list_pull_batches"] >= 1


_IWANT_PHASE = T0 % 1_000_000_000  # a heartbeat at the publish instant: IHAVEs race the eager wave


@pytest.mark.parametrize("kw", [dict(), dict(fragments=3), dict(flood_publish=0), dict(node=1, fragments=2),
                                dict(muxer=1, signed_msgs=0), dict(lazy_gossip=0),
                                dict(hb_phase_ns=_IWANT_PHASE), dict(hb_phase_ns=_IWANT_PHASE, fragments=4),
                                dict(node=2, hb_phase_ns=_IWANT_PHASE)])
def test_peer_traffic_counters(kw):
    """gs_set_traffic: per-peer tx/rx bytes, packets, header bytes and ACKs
    (Shadow's tracker counters) bit-exact against the oracle, on the pull path
    (gossip a no-op: IHAVEs only), the push path (go preset: IDONTWANT) and
    with gossip sending IWANTs, accumulated over two runs."""
    p = oracle.params_for(kw.pop("node", 0), peers=900, seed=71, **kw)
    sched = _sched(12, 900)
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched, traffic=True)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    sim.set_traffic(True)
    sim.run((sched[0][:5], sched[1][:5], sched[2][:5]))
    sim.run((sched[0][5:], sched[1][5:], sched[2][5:]))
    np.testing.assert_array_equal(sim.traffic(), ref["traffic"])
    if p.hb_phase_ns == _IWANT_PHASE:
        assert ref["stats"]["gossip_iwant"] > 0
    sim.reset_stats()
    assert not sim.traffic().any()


@pytest.mark.parametrize("kw", [dict(), dict(fragments=2), dict(flood_publish=0, lazy_gossip=0)])
def test_peer_traffic_under_churn(kw):
    """Config #3 semantics (heterogeneous links, churn, lazy gossip with IWANTs):
    lost sends count at the sender only, ACKs only for arrivals; bit-exact
    against the oracle."""
    N = 1500
    p = oracle.params(peers=N, seed=73, churn_ppm=20000, heartbeat_ns=200_000_000,
                      hb_phase_ns=T0 - 2_000_000_000, churn_horizon=10, **kw)
    sched = _sched(24, N)
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched, traffic=True)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    sim.set_traffic(True)
    res = sim.run(sched)
    np.testing.assert_array_equal(res["t_complete"], ref["t_complete"])
    tr = sim.traffic()
    np.testing.assert_array_equal(tr, ref["traffic"])
    assert tr[:, 0].sum() > tr[:, 1].sum()


def test_peer_traffic_needs_enabling():
    """gs_get_traffic before gs_set_traffic(ctx, 1) is a state error (the
    partitioned mode refuses traffic: test_gpu_partition)."""
    p = oracle.params(peers=300, seed=72)
    sim, _ = gpu_sim(p, 1, (50, 50, 50, 50))
    with pytest.raises(gossipsim.GossipSimError, match="GS_ESTATE"):
        sim.traffic()


def test_shadow_experiment_files_drive_the_run():
    """set_shadow_links(network_topology.gml, shadow.yaml) of topogen's run.sh
    example == the same links from topogen's parameters (the injector node is
    an extra link class no peer uses)."""
    p = oracle.params(peers=100, seed=81)
    sched = _sched(6, 100)
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
    kw = _knobs(p)
    sim = gossipsim.Simulator(batch=8, **kw)
    sim.set_shadow_links(os.path.join(GOLDEN, "topogen_runsh_example.gml"),
                         os.path.join(GOLDEN, "topogen_runsh_example.yaml"))
    sim.connect_gossipsub_peers()
    sim.mesh_converge()
    res = sim.run(sched)
    np.testing.assert_array_equal(res["t_complete"], ref["t_complete"])
    np.testing.assert_array_equal(res["hops"], ref["hops"])


def test_cli_runs_a_shadow_experiment(tmp_path):
    """gossipsim-node (the C++ host) on topogen's GML + shadow.yaml with the
    reference's env knobs: its arrival log equals the Python host's for the
    same run, and it writes the tracker heartbeat and metrics files."""
    import subprocess
    exe = os.path.join(os.path.dirname(gossipsim.LIB_PATH), "gossipsim-node")
    env = dict(os.environ, PEERS="100", CONNECTTO="10", FRAGMENTS="2", MUXER="yamux", GS_SEED="5")
    out = {k: str(tmp_path / k) for k in ("lat", "shadowlog", "metrics")}
    subprocess.run([exe, "--gml", os.path.join(GOLDEN, "topogen_runsh_example.gml"), "--yaml",
                    os.path.join(GOLDEN, "topogen_runsh_example.yaml"), "-s", "15000", "-m", "4",
                    "--publisher", "6", "--rotation", "1", "--delay-ms", "1000", "--latencies", out["lat"],
                    "--shadowlog", out["shadowlog"], "--metrics", out["metrics"]],
                   env=env, check=True, timeout=60)
    p = oracle.params(peers=100, seed=5, fragments=2)
    sim = gossipsim.Simulator(**_knobs(p))
    sim.set_shadow_links(os.path.join(GOLDEN, "topogen_runsh_example.gml"),
                         os.path.join(GOLDEN, "topogen_runsh_example.yaml"))
    sim.connect_gossipsub_peers()
    sim.mesh_converge()
    sched = gossipsim.schedule_runsh(4, 100, 6, 1, gossipsim.T0_NS, gossipsim.DELAY_NS, 15000)
    res = sim.run(sched)
    sim.write_latency_log(str(tmp_path / "py_lat"), res)
    # the CLI streams its log block by block: same lines, message-major order
    assert sorted(open(out["lat"]).read().splitlines()) == sorted(open(str(tmp_path / "py_lat")).read().splitlines())
    assert len(open(out["shadowlog"]).read().splitlines()) == 100
    assert open(out["metrics"]).read().endswith("# EOF\n")


def test_cli_injector_args_and_schedule_file(tmp_path):
    """A1 inputs: (1) --gml/--yaml alone takes traffic_sync.py's -s/-m/-d and
    start_time from shadow.yaml (topogen.py:125-136); (2) --schedule FILE with
    per-message chunk counts; both bit-exact against the oracle."""
    import subprocess
    exe = os.path.join(os.path.dirname(gossipsim.LIB_PATH), "gossipsim-node")
    gml, yml = (os.path.join(GOLDEN, "topogen_runsh_example." + x) for x in ("gml", "yaml"))
    env = dict(os.environ, PEERS="100", CONNECTTO="10", FRAGMENTS="1", GS_SEED="7")
    p = oracle.params(peers=100, seed=7)
    inj = gossipsim.shadow_injector(yml)
    t = np.uint64(946684800_000_000_000 + inj["start_ns"] + gossipsim.HTTP_TRANSIT_NS) + \
        np.arange(inj["messages"], dtype=np.uint64) * np.uint64(inj["delay_ns"])
    pub = (6 + np.arange(inj["messages"])) % 100
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=(t, pub, np.full(len(t), inj["msg_size"])))
    subprocess.run([exe, "--gml", gml, "--yaml", yml, "--latencies", str(tmp_path / "a")], env=env, check=True,
                   timeout=60)
    sim = gossipsim.Simulator(**_knobs(p))
    sched = gossipsim.schedule_runsh(len(t), 100, 6, 1, int(t[0]), inj["delay_ns"], inj["msg_size"])
    sim.write_latency_log(str(tmp_path / "b"), {"schedule": sched, "t_complete": ref["t_complete"]})
    assert sorted(open(str(tmp_path / "a")).read().splitlines()) == sorted(open(str(tmp_path / "b")).read().splitlines())
    # schedule file: mixed chunk counts, publishes 700 ms apart (overlapping in time)
    rows = [(int(T0) + i * 700_000_000, (11 * i + 3) % 100, 15000, [0, 3, 8, 1, 2, 16][i % 6]) for i in range(9)]
    (tmp_path / "sched").write_text("".join("%d %d %d %d\n" % r for r in rows))
    env2 = dict(env, FRAGMENTS="2")
    p2 = oracle.params(peers=100, seed=7, fragments=2)
    subprocess.run([exe, "--gml", gml, "--yaml", yml, "--schedule", str(tmp_path / "sched"), "--latencies",
                    str(tmp_path / "c")], env=env2, check=True, timeout=60)
    cols = [np.array([r[k] for r in rows]) for k in range(4)]
    ref2 = oracle.simulate(p2, 5, (50, 150, 40, 130), sched=(cols[0].astype(np.uint64), cols[1], cols[2], cols[3]))
    sched2 = gossipsim.read_schedule(str(tmp_path / "sched"))
    sim2 = gossipsim.Simulator(**_knobs(p2))
    sim2.write_latency_log(str(tmp_path / "d"), {"schedule": sched2, "t_complete": ref2["t_complete"]})
    assert sorted(open(str(tmp_path / "c")).read().splitlines()) == sorted(open(str(tmp_path / "d")).read().splitlines())


def test_cli_latency_past_u16(tmp_path):
    """A logged latency of 65535 ms or more (70 s heartbeats: a peer offline
    during the eager spread gets the message by IWANT one heartbeat later) does
    not fit the CLI's u16 latency stream: gossipsim-node re-delivers the run as
    completion times and writes the whole log, equal to the oracle's."""
    import subprocess
    exe = os.path.join(os.path.dirname(gossipsim.LIB_PATH), "gossipsim-node")
    hb = 70_000_000_000
    t0 = (946684800 + 500) * 1_000_000_000
    phase = t0 - 10 * hb + 20_000_000_000
    env = dict(os.environ, PEERS="300", CONNECTTO="10", FRAGMENTS="1", GS_SEED="5", GS_CHURN_PPM="150000",
               GS_CHURN_DOWN="1", GS_CHURN_HORIZON="4", GOSSIPSUB_HEARTBEAT_MS=str(hb // 1_000_000),
               GS_HB_PHASE_NS=str(phase), GS_LAZY_GOSSIP="1")
    subprocess.run([exe, "-st", "5", "-bl", "50", "-bh", "150", "-ll", "40", "-lh", "130", "-m", "6", "-s", "15000",
                    "--latencies", str(tmp_path / "a")], env=env, check=True, timeout=120)
    p = oracle.params(peers=300, seed=5, churn_ppm=150000, churn_down=1, churn_horizon=4, heartbeat_ns=hb,
                      hb_phase_ns=phase, lazy_gossip=1)
    sched = gossipsim.schedule_runsh(6, 300, 6, 1, t0 + gossipsim.HTTP_TRANSIT_NS, 1_000_000_000, 15000)
    cols = (np.array([r.t_pub_ns for r in sched], dtype=np.uint64), np.array([r.publisher for r in sched]),
            np.array([r.msg_size for r in sched]))
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=cols)
    sim = gossipsim.Simulator(**_knobs(p))
    sim.write_latency_log(str(tmp_path / "b"), {"schedule": sched, "t_complete": ref["t_complete"]})
    a = open(str(tmp_path / "a")).read().splitlines()
    assert sorted(a) == sorted(open(str(tmp_path / "b")).read().splitlines())
    assert max(int(x.rsplit(" ", 1)[1]) for x in a) >= 65535


def test_fragment_collision_defect_d8():
    p = oracle.params(peers=100, fragments=4)
    sim, res = compare(p, 1, (50, 50, 50, 50), _sched(2, 100, size=40))
    assert sim.stats()["deliveries"] == 0


def test_errors_are_reported_not_hidden():
    sim = gossipsim.Simulator(peers=100)
    with pytest.raises(gossipsim.GossipSimError, match="GS_ESTATE"):
        sim.run(_sched(1, 100))
    sim.set_topogen_links()
    sim.connect_gossipsub_peers()
    sim.mesh_converge()
    with pytest.raises(gossipsim.GossipSimError, match="GS_EINVAL"):
        sim.run((np.array([T0], np.uint64), np.array([100]), np.array([15000])))
    with pytest.raises(gossipsim.GossipSimError, match="8-byte"):
        sim.run((np.array([T0], np.uint64), np.array([1]), np.array([7])))
    with pytest.raises(gossipsim.GossipSimError):
        gossipsim.Simulator(peers=10, connect_to=10)  # env.rs:73-75


def test_large_graph_properties_and_sampled_parity():
    """100k peers, one 64-message batch: structure invariants + 2 messages vs the oracle."""
    N = 100_000
    p = oracle.params(peers=N, seed=21)
    sim, ep = gpu_sim(p, 5, (50, 150, 40, 130), batch=64)
    row, col, flags = sim.csr()
    mesh, cnt = sim.mesh()
    deg = np.diff(row.astype(np.int64))
    assert deg.min() >= 11 and (flags & 1).reshape(-1).sum() == 11 * N
    assert cnt.min() >= p.d_lo and cnt.max() <= p.d_hi
    sched = _sched(64, N)
    res = sim.run(sched)
    st = sim.stats()
    assert st["deliveries"] == 64 * (N - 1)  # connected mesh: everyone completes
    assert (res["hops"][res["t_complete"] != UND] < 63).all()
    # oracle on the GPU's own graph for 2 of the 64 messages
    lat, bw = oracle.topogen_links(5, 50, 150, 40, 130)
    stage = (np.arange(N) % 5).astype(np.uint8)
    for m in (0, 37):
        tc, hp, _ = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, sched[0][m:m + 1],
                               sched[1][m:m + 1], sched[2][m:m + 1])
        np.testing.assert_array_equal(res["t_complete"][m], tc[0])
        np.testing.assert_array_equal(res["hops"][m], hp[0])


@pytest.mark.parametrize("variant", list(range(8)) + [8, 9, 10, 11, 13, 15, 45, 109, 237])
def test_relax_kernel_variants_exact(variant, monkeypatch):
    """Every bucket implementation (fused with read-filter / tile-skip / final-bitset,
    split scan+frontier, owner-computes pull over dense rows = 45, over candidate
    lists = 109, the default, and 237 = lists for fragmented batches too) is bit-exact."""
    monkeypatch.setenv("GS_RELAX_VARIANT", str(variant))
    if variant & 64:
        monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    # lazy gossip off: a wrong eager result must not hide behind the push-path
    # fallback that a failed gossip no-op proof takes
    p = oracle.params(peers=2000, seed=31, fragments=2, lazy_gossip=0)
    compare(p, 5, (50, 150, 40, 130), _sched(40, 2000), batch=16)
    p = oracle.params(peers=3000, seed=32, lazy_gossip=0)
    compare(p, 3, (20, 200, 10, 90), _sched(70, 3000), batch=64)


@pytest.mark.parametrize("variant,frags", [(45, 1), (109, 1), (237, 2), (237, 4)])
def test_pull_wide_rows_exact(variant, frags, monkeypatch):
    """Rows of 1024 lanes (16 chunks of 64, the bench layout) on both pull
    kernels: every chunk of a row is live in the peak windows, candidate lists
    span several destination windows, more than 64 lanes per row pend at once."""
    monkeypatch.setenv("GS_RELAX_VARIANT", str(variant))
    if variant & 64:
        monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    B = 1024 // frags
    p = oracle.params(peers=2500, seed=33, fragments=frags, lazy_gossip=0)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(B, 2500), batch=B)
    assert sim.stats()["gossip_fallback_batches"] == 0


def test_pull_list_overflow_reruns_on_dense_rows(monkeypatch):
    """Candidate lists capped at 2 entries (GS_LPULL_CAP): the list pull path
    overflows, restores the counters and re-runs the batch on k_pull; the
    result is still bit-exact."""
    monkeypatch.setenv("GS_LPULL_CAP", "2")
    p = oracle.params(peers=2500, seed=34, lazy_gossip=0)
    compare(p, 5, (50, 150, 40, 130), _sched(256, 2500), batch=256)


def test_pull_list_overflow_counts_past_stride(monkeypatch):
    """Capacity 1 with 1024-lane rows and publishers up to the last peer: list
    lengths run far past the capacity (and can pass the list stride); the pass
    reads only the entries that were written (no read past the row's list or
    the last slot), flags the overflow and the batch re-runs on k_pull."""
    monkeypatch.setenv("GS_LPULL_CAP", "1")
    N = 1200
    p = oracle.params(peers=N, seed=35, lazy_gossip=0)
    t, _, size = _sched(1024, N)
    pub = (N - 1 - np.arange(1024) % 7).astype(np.int64)  # 7 publishers at the top of the id range
    sim, _ = compare(p, 5, (50, 150, 40, 130), (t, pub, size), batch=1024)
    assert sim.stats()["list_pull_batches"] == 0  # every batch went to k_pull


def test_pull_ring_violation_reruns_on_dense_rows(monkeypatch):
    """A ring of K = 2 destination windows (GS_LPULL_K), below the host bound:
    candidates land beyond the ring, the pass flags ERR_RING (not the
    time-overflow error) and the batch re-runs on k_pull, bit-exact."""
    monkeypatch.setenv("GS_LPULL_K", "2")
    p = oracle.params(peers=1500, seed=36, lazy_gossip=0)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(128, 1500), batch=128)
    assert sim.stats()["list_pull_batches"] == 0


@pytest.mark.parametrize("frags,gossip,fast,idw", [(1, 0, 0, 0), (2, 0, 0, 0), (1, 1, 0, 0), (1, 0, 1, 0),
                                                   (1, 1, 1, 0), (2, 1, 1, 0), (1, 0, 1, 1)])
def test_churn_time_varying_mesh(frags, gossip, fast, idw):
    """Churn (config #3 semantics) at small size: the device's
    per-epoch snapshot ring (advanced from the converged state, or replayed from
    epoch 0), offline peers, lost deliveries and the message lifetime, with and
    without lazy gossip / IDONTWANT; bit-exact against the oracle."""
    kw = dict(churn_ppm=20000, lazy_gossip=gossip, fragments=frags, idontwant=1000 if idw else 0)
    if fast:  # 100 ms heartbeats from T0 - 2 s: several epochs per dissemination, replay from epoch 0
        kw.update(heartbeat_ns=100_000_000, hb_phase_ns=T0 - 2_000_000_000 + 37_000_000, churn_down=8,
                  churn_horizon=12)
    else:  # heartbeat 0 at the Shadow process start: publishes at epoch ~495, ring advanced from epoch 400
        kw.update(hb_phase_ns=gossipsim.SHADOW_START_NS)
    p = oracle.params(peers=700, seed=51, **kw)
    sim, res = compare(p, 5, (50, 150, 40, 130), _sched(24, 700), batch=8)
    st = sim.stats()
    assert 0 < st["deliveries"] < 24 * 699  # churn loses deliveries
    if gossip:
        assert st["gossip_iwant"] > 0


@pytest.mark.parametrize("switch", ["0", "1", "3", "1000"])
def test_churn_gossip_sender_receiver_switch(monkeypatch, switch):
    """Lazy gossip under churn decides a message's heartbeats k < GS_GOSSIP_SWITCH
    receiver-centric (inverse IHAVE lists, undelivered lanes) and the later ones
    sender-centric (holders within their history window): every split point,
    from all-sender (0) to all-receiver (1000), is bit-exact against the oracle,
    IWANT count included."""
    monkeypatch.setenv("GS_GOSSIP_SWITCH", switch)
    kw = dict(churn_ppm=20000, lazy_gossip=1, heartbeat_ns=100_000_000, hb_phase_ns=T0 - 2_000_000_000 + 37_000_000,
              churn_down=8, churn_horizon=12)
    p = oracle.params(peers=800, seed=52, **kw)
    sim, res = compare(p, 5, (50, 150, 40, 130), _sched(32, 800), batch=32)
    st = sim.stats()
    assert 0 < st["deliveries"] < 32 * 799 and st["gossip_iwant"] > 0


@pytest.mark.parametrize("gossip,hb_ms,phase_ms,frags,switch", [(0, 1000, 370, 1, 3), (1, 1000, 370, 1, 3), (1, 1000, 370, 1, 0), (1, 1000, 370, 1, 1000), (1, 400, 150, 1, 3), (1, 400, 150, 1, 1),
                                                                  (0, 400, 330, 1, 3), (1, 300, 20, 1, 3),
                                                                  (1, 400, 150, 2, 3), (0, 1000, 370, 2, 3),
                                                                  (1, 1000, 370, 3, 3), (1, 400, 150, 8, 3)])
def test_churn_list_pass(monkeypatch, gossip, hb_ms, phase_ms, frags, switch):
    """Churn on the owner-computes list pass (gs_cpull.h, k_lpull<.., CHN>):
    per-lane epoch meshes as CSR masks, 16-B records, forwards that cross an
    epoch boundary into a receiver's offline epoch, IWANT answers lost the same
    way, the lifetime cut; heartbeats short enough that several boundaries fall
    inside a dissemination; heartbeats from GS_GOSSIP_SWITCH on may push their
    IHAVEs into the targets' lists (1000: none). Bit-exact against the
    oracle, IWANTs included; every batch must take the list pass
    (GS_REQUIRE_LPULL), fragmented ones as rows of fragment groups (F = 2, 3
    in groups of 4 lanes, 8)."""
    monkeypatch.setenv("GS_GOSSIP_SWITCH", str(switch))
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    hb = hb_ms * 1_000_000
    kw = dict(churn_ppm=30000, lazy_gossip=gossip, fragments=frags, heartbeat_ns=hb, churn_down=6,
              churn_horizon=10, hb_phase_ns=T0 - 30 * hb + phase_ms * 1_000_000)
    p = oracle.params(peers=900, seed=57, **kw)
    t = T0 + np.arange(40, dtype=np.uint64) * np.uint64(hb)  # lockstep: one publish per heartbeat
    sched = (t, (6 + np.arange(40)) % 900, np.full(40, 15000))
    sim, res = compare(p, 5, (50, 150, 40, 130), sched, batch=40)
    st = sim.stats()
    assert 0 < st["deliveries"] < 40 * 899
    assert st["list_pull_batches"] == 1
    if gossip:
        assert st["gossip_list_batches"] == 1 and st["gossip_iwant"] > 0


def test_churn_list_pass_equals_push_path_at_10k(monkeypatch):
    """The churn list pass against the push path on a 10k-peer, 256-message
    config #3-shaped batch (heterogeneous links, lazy gossip, 1 % churn,
    heartbeats 370 ms after each publish): every completion time, hop count and
    counter equal."""
    p = oracle.params(peers=10_000, seed=3, lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                      hb_phase_ns=T0 - 20 * 1_000_000_000 + 370_000_000)
    sched = _sched(256, 10_000)
    out = []
    for chl in ("1", "0"):
        monkeypatch.setenv("GS_CHURN_LIST", chl)
        sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=256)
        res = sim.run(sched)
        out.append((res, sim.stats()))
        sim.close()
    (a, sa), (b, sb) = out
    assert sa["list_pull_batches"] == 1 and sb["list_pull_batches"] == 0
    np.testing.assert_array_equal(a["t_complete"], b["t_complete"])
    np.testing.assert_array_equal(a["hops"], b["hops"])
    for k in ("deliveries", "frag_deliveries", "relaxations", "gossip_iwant", "latency_sum_ms"):
        assert sa[k] == sb[k], k
    assert sa["gossip_iwant"] > 0


def test_churn_errors():
    p = oracle.params(peers=200, seed=3, churn_ppm=10000)  # hb_phase 0: publishes ~1e9 heartbeats later
    sim, _ = gpu_sim(p, 1, (50, 50, 50, 50))
    with pytest.raises(gossipsim.GossipSimError, match="2\\^20 heartbeats"):
        sim.run(_sched(2, 200))


@pytest.mark.parametrize("connect_to", [20, 30])
def test_churn_gossip_wide_target_lists(connect_to):
    """Lazy gossip under churn where many peers have more IHAVE targets than the
    per-epoch precomputed list holds (GT_W = 8; degree ~2*CONNECTTO, targets =
    max(d_lazy, gossip_factor * candidates)): those peers take k_gossip's own
    selection (GT_NONE), the rest the k_gossip_targets list; both bit-exact
    against the oracle."""
    kw = dict(churn_ppm=20000, lazy_gossip=1, connect_to=connect_to, heartbeat_ns=100_000_000,
              hb_phase_ns=T0 - 2_000_000_000 + 37_000_000, churn_down=8, churn_horizon=12)
    p = oracle.params(peers=500, seed=61, **kw)
    sim, res = compare(p, 5, (50, 150, 40, 130), _sched(16, 500), batch=8)
    st = sim.stats()
    assert 0 < st["deliveries"] < 16 * 499
    assert st["gossip_iwant"] > 0


@pytest.mark.parametrize("second", ["bigmsg", "idontwant"])
def test_churn_push_batch_after_list_pass_batch(monkeypatch, second):
    """a churn batch on the list pass skips the ELL snapshots and
    inverse IHAVE lists of its epochs; the next batch, on the push path (2 MB
    messages, whose uplink serialisation outlasts a heartbeat, or an
    IDONTWANT-sized payload), overlaps its last epochs and must find them
    rebuilt. Bit-exact against the oracle, IWANTs included."""
    hb = 400_000_000
    kw = dict(churn_ppm=30000, lazy_gossip=1, heartbeat_ns=hb, churn_down=6, churn_horizon=10,
              hb_phase_ns=T0 - 30 * hb + 150_000_000)
    if second == "idontwant":
        kw["idontwant"] = 1000
    p = oracle.params(peers=900, seed=57, **kw)
    M1, M2 = 40, 16
    t = T0 + np.arange(M1 + M2, dtype=np.uint64) * np.uint64(hb)
    pub = (6 + np.arange(M1 + M2)) % 900
    if second == "bigmsg":
        size, frags = np.r_[np.full(M1, 15000), np.full(M2, 2_000_000)], np.ones(M1 + M2, np.uint32)
    else:  # first batch under the IDONTWANT threshold (list pass), second above it (push path)
        size, frags = np.r_[np.full(M1, 500), np.full(M2, 15000)], np.ones(M1 + M2, np.uint32)
    sim, res = compare(p, 5, (50, 150, 40, 130), (t, pub, size, frags), batch=64)
    st = sim.stats()
    assert st["batches"] == 2 and st["list_pull_batches"] == 1
    assert st["gossip_iwant"] > 0


def test_churn_links_changed_between_runs():
    """new links on the same topology invalidate the churn list
    pass's 64-wide CSR rows (stage << 24 | peer): a second run after
    set_links + mesh_converge equals a fresh oracle run on the new links."""
    hb = 400_000_000
    kw = dict(churn_ppm=30000, lazy_gossip=1, heartbeat_ns=hb, churn_down=6, churn_horizon=10,
              hb_phase_ns=T0 - 30 * hb + 150_000_000)
    p = oracle.params(peers=900, seed=58, **kw)
    t = T0 + np.arange(32, dtype=np.uint64) * np.uint64(hb)
    sched = (t, (6 + np.arange(32)) % 900, np.full(32, 15000))
    links_a, links_b = (50, 150, 40, 130), (30, 100, 30, 120)
    sim, _ = gpu_sim(p, 5, links_a, batch=32)
    sim.run(sched)
    assert sim.stats()["list_pull_batches"] == 1
    sim.set_topogen_links(3, *links_b)
    ep = sim.mesh_converge(400)
    sim.reset_stats()
    res = sim.run(sched)
    ref = oracle.simulate(p, 3, links_b, sched=sched)
    assert ep == ref["epochs"]
    np.testing.assert_array_equal(res["t_complete"], ref["t_complete"], err_msg="t_complete")
    np.testing.assert_array_equal(res["hops"], ref["hops"], err_msg="hops")
    st = sim.stats()
    assert st["list_pull_batches"] == 1
    for k in ("deliveries", "relaxations", "gossip_iwant", "latency_sum_ms"):
        assert st[k] == ref["stats"][k], k


@pytest.mark.parametrize("gossip,pipe", [(1, "1"), (0, "1"), (1, "0")])
def test_churn_list_pass_chain_ahead(monkeypatch, gossip, pipe):
    """Churn batches back to back on the list pass: with GS_CHN_PIPE on (the
    default on a 256-CU MI355X), batch k+1's epoch chain and tables are
    enqueued on the chain's XCD while batch k's passes run on the others
    (gs_relax.hip ChnAhead). Bit-exact against the oracle over 4 batches."""
    monkeypatch.setenv("GS_CHN_PIPE", pipe)
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    hb = 400_000_000
    kw = dict(churn_ppm=30000, lazy_gossip=gossip, heartbeat_ns=hb, churn_down=6, churn_horizon=10,
              hb_phase_ns=T0 - 30 * hb + 150_000_000)
    p = oracle.params(peers=900, seed=59, **kw)
    M = 160
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(hb)
    sched = (t, (6 + np.arange(M)) % 900, np.full(M, 15000))
    sim, res = compare(p, 5, (50, 150, 40, 130), sched, batch=40)
    st = sim.stats()
    assert st["batches"] == 4 and st["list_pull_batches"] == 4
    if gossip:
        assert st["gossip_iwant"] > 0


def test_churn_chain_ahead_then_push_fallback(monkeypatch):
    """A batch whose candidate lists overflow falls back to the push path after
    the next batch's chain already ran ahead (overwriting ring slots): it joins
    that chain, churn_ring replays its ring slots, and every batch stays
    bit-exact against the oracle."""
    monkeypatch.setenv("GS_LPULL_CAP", "3")
    hb = 400_000_000
    kw = dict(churn_ppm=30000, lazy_gossip=1, heartbeat_ns=hb, churn_down=6, churn_horizon=10,
              hb_phase_ns=T0 - 30 * hb + 150_000_000)
    p = oracle.params(peers=900, seed=60, **kw)
    M = 120
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(hb)
    sched = (t, (6 + np.arange(M)) % 900, np.full(M, 15000))
    sim, res = compare(p, 5, (50, 150, 40, 130), sched, batch=40)
    st = sim.stats()
    assert st["batches"] == 3 and st["list_pull_batches"] < 3


def _nonlockstep_check(sim, st_expect_batches=None):
    st = sim.stats()
    # every batch on the list pass: GS_REQUIRE_LPULL fails any push-path batch; a batch
    # whose eager pass failed the gossip no-op proof counts twice (the re-run in-pass)
    assert st["list_pull_batches"] >= st["batches"], st
    if st_expect_batches is not None:
        assert st["batches"] == st_expect_batches, st
    return st


def test_nonlockstep_delay_1500ms_gossip_on_list_pass(monkeypatch):
    """run.sh's free message_delay (run.sh:36) at 1500 ms: publishes alternate
    between two offsets into the heartbeat (+120 ms and +620 ms here), so no
    batch is lockstep. The run regroups each batch's messages by offset class
    (gs_relax.hip class_plan): one lockstep batch per class, IHAVE / IWANT
    inside the list pass, results back in schedule order; bit-exact against
    the oracle, IWANTs included, and no batch on the push path."""
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    p = oracle.params(peers=1500, seed=81, hb_phase_ns=(T0 + 120_000_000) % 1_000_000_000)
    M = 48
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(1_500_000_000)
    sched = (t, (6 + np.arange(M)) % 1500, np.full(M, 15000))
    sim, res = compare(p, 5, (50, 150, 40, 130), sched, batch=64)
    st = _nonlockstep_check(sim, 2)
    assert st["gossip_iwant"] > 0 and st["gossip_list_batches"] >= 1


def test_nonlockstep_random_schedule_file_gossip(tmp_path, monkeypatch):
    """An arbitrary POST /publish sequence (main.rs:146-221) read from a
    schedule file (gs_read_schedule): random publish times at 1 ms grain,
    random publishers, every message its own offset class; each runs as a
    lockstep list-pass batch with the gossip inside the passes; bit-exact
    against the oracle and never on the push path."""
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    rng = np.random.default_rng(5)
    M, N = 24, 1200
    t = np.sort(T0 + rng.integers(0, 30_000, M).astype(np.uint64) * np.uint64(1_000_000))
    pub = rng.integers(0, N, M)
    f = tmp_path / "sched.txt"
    f.write_text("".join("%d %d %d\n" % (int(a), int(b), 15000) for a, b in zip(t, pub)))
    arr = np.ctypeslib.as_array(gossipsim.read_schedule(str(f)))
    np.testing.assert_array_equal(arr["t_pub_ns"], t)
    np.testing.assert_array_equal(arr["publisher"], pub)
    sched = (arr["t_pub_ns"].copy(), arr["publisher"].astype(np.int64), arr["msg_size"].astype(np.int64))
    p = oracle.params(peers=N, seed=82, hb_phase_ns=(T0 + 120_000_000) % 1_000_000_000)
    sim, res = compare(p, 5, (50, 150, 40, 130), sched, batch=64)
    st = _nonlockstep_check(sim)
    assert st["batches"] == len(set(int(x) % 1_000_000_000 for x in t))


@pytest.mark.parametrize("gossip", [1, 0])
def test_nonlockstep_churn_delay_on_list_pass(monkeypatch, gossip):
    """Churn with publishes 1.5 heartbeats apart: two offsets into the epoch,
    regrouped into one churn list-pass batch each (the ring holds the batch's
    epochs for both; the second batch's tables come from the ring). Bit-exact
    against the oracle, no push-path batch."""
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    hb = 400_000_000
    kw = dict(churn_ppm=30000, lazy_gossip=gossip, heartbeat_ns=hb, churn_down=6, churn_horizon=10,
              hb_phase_ns=T0 - 30 * hb + 150_000_000)
    p = oracle.params(peers=900, seed=83, **kw)
    M = 40
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(600_000_000)
    sched = (t, (6 + np.arange(M)) % 900, np.full(M, 15000))
    sim, res = compare(p, 5, (50, 150, 40, 130), sched, batch=64)
    st = _nonlockstep_check(sim, 2)
    assert 0 < st["deliveries"] < M * 899
    if gossip:
        assert st["gossip_iwant"] > 0
