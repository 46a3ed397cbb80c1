"""GPU runs at BASELINE.json's full config sizes (configs #2, #3, #4; config #1
is tests/test_gpu_parity.py::test_config1_1k_peers_100_publishes).

At these sizes the whole oracle run would take minutes, so each test checks
size-independent properties (every peer completes on a connected mesh, the
publisher's own row, hop bounds, message sharding = the whole run, peer
partition = one device) and a sample of messages bit-exact against the CPU
oracle run on the GPU's own graph and mesh."""
import numpy as np
import pytest

import gossipsim
import oracle
import partition

pytestmark = pytest.mark.gpu
T0 = gossipsim.T0_NS
UND = np.iinfo(np.uint64).max
LINKS = (50, 150, 40, 130)  # run.sh / shadow/README.md example: 5 stages, 50-150 Mbit, 40-130 ms


def _sched(M, N, size=15000, pub0=6):
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
    return t, (pub0 + np.arange(M)) % N, np.full(M, size)


def _sim(p, S, links, batch):
    kw = {n: getattr(p, n) for n, _ in oracle.OrParams._fields_}
    kw["batch"] = batch
    sim = gossipsim.Simulator(**kw)
    sim.set_topogen_links(S, *links)
    sim.connect_gossipsub_peers()
    sim.mesh_converge()
    return sim


def _links(p, S, links):
    lat, bw = oracle.topogen_links(S, *links)
    return lat, bw, (np.arange(p.peers) % S).astype(np.uint8)


def _sub(sched, idx):
    return tuple(np.asarray(x)[idx] for x in sched)


def _publisher_rows(res, sched):
    M = len(sched[0])
    np.testing.assert_array_equal(res["t_complete"][np.arange(M), sched[1]], sched[0])
    assert (res["hops"][np.arange(M), sched[1]] == 0).all()


def test_config2_10k_peers_f8_1000_msgs():
    """Config #2: 10k peers, FRAGMENTS=8 (1875 B fragments), 1000 messages, 5-stage links."""
    N, M, S = 10_000, 1000, 5
    p = oracle.params(peers=N, seed=2, fragments=8)
    sched = _sched(M, N)
    sim = _sim(p, S, LINKS, batch=128)
    res = sim.run(sched)
    st = sim.stats()
    assert st["deliveries"] == M * (N - 1) and st["frag_deliveries"] == 8 * M * (N - 1)
    tc, hp = res["t_complete"], res["hops"]
    assert (tc >= sched[0][:, None]).all() and (hp < 63).all()
    _publisher_rows(res, sched)
    lat_ms = (tc - sched[0][:, None]) // 1_000_000
    assert st["latency_sum_ms"] == int(lat_ms.sum()) and st["latency_max_ms"] == int(lat_ms.max())
    # sampled parity against the oracle on the GPU's graph and mesh
    row, col, _ = sim.csr()
    mesh, cnt = sim.mesh()
    lat, bw, stage = _links(p, S, LINKS)
    idx = np.linspace(0, M - 1, 17).astype(int)  # 17 messages spread over all 8 batches
    otc, ohp, _ = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, *_sub(sched, idx))
    np.testing.assert_array_equal(tc[idx], otc)
    np.testing.assert_array_equal(hp[idx], ohp)
    # message sharding (bench.py --gpus N): shards on fresh contexts == the whole run
    for lo, hi in ((0, 384), (384, M)):
        r2 = _sim(p, S, LINKS, batch=128).run(_sub(sched, slice(lo, hi)))
        np.testing.assert_array_equal(r2["t_complete"], tc[lo:hi])
        np.testing.assert_array_equal(r2["hops"], hp[lo:hi])


def test_config3_100k_hetero_gossip_churn():
    """Config #3: 100k peers, heterogeneous topogen links, lazy IHAVE/IWANT and
    churn (1 % of peers start a 10-heartbeat outage every heartbeat), 1000 msgs."""
    N, M, S = 100_000, 1000, 5
    hb = 1_000_000_000
    p = oracle.params(peers=N, seed=3, lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                      heartbeat_ns=hb, hb_phase_ns=T0 - 20 * hb + 370_000_000)
    sched = _sched(M, N)
    sim = _sim(p, S, LINKS, batch=64)
    res = sim.run(sched)
    st = sim.stats()
    tc, hp = res["t_complete"], res["hops"]
    got = tc != UND
    assert 0.5 * M * (N - 1) < st["deliveries"] < M * (N - 1)  # churn loses deliveries, most still arrive
    assert st["gossip_iwant"] > 0
    assert (hp[got] < 63).all() and ((tc >= sched[0][:, None]) | ~got).all()
    # nothing arrives past the message lifetime (epoch of t_pub + horizon)
    ep_pub = (sched[0] - np.uint64(p.hb_phase_ns)) // np.uint64(hb)
    limit = np.uint64(p.hb_phase_ns) + (ep_pub + np.uint64(p.churn_horizon + 1)) * np.uint64(hb)
    assert (tc[got] < np.broadcast_to(limit[:, None], tc.shape)[got]).all()
    # sampled parity: the oracle replays churn from epoch 0 on the GPU's graph;
    # 16 messages from the first two 64-message batches, half of them after the
    # first ring advance
    row, col, flags = sim.csr()
    lat, bw, stage = _links(p, S, LINKS)
    idx = np.array([0, 1, 9, 17, 30, 41, 55, 63, 64, 65, 77, 88, 99, 110, 121, 127])
    t, pub, size = _sub(sched, idx)
    h_lo = min(oracle.epoch_at(p, x) for x in t)
    h_hi = max(oracle.epoch_at(p, x) for x in t) + p.churn_horizon
    snaps = oracle.mesh_churn(p, row, col, (flags & 1).astype(np.uint8), stage, lat, h_lo, h_hi)
    otc, ohp, ost = oracle.run_churn(p, row, col, snaps, h_lo, stage, lat, bw, bw, t, pub, size)
    np.testing.assert_array_equal(tc[idx], otc)
    np.testing.assert_array_equal(hp[idx], ohp)
    del snaps
    # message sharding under churn: a fresh context on a later shard reproduces it
    r2 = _sim(p, S, LINKS, batch=64).run(_sub(sched, slice(600, 700)))
    np.testing.assert_array_equal(r2["t_complete"], tc[600:700])
    np.testing.assert_array_equal(r2["hops"], hp[600:700])


def _oracle_churn_sample(p, sim, S, links, sched, idx, threads=8):
    """The oracle on sampled messages of a churn run, on the GPU's graph: one
    churn replay from epoch 0 keeping only the epochs the sample needs
    (oracle.mesh_churn_ranges), then oracle.run_churn per group of messages
    whose lifetimes overlap, groups on parallel host threads."""
    from concurrent.futures import ThreadPoolExecutor
    row, col, flags = sim.csr()
    lat, bw, stage = _links(p, S, links)
    t, pub, size = _sub(sched, idx)
    ep = np.array([oracle.epoch_at(p, x) for x in t])
    groups = []  # (h_lo, h_hi, positions in idx)
    for k in np.argsort(ep, kind="stable"):
        lo, hi = int(ep[k]), int(ep[k]) + p.churn_horizon
        if groups and lo <= groups[-1][1]:
            groups[-1][1] = max(groups[-1][1], hi)
            groups[-1][2].append(k)
        else:
            groups.append([lo, hi, [k]])
    snaps = oracle.mesh_churn_ranges(p, row, col, (flags & 1).astype(np.uint8), stage, lat,
                                     [(g[0], g[1]) for g in groups], threads=threads)

    def one(g):
        ks = np.array(g[2])
        return ks, oracle.run_churn(p, row, col, snaps[(g[0], g[1])], g[0], stage, lat, bw, bw,
                                    t[ks], pub[ks], size[ks])

    otc = np.zeros((len(idx), p.peers), np.uint64)
    ohp = np.zeros((len(idx), p.peers), np.uint8)
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for ks, (tc, hp, _) in ex.map(one, groups):
            otc[ks], ohp[ks] = tc, hp
    return otc, ohp


@pytest.mark.timeout(900)
def test_config3_bench_shape_batch1024_spread_sample():
    """Config #3 at the shape bench.py times it (configs_1gpu.c3_100k_gossip_churn:
    100k peers, 5-stage topogen links, lazy gossip, 1 % churn, the messages in
    ONE batch of up to 1024): 18 messages spread over all 1000 (6 of them at
    index >= 600, incl. the last two) bit-exact against the oracle, which
    replays churn from epoch 0 on the GPU's graph."""
    N, M, S = 100_000, 1000, 5
    hb = 1_000_000_000
    p = oracle.params(peers=N, seed=3, lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                      heartbeat_ns=hb, hb_phase_ns=T0 - 20 * hb + 370_000_000)
    sched = _sched(M, N)
    sim = _sim(p, S, LINKS, batch=1024)
    res = sim.run(sched)
    st = sim.stats()
    assert st["batches"] == 1 and st["gossip_iwant"] > 0
    assert 0.5 * M * (N - 1) < st["deliveries"] < M * (N - 1)
    idx = np.array([0, 1, 57, 130, 131, 250, 333, 402, 499, 555, 600, 601, 689, 777, 850, 912, 998, 999])
    assert len(idx) >= 16 and (idx >= 600).sum() >= 4
    otc, ohp = _oracle_churn_sample(p, sim, S, LINKS, sched, idx)
    np.testing.assert_array_equal(res["t_complete"][idx], otc)
    np.testing.assert_array_equal(res["hops"][idx], ohp)


@pytest.mark.timeout(900)
def test_config4_1m_peers_c_abi_p8_loopback():
    """Config #4's split through the C ABI: gs_run_partitioned over
    gs_comm_init_local(8) (eight parts of 125k peers on this GPU, records
    routed per bucket to the parts owning a target) at 1M peers == gs_run on
    one context == the oracle on 4 of the 8 messages."""
    N, S, M = 1_000_000, 5, 8
    p = oracle.params(peers=N, seed=41)
    sched = _sched(M, N)
    whole = _sim(p, S, LINKS, batch=M)
    ref = whole.run(sched)
    assert whole.stats()["deliveries"] == M * (N - 1)
    row, col, _ = whole.csr()
    mesh, cnt = whole.mesh()
    whole.close()
    sims = [_sim(p, S, LINKS, batch=M) for _ in range(8)]
    for i, s in enumerate(sims):
        s.set_partition(8, i)
    comm = gossipsim.Comm(local_parts=8)
    res = comm.run_partitioned(sims, sched)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ref["t_complete"])
    np.testing.assert_array_equal(np.concatenate([r["hops"] for r in res], axis=1), ref["hops"])
    assert sum(s.stats()["deliveries"] for s in sims) == M * (N - 1)
    comm.close()
    for s in sims:
        s.close()
    lat, bw, stage = _links(p, S, LINKS)
    idx = np.array([0, 2, 5, 7])
    otc, ohp, _ = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, *_sub(sched, idx), threads=4)
    np.testing.assert_array_equal(ref["t_complete"][idx], otc)
    np.testing.assert_array_equal(ref["hops"][idx], ohp)


def test_config4_1m_peers_peer_partitioned():
    """Config #4 at 1M peers: peers partitioned over 2 contexts exchanging each
    window's records (loop-back all-gather, the same protocol as RCCL across
    GPUs) == one device == the oracle on a sampled message."""
    import torch
    N, S, M = 1_000_000, 5, 8
    p = oracle.params(peers=N, seed=4)
    sched = _sched(M, N)
    whole = _sim(p, S, LINKS, batch=M)
    ref = whole.run(sched)
    _publisher_rows(ref, sched)
    assert whole.stats()["deliveries"] == M * (N - 1)
    sims = [_sim(p, S, LINKS, batch=M) for _ in range(2)]
    for i, s in enumerate(sims):
        s.set_partition(2, i)
    bufs = [partition.RecordBuffer(torch.device("cuda", 0), capacity=1 << 22) for _ in sims]
    res, info = partition.run_partitioned(sims, sched, partition.LoopbackExchange(), bufs=bufs)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ref["t_complete"])
    np.testing.assert_array_equal(np.concatenate([r["hops"] for r in res], axis=1), ref["hops"])
    assert sum(s.stats()["deliveries"] for s in sims) == M * (N - 1)
    row, col, _ = whole.csr()
    mesh, cnt = whole.mesh()
    lat, bw, stage = _links(p, S, LINKS)
    idx = np.array([0, 3, 5, 7])
    otc, ohp, _ = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, *_sub(sched, idx))
    np.testing.assert_array_equal(ref["t_complete"][idx], otc)
    np.testing.assert_array_equal(ref["hops"][idx], ohp)


def test_config3_small_ring_cuts_batches(monkeypatch):
    """Churn + lazy gossip with a snapshot ring too small for the batch
    (GS_RING_BUDGET_MB): gs_run cuts batches at the ring size and advances the
    ring between them (incl. the IHAVE target lists); bit-exact against the
    oracle on every message."""
    monkeypatch.setenv("GS_RING_BUDGET_MB", "1")
    N, M, S = 700, 40, 5
    hb = 100_000_000
    p = oracle.params(peers=N, seed=33, lazy_gossip=1, churn_ppm=20000, churn_down=8, churn_horizon=12,
                      heartbeat_ns=hb, hb_phase_ns=T0 - 2_000_000_000 + 37_000_000)
    sched = _sched(M, N)
    sim = _sim(p, S, LINKS, batch=64)
    res = sim.run(sched)
    ref = oracle.simulate(p, S, LINKS, sched=sched)
    np.testing.assert_array_equal(res["t_complete"], ref["t_complete"])
    np.testing.assert_array_equal(res["hops"], ref["hops"])
    st = sim.stats()
    for k in ("deliveries", "relaxations", "gossip_iwant", "latency_sum_ms"):
        assert st[k] == ref["stats"][k], k


@pytest.mark.parametrize("B", [512, 1024])
def test_list_pull_equals_dense_rows_at_1m(monkeypatch, B):
    """The bench layout at full size (1M peers, rows of 512 lanes — the pass
    with 8 chunks per row and 6 waves per SIMD — and of 1024 lanes — 16
    chunks, the bench's —, 5-stage topogen links): the list pull path (variant
    109) and k_pull over dense rows (45) agree lane for lane. Lazy gossip off so that
    neither result can hide behind the push-path fallback; the completion
    times and hops stream out in blocks of 64 messages and are compared by
    checksums of every block."""
    N = 1_000_000
    p = oracle.params(peers=N, seed=1, lazy_gossip=0)
    sim = _sim(p, 5, LINKS, B)
    sched = _sched(B, N)
    out = {}
    for v in ("45", "109"):
        monkeypatch.setenv("GS_RELAX_VARIANT", v)
        if v == "109":
            monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
        sums = []

        def blk(first, tc, hp):
            t = tc.view(np.uint64)
            w = np.arange(t.size, dtype=np.uint64).reshape(t.shape) * np.uint64(0x9E3779B97F4A7C15)
            sums.append((first, int(np.bitwise_xor.reduce(t, axis=None)), int(np.sum(t * (w | np.uint64(1)))),
                         int(np.sum(hp.astype(np.uint64))), int((t == UND).sum())))

        sim.reset_stats()
        sim.run(sched, on_block=blk, block_msgs=64)
        st = sim.stats()
        assert st["deliveries"] == B * (N - 1)
        out[v] = (sums, st["list_pull_batches"], st["relaxations"])
    assert out["45"][1] == 0 and out["109"][1] >= 1
    assert out["45"][2] == out["109"][2]
    assert out["45"][0] == out["109"][0]
