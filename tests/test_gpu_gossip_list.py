"""Lazy gossip inside the list pass (gs_lpull_kernel.h GOS):
IHAVE / IWANT decided per Delta-window on the device, bit-exact against the
CPU oracle with gossip on — completion times, hops, and the IWANT and
relaxation counts — at small sizes over the knobs that shape gossip, and at
the bench's 1M-peer x 1024-message shape on sampled messages.

Reference: rust-test-node/src/main.rs:228-235 (heartbeat 1 s, gossip_lazy 6,
gossip_factor 0.25); the IHAVE / IWANT rules are libp2p-gossipsub's
emit_gossip / handle_ihave / handle_iwant (upstream, not vendored: parity
with the reference unpinned, the oracle is the restatement of DESIGN.md §2.7)."""
import numpy as np
import pytest

import gossipsim
import oracle
from test_gpu_parity import T0, UND, _sched, compare, gpu_sim

pytestmark = pytest.mark.gpu
LINKS = (50, 150, 40, 130)
HB = 1_000_000_000


def _phase(ms):
    """hb_phase_ns putting a heartbeat `ms` after every publish of _sched."""
    return (T0 + ms * 1_000_000) % HB


@pytest.mark.parametrize("phase_ms", [0, 55, 120, 370, 700])
def test_gossip_in_list_pass_heartbeat_phases(phase_ms):
    """Heartbeats at several offsets after the publishes (mid-dissemination
    ones take IWANTs): every batch keeps its gossip inside the list pass."""
    p = oracle.params(peers=3000, seed=200 + phase_ms, hb_phase_ns=_phase(phase_ms))
    sim, _ = compare(p, 5, LINKS, _sched(48, 3000), batch=16)
    st = sim.stats()
    assert st["gossip_fallback_batches"] <= 1 and st["list_pull_batches"] >= 3
    if phase_ms in (55, 120):
        assert st["gossip_iwant"] > 0 and st["gossip_list_batches"] >= 2


@pytest.mark.parametrize("case", ["hist1", "dlazy3_f500", "uniform_links", "quic_unsigned", "d8", "nim"])
def test_gossip_in_list_pass_knobs(case):
    kw = dict(peers=2500, seed=210, hb_phase_ns=_phase(150))
    S, links = 5, LINKS
    if case == "hist1":
        kw.update(history_gossip=1)
    elif case == "dlazy3_f500":
        kw.update(d_lazy=3, gossip_factor_milli=500)
    elif case == "uniform_links":
        S, links = 1, (50, 50, 50, 50)
    elif case == "quic_unsigned":
        kw.update(muxer=1, signed_msgs=0)
    elif case == "d8":
        kw.update(d=8, d_lo=6, d_hi=12, d_out=2)
    p = oracle.params_for("nim", **kw) if case == "nim" else oracle.params(**kw)
    sim, _ = compare(p, S, links, _sched(24, 2500), batch=8)
    st = sim.stats()
    assert st["gossip_iwant"] > 0 and st["gossip_list_batches"] >= 2


def test_gossip_carries_messages_across_heartbeats():
    """A mesh left empty (no subscription grafting, no heartbeat): only the
    publisher's flood and lazy gossip spread a message, one hop per heartbeat,
    so the passes run IHAVE windows of many heartbeats and the sender planes
    are rebuilt each time; some peers are never reached."""
    N = 1500
    p = oracle.params(peers=N, seed=220, sub_graft=0, hb_phase_ns=_phase(200))
    sched = _sched(6, N)
    sim, _ = gpu_sim(p, 5, LINKS, batch=6, max_hb=0)
    assert (sim.mesh()[1] == 0).all()
    ref = oracle.simulate(p, 5, LINKS, sched=sched, max_hb=0)
    res = sim.run(sched)
    np.testing.assert_array_equal(res["t_complete"], ref["t_complete"])
    np.testing.assert_array_equal(res["hops"], ref["hops"])
    st = sim.stats()
    for k in ("deliveries", "relaxations", "gossip_iwant", "latency_sum_ms", "latency_max_ms"):
        assert st[k] == ref["stats"][k], k
    assert st["gossip_list_batches"] == 1
    assert ref["stats"]["latency_max_ms"] > 2000  # reached over several heartbeats


@pytest.mark.parametrize("path", ["list", "push"])
def test_gossip_list_pass_equals_push_path(monkeypatch, path):
    """The same gossip-active batches on the list pass and, with
    GS_GOSSIP_LIST=0, on the eager pass + push-path fallback: both equal the
    oracle (and so each other)."""
    if path == "push":
        monkeypatch.setenv("GS_GOSSIP_LIST", "0")
    p = oracle.params(peers=2000, seed=93, hb_phase_ns=_phase(0))
    sim, _ = compare(p, 5, LINKS, _sched(24, 2000), batch=8)
    st = sim.stats()
    if path == "list":
        assert st["gossip_fallback_batches"] == 1 and st["gossip_list_batches"] == 3
    else:
        assert st["gossip_fallback_batches"] == 3 and st["gossip_list_batches"] == 0


def test_gossip_not_lockstep_stays_exact():
    """Publishes off the 1 s grid (heartbeats at different offsets per message):
    since round 6 a batch's messages are regrouped by heartbeat-offset class
    into lockstep slices, so the list pass's gossip takes
    them (a slice whose gossip is not a no-op still falls back to the push
    path); bit-exact against the oracle."""
    N, M = 1800, 16
    rs = np.random.default_rng(5)
    t = T0 + np.sort(rs.integers(0, 20 * HB, M)).astype(np.uint64)
    sched = (t, (6 + np.arange(M)) % N, np.full(M, 15000))
    p = oracle.params(peers=N, seed=230, hb_phase_ns=0)
    sim, _ = compare(p, 5, LINKS, sched, batch=8)
    assert sim.stats()["gossip_list_batches"] > 0


def _rows(sim, sched, idx, N):
    """Run the whole schedule with results streamed in 64-message blocks,
    keeping the rows of messages idx (the [M, N] arrays would be 9 GB)."""
    want = {int(i): k for k, i in enumerate(idx)}
    tc = np.zeros((len(idx), N), np.uint64)
    hp = np.zeros((len(idx), N), np.uint8)

    def blk(first, t, h):
        for r in range(t.shape[0]):
            k = want.get(first + r)
            if k is not None:
                tc[k] = t[r]
                hp[k] = h[r]

    sim.run(sched, on_block=blk, block_msgs=64)
    return tc, hp


def _bench_sim(p, B):
    kw = {n: getattr(p, n) for n, _ in oracle.OrParams._fields_}
    sim = gossipsim.Simulator(batch=B, **kw)
    sim.set_topogen_links(5, *LINKS)
    sim.connect_gossipsub_peers()
    sim.mesh_converge()
    return sim


def _oracle_rows(p, sim, sched, idx):
    row, col, _ = sim.csr()
    mesh, cnt = sim.mesh()
    lat, bw = oracle.topogen_links(5, *LINKS)
    stage = (np.arange(p.peers) % 5).astype(np.uint8)
    sub = tuple(np.asarray(x)[idx] for x in sched)
    return oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, *sub, threads=len(idx))


@pytest.mark.timeout(900)
def test_headline_shape_1m_x_1024_lazy_gossip_on(monkeypatch):
    """The bench's headline workload exactly (1M peers, 5-stage topogen links,
    rust preset with lazy gossip on, one batch of 1024 messages, rows of 1024
    lanes: k_lpull<1, 16>): the device proves every IHAVE a no-op, and 4
    messages spread over the batch, the last included, equal the oracle run
    with gossip on (every IHAVE simulated) on the device's graph and mesh."""
    monkeypatch.setenv("GS_REQUIRE_LPULL", "1")
    N, B = 1_000_000, 1024
    p = oracle.params(peers=N, seed=1)
    sim = _bench_sim(p, B)
    sched = gossipsim.shard_messages(0, 0, 1, B, N, 15000)
    sim.run(sched, collect=False)  # the bench's own path: final logs, k_lcomplete
    st0 = sim.stats()
    assert st0["list_pull_batches"] == 1 and st0["gossip_noop_msgs"] == B and st0["gossip_fallback_batches"] == 0
    assert st0["deliveries"] == B * (N - 1)
    sim.reset_stats()
    idx = np.array([0, 341, 682, B - 1])
    tc, hp = _rows(sim, sched, idx, N)
    st = sim.stats()
    for k in ("deliveries", "relaxations", "latency_sum_ms", "latency_max_ms"):
        assert st[k] == st0[k], k
    otc, ohp, ost = _oracle_rows(p, sim, sched, idx)
    assert ost["gossip_iwant"] == 0
    np.testing.assert_array_equal(tc, otc)
    np.testing.assert_array_equal(hp, ohp)
    sim.close()


@pytest.mark.timeout(900)
def test_gossip_active_1m_x_1024_heartbeat_370ms(monkeypatch):
    """The headline graph with heartbeats 370 ms after every publish (mid-
    dissemination: IWANT answers overtake eager forwards): the batch's gossip
    runs inside the list pass (no push-path run), equals the push path lane
    for lane (checksums of every 64-message block), and 3 messages, the last
    included, equal the oracle with gossip on."""
    N, B = 1_000_000, 1024
    p = oracle.params(peers=N, seed=1, hb_phase_ns=(gossipsim.T0_NS + 370_000_000) % HB)
    sim = _bench_sim(p, B)
    sched = gossipsim.shard_messages(0, 0, 1, B, N, 15000)
    idx = np.array([0, 511, B - 1])
    tc, hp = _rows(sim, sched, idx, N)
    st = sim.stats()
    assert st["gossip_list_batches"] == 1 and st["gossip_iwant"] > 0
    otc, ohp, ost = _oracle_rows(p, sim, sched, idx)
    assert ost["gossip_iwant"] > 0
    np.testing.assert_array_equal(tc, otc)
    np.testing.assert_array_equal(hp, ohp)
    # the whole batch against the push path (eager pass, failed proof, gossip on k_scan / k_frontier / k_gossip)
    sums = {}
    for path in ("list", "push"):
        monkeypatch.setenv("GS_GOSSIP_LIST", "1" if path == "list" else "0")
        got = []

        def blk(first, t, h):
            t = t.view(np.uint64)
            w = np.arange(t.size, dtype=np.uint64).reshape(t.shape) * np.uint64(0x9E3779B97F4A7C15)
            got.append((first, int(np.bitwise_xor.reduce(t, axis=None)), int(np.sum(t * (w | np.uint64(1)))),
                        int(np.sum(h.astype(np.uint64)))))

        sim.reset_stats()
        sim.run(sched, on_block=blk, block_msgs=64)
        s2 = sim.stats()
        sums[path] = (got, s2["relaxations"], s2["gossip_iwant"], s2["deliveries"])
    assert sums["list"] == sums["push"]
    sim.close()


@pytest.mark.parametrize("frags,phase_ms", [(2, 120), (3, 55), (8, 0), (8, 120)])
def test_gossip_in_list_pass_fragment_groups(frags, phase_ms):
    """Fragmented messages with gossip-active heartbeats: every fragment is
    gossiped on its own (the oracle's sched_gossip per (peer, fragment)); after
    the first batch's failed no-op proof the batches' IHAVE/IWANT run inside
    the list pass of fragment-group rows — bit-exact with the oracle."""
    p = oracle.params(peers=2200, seed=250 + frags, fragments=frags, hb_phase_ns=_phase(phase_ms))
    sim, _ = compare(p, 5, LINKS, _sched(32, 2200), batch=8)
    st = sim.stats()
    assert st["gossip_iwant"] > 0
    assert st["gossip_fallback_batches"] <= 1 and st["gossip_list_batches"] >= 3


@pytest.mark.parametrize("path", ["list", "push"])
def test_gossip_fragment_groups_list_equals_push(monkeypatch, path):
    """F = 8 gossip-active batches on the list pass and (GS_GOSSIP_LIST=0) on
    the push path: both equal the oracle."""
    if path == "push":
        monkeypatch.setenv("GS_GOSSIP_LIST", "0")
    p = oracle.params(peers=1800, seed=96, fragments=8, hb_phase_ns=_phase(0))
    sim, _ = compare(p, 5, LINKS, _sched(24, 1800), batch=8)
    st = sim.stats()
    if path == "list":
        assert st["gossip_fallback_batches"] == 1 and st["gossip_list_batches"] == 3
    else:
        assert st["gossip_fallback_batches"] == 3 and st["gossip_list_batches"] == 0


@pytest.mark.parametrize("phase_ms", [55, 120])
def test_gossip_in_list_pass_idontwant(phase_ms):
    """The go preset (IDONTWANT >= 1000 B, go-test-node/main.go:165) with
    gossip-active heartbeats: the IDONTWANT list pass (dense final keys, the
    neighbours' IDONTWANTs read in the emit step) takes the IHAVE / IWANT too —
    the sender planes come from the dense rows — bit-exact with the oracle."""
    p = oracle.params_for("go", peers=2400, seed=260 + phase_ms, hb_phase_ns=_phase(phase_ms))
    sim, _ = compare(p, 5, LINKS, _sched(32, 2400), batch=8)
    st = sim.stats()
    assert st["gossip_iwant"] > 0
    assert st["gossip_fallback_batches"] <= 1 and st["gossip_list_batches"] >= 3
