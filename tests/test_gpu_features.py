"""GPU tests of the round-2 features, each bit-exact against the CPU oracle:
config #0 (shadow/run.sh), subscription-time grafting, lazy gossip on the
owner-computes pull path (the no-op proof and the push-path fallback),
per-message fragment counts, the device-side per-message latency summary and
the streaming result sink / arrival log."""
import numpy as np
import pytest

import gossipsim
import oracle
from test_gpu_parity import T0, UND, _knobs, _sched, compare, gpu_sim

pytestmark = pytest.mark.gpu


def test_config0_shadow_runsh_100_peers():
    """Config #0 exactly as SURVEY §8(d) defines it (shadow/run.sh:9-19,38 with
    topogen.py's defaults 1 stage / 50 Mbit / 100 ms, topogen.py:15-20): 100
    peers, CONNECTTO 10, one 15 000 B message, FRAGMENTS 1, publisher 4, seed 1."""
    p = oracle.params(peers=100, connect_to=10, seed=1)
    sched = (np.array([T0], np.uint64), np.array([4]), np.array([15000]))
    sim, res = compare(p, 1, (50, 50, 100, 100), sched, batch=1)
    st = sim.stats()
    assert st["deliveries"] == 99 and st["gossip_iwant"] == 0
    assert res["t_complete"][0, 4] == T0 and res["hops"][0, 4] == 0


def test_subscription_grafting_on_heterogeneous_links():
    """A5 (i) on the device: the converged mesh built from the handshake-ordered
    subscription epoch equals the oracle's (compare checks CSR flags and mesh),
    and it differs from heartbeat-only formation (sub_graft = 0)."""
    p = oracle.params(peers=1500, seed=91)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(8, 1500), batch=8)
    p0 = oracle.params(peers=1500, seed=91, sub_graft=0)
    sim0, _ = compare(p0, 5, (50, 150, 40, 130), _sched(8, 1500), batch=8)
    assert (sim.mesh()[0] != sim0.mesh()[0]).any()


def test_lazy_gossip_noop_proof_on_pull_path():
    """The rust preset gossips (main.rs:230,235). With publishes 3 ms after a
    heartbeat the first IHAVE lands after the last delivery: the pull path
    proves it per batch and keeps its result (bit-exact against the oracle
    with gossip on, no IWANT)."""
    p = oracle.params(peers=2000, seed=92, lazy_gossip=1)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(40, 2000), batch=16)
    st = sim.stats()
    assert st["gossip_noop_msgs"] == 40 and st["gossip_fallback_batches"] == 0 and st["gossip_iwant"] == 0


@pytest.mark.parametrize("phase_ms", [0, 120])
def test_lazy_gossip_fallback_to_push_path(monkeypatch, phase_ms):
    """A heartbeat at (or shortly after) the publish instant: IHAVEs can land
    before the last delivery, the batch is re-run with gossip on the push path
    and the eager run's counters are discarded (bit-exact, IWANTs taken).
    GS_GOSSIP_LIST=0 keeps these batches off the list pass's own gossip
    (tests/test_gpu_gossip_list.py), the push path being the one tested here."""
    monkeypatch.setenv("GS_GOSSIP_LIST", "0")
    p = oracle.params(peers=2000, seed=93, lazy_gossip=1,
                      hb_phase_ns=(T0 + phase_ms * 1_000_000) % 1_000_000_000)
    sim, _ = compare(p, 5, (50, 150, 40, 130), _sched(24, 2000), batch=8)
    st = sim.stats()
    assert st["gossip_fallback_batches"] == 3 and st["gossip_noop_msgs"] == 0 and st["gossip_iwant"] > 0


def test_per_message_fragment_counts():
    """gs_publish.frags (PublishCommand.chunks, main.rs:65-71): batches split
    where the chunk count changes; 0 = FRAGMENTS."""
    p = oracle.params(peers=900, seed=94, fragments=2)
    t, pub, size = _sched(20, 900)
    frags = np.array([0, 0, 3, 3, 3, 1, 8, 8, 0, 5, 5, 5, 5, 16, 2, 2, 0, 0, 4, 4], np.uint32)
    sim, res = compare(p, 5, (50, 150, 40, 130), (t, pub, size, frags), batch=6)
    assert sim.stats()["deliveries"] == 20 * 899


def _np_summary(res, sched, self_log=False):
    tc = res["t_complete"].astype(np.uint64)
    M, N = tc.shape
    out = {k: [] for k in ("delivered", "lat_sum_ms", "p50_ms", "p95_ms", "max_ms")}
    hist = np.zeros((M, gossipsim.HIST_BINS), np.uint32)
    for m in range(M):
        ok = tc[m] != UND
        if not self_log:
            ok[sched[1][m]] = False
        ms = np.sort(((tc[m][ok] - np.uint64(sched[0][m])) // np.uint64(1_000_000)).astype(np.int64))
        n = len(ms)
        out["delivered"].append(n)
        out["lat_sum_ms"].append(int(ms.sum()))
        out["max_ms"].append(int(ms.max()) if n else 0)
        out["p50_ms"].append(int(ms[(n * 50 + 99) // 100 - 1]) if n else 0)
        out["p95_ms"].append(int(ms[(n * 95 + 99) // 100 - 1]) if n else 0)
        np.add.at(hist[m], np.minimum(ms // gossipsim.HIST_MS, gossipsim.HIST_BINS - 1), 1)
    return out, hist


@pytest.mark.parametrize("case", ["hetero", "slow_links", "churn", "nim_self_log"])
def test_device_latency_summary(case):
    """gs_msg_summary: delivered count, latency sum / max, the
    100 ms histogram of summary_latency.awk's hop_lat and exact nearest-rank
    p50 / p95, reduced on the device, equal numpy on the copied-out results
    (slow links put the percentiles in the open last bin: the column path)."""
    N, M = 1200, 20
    kw = dict(peers=N, seed=95)
    S, links = 5, (50, 150, 40, 130)
    if case == "slow_links":
        S, links = 1, (50, 50, 3000, 3000)
        kw.update(lazy_gossip=0)
    elif case == "churn":
        kw.update(churn_ppm=20000, hb_phase_ns=gossipsim.SHADOW_START_NS)
    elif case == "nim_self_log":
        p = oracle.params_for("nim", **kw)
    p = p if case == "nim_self_log" else oracle.params(**kw)
    sched = _sched(M, N)
    sim, _ = gpu_sim(p, S, links, batch=8)
    res = sim.run(sched, summary=True)
    ref, hist = _np_summary(res, sched, self_log=bool(p.self_log))
    for k, v in ref.items():
        np.testing.assert_array_equal(res["summary"][k], np.array(v), err_msg=k)
    np.testing.assert_array_equal(res["summary"]["hist"], hist)
    if case == "slow_links":
        assert (res["summary"]["p50_ms"] >= 6300).all()


def test_streaming_sink_and_log(tmp_path):
    """gs_result_sink.on_block streams message-major blocks (no [M][N] host
    array); gs_log_* writes the same lines as the grouped writer."""
    N, M = 3000, 70
    p = oracle.params(peers=N, seed=96)
    sched = _sched(M, N)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=32)
    whole = sim.run(sched)
    sim.write_latency_log(str(tmp_path / "grouped"), whole)
    sch = whole["schedule"]
    log = sim.open_log(str(tmp_path / "stream"))
    blocks, seen = [], []

    def on_block(first, tc, hp):
        seen.append((first, tc.shape[0]))
        np.testing.assert_array_equal(tc, whole["t_complete"][first:first + tc.shape[0]])
        np.testing.assert_array_equal(hp, whole["hops"][first:first + tc.shape[0]])
        log.write(sch[first:first + tc.shape[0]], tc)
        blocks.append(first)

    sim.run(sched, on_block=on_block, block_msgs=10)
    log.close()
    assert sum(n for _, n in seen) == M and [f for f, _ in seen] == sorted(f for f, _ in seen)
    a = sorted(open(str(tmp_path / "grouped")).read().splitlines())
    b = sorted(open(str(tmp_path / "stream")).read().splitlines())
    assert a == b and len(a) == M * (N - 1)


def test_streaming_sink_want_bits():
    """ABI 7: an on_block sink selects its outputs with gs_result_sink.want
    (GS_WANT_T_COMPLETE / GS_WANT_HOPS); array pointers set together with
    on_block (the ABI-6 flag convention) are refused with GS_EINVAL."""
    import ctypes
    N, M = 1500, 12
    p = oracle.params(peers=N, seed=97)
    sched = _sched(M, N)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=16)
    whole = sim.run(sched)
    for want, has_tc, has_hp in ((gossipsim.WANT_T_COMPLETE, True, False), (gossipsim.WANT_HOPS, False, True),
                                 (0, True, True)):
        got = []

        def blk(first, tc, hp):
            got.append((first, None if tc is None else tc.copy(), None if hp is None else hp.copy()))

        sim.run(sched, on_block=blk, block_msgs=5, want=want)
        assert [g[0] for g in got] == [0, 5, 10]
        for first, tc, hp in got:
            assert (tc is not None) == has_tc and (hp is not None) == has_hp
            if has_tc:
                np.testing.assert_array_equal(tc, whole["t_complete"][first:first + tc.shape[0]])
            if has_hp:
                np.testing.assert_array_equal(hp, whole["hops"][first:first + hp.shape[0]])
    lib = gossipsim.lib()
    cb = gossipsim.BLOCK_FN(lambda *a: None)
    flag = np.zeros(1, np.uint64)
    sink = gossipsim.GsResultSink()
    sink.t_complete_ns = flag.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    sink.on_block = cb
    rc = lib.gs_run(sim.ctx, sim._schedule(sched), M, ctypes.byref(sink))
    assert rc == gossipsim.GS_EINVAL and b"want" in lib.gs_last_error(sim.ctx)


def _logged_ms(tc, sched, self_log):
    """The oracle side of GS_WANT_LAT_MS: (t_complete - tx_time) // 1e6 where a
    line is logged (main.rs:91-93), LAT_NONE elsewhere."""
    tx = np.asarray(sched[0], np.uint64)[:, None]
    ok = tc != UND
    if not self_log:
        ok[np.arange(tc.shape[0]), np.asarray(sched[1])] = False
    out = np.full(tc.shape, gossipsim.LAT_NONE, np.uint16)
    out[ok] = ((tc - tx) // np.uint64(1_000_000))[ok].astype(np.uint16)
    return out


@pytest.mark.parametrize("case", ["rust", "nim_self_log", "churn", "frags3", "gossip_370"])
@pytest.mark.parametrize("with_rows", [False, True])
def test_latency_ms_stream(case, with_rows):
    """ABI 9's u16 latency stream (gs_result_sink.on_lat, GS_WANT_LAT_MS):
    exactly the ms each peer's log line carries (main.rs:91-93), GS_LAT_NONE
    for the undelivered and the publisher (unless SELFTRIGGER), against the
    oracle; alone (the list pass's final logs, k_lcomplete) and beside the
    t_complete / hops stream (dense rows, k_complete)."""
    N, M = 1400, 20
    kw = dict(peers=N, seed=98)
    if case == "churn":
        kw.update(churn_ppm=30000, hb_phase_ns=gossipsim.SHADOW_START_NS)
    elif case == "frags3":
        kw.update(fragments=3)
    elif case == "gossip_370":
        kw.update(hb_phase_ns=(T0 + 370_000_000) % 1_000_000_000)
    p = oracle.params_for("nim", **kw) if case == "nim_self_log" else oracle.params(**kw)
    sched = _sched(M, N)
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    lat, rows = {}, {}

    def on_lat(first, v):
        lat[first] = v.copy()

    def on_block(first, tc, hp):
        rows[first] = tc.copy()

    sim.run(sched, on_lat=on_lat, on_block=on_block if with_rows else None, block_msgs=6,
            want=gossipsim.WANT_T_COMPLETE)
    assert sorted(lat) == [0, 6, 8, 14, 16]  # blocks of 6 inside each batch of 8
    got = np.concatenate([lat[k] for k in sorted(lat)])
    np.testing.assert_array_equal(got, _logged_ms(ref["t_complete"], sched, p.self_log))
    if with_rows:
        np.testing.assert_array_equal(np.concatenate([rows[k] for k in sorted(rows)]), ref["t_complete"])
    st = sim.stats()
    assert st["deliveries"] == ref["stats"]["deliveries"]


def test_latency_ms_stream_writes_the_log(tmp_path):
    """gs_log_write_lat over the u16 stream writes the same lines as the
    grouped writer over t_complete (the C++ CLI streams this way)."""
    N, M = 900, 10
    p = oracle.params(peers=N, seed=99)
    sched = _sched(M, N)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    whole = sim.run(sched)
    a, b = tmp_path / "grouped", tmp_path / "stream"
    sim.write_latency_log(str(a), whole)
    log = gossipsim.LogStream(sim.cfg, str(b))
    rows = sim._schedule(sched)
    sim.run(sched, on_lat=lambda first, v: log.write_lat(rows[first:first + v.shape[0]], v), block_msgs=4)
    log.close()
    assert sorted(open(a).read().splitlines()) == sorted(open(b).read().splitlines())


def test_shadow_parity_harness_end_to_end(tmp_path):
    """shadow_parity.py end to end on the GPU: a synthetic Shadow `latencies1`
    (an oracle run written in the grep format run.sh:61 produces) -> schedule
    rebuilt from the log -> the GPU run with gs_msg_summary's device
    percentiles -> 0 error on every message's p50 / p95 / max; the same log with
    every latency +8 % fails the +-5 % gate."""
    import json
    import shadow_parity as sp
    N, M = 400, 5
    p = oracle.params(peers=N, seed=21)
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(3_000_000_000)
    sched = (t, (9 + 7 * np.arange(M)) % N, np.full(M, 15000))
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    sim.write_latency_log(str(tmp_path / "latencies1"), {"schedule": sim._schedule(sched),
                                                         "t_complete": ref["t_complete"]})
    sim.close()
    args = ["--latencies", str(tmp_path / "latencies1"), "--peers", str(N), "--seed", "21",
            "--topogen", "5,50,150,40,130", "--json", str(tmp_path / "rep.json")]
    assert sp.main(args) == 0
    rep = json.load(open(tmp_path / "rep.json"))
    assert rep["pass"] and rep["messages"] == M
    assert rep["worst_abs_rel_err"] == {"p50": 0.0, "p95": 0.0, "max": 0.0}
    assert rep["deliveries"]["sim"] == rep["deliveries"]["shadow"] == ref["stats"]["deliveries"]
    lines = open(tmp_path / "latencies1").read().splitlines()
    with open(tmp_path / "latencies2", "w") as f:
        for ln in lines:
            head, ms = ln.rsplit(" ", 1)
            f.write("%s %d\n" % (head, int(ms) * 108 // 100))
    args[1] = str(tmp_path / "latencies2")
    assert sp.main(args) == 1


def _stats_no_time(sim):
    # pushes counts atomicMin calls past a racy pre-read filter: a diagnostic, not deterministic
    return {k: v for k, v in sim.stats().items() if not k.endswith("_ms") and k != "pushes"}


@pytest.mark.parametrize("case", ["frozen_traffic", "churn_gossip", "churn_replay"])
def test_checkpoint_resume(tmp_path, case):
    """gs_save_state / gs_load_state (SURVEY §5 checkpoint/resume): a schedule
    split at a save point and continued on a context loaded from the file (on a
    fresh context, the saved one destroyed) gives the same results, counters and
    per-peer traffic as the uninterrupted context; the results are also the
    oracle's. churn_gossip resumes after the churn mesh state moved forward;
    churn_replay's second half publishes before the saved state, so the loaded
    context replays the churn epochs from epoch 0."""
    N, M = 1500, 24
    kw = dict(peers=N, seed=98)
    if case != "frozen_traffic":
        kw.update(churn_ppm=20000, hb_phase_ns=gossipsim.SHADOW_START_NS, lazy_gossip=1)
    p = oracle.params(**kw)
    t, pub, size = _sched(M, N)
    if case == "churn_replay":  # the later half of the publishes first
        t, pub = np.roll(t, -(M // 2)), np.roll(pub, -(M // 2))
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=(t, pub, size))
    h = M // 2
    first, second = (t[:h], pub[:h], size[:h]), (t[h:], pub[h:], size[h:])
    whole, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    whole.set_traffic(True)
    a = whole.run(first)
    b = whole.run(second)
    part, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    part.set_traffic(True)
    a2 = part.run(first)
    part.save_state(tmp_path / "gs.state")
    mesh0, csr0 = part.mesh(), part.csr()
    part.close()
    res = gossipsim.Simulator.load_state(tmp_path / "gs.state", device=0)
    for x, y in zip(res.mesh() + res.csr(), mesh0 + csr0):
        np.testing.assert_array_equal(x, y)
    assert res.peers == N and res.cfg.churn_ppm == p.churn_ppm and res.cfg.batch == 8
    b2 = res.run(second)
    for k in ("t_complete", "hops"):
        np.testing.assert_array_equal(a2[k], a[k])
        np.testing.assert_array_equal(b2[k], b[k])
        np.testing.assert_array_equal(np.concatenate([a2[k], b2[k]]), ref[k])
    assert _stats_no_time(res) == _stats_no_time(whole)
    assert res.stats()["deliveries"] == ref["stats"]["deliveries"]
    np.testing.assert_array_equal(res.traffic(), whole.traffic())


@pytest.mark.parametrize("case", ["rust", "nim_self_log", "gossip_370", "gossip_55", "not_lockstep"])
def test_completion_counted_by_the_passes(case):
    """Results left on the device (nothing streamed out, the bench's path): the
    counters come from the list pass's final logs (k_lcomplete) and the lazy
    gossip no-op proof from its per-message reductions; lockstep or not, with
    gossip proven a no-op or taken inside the passes, they equal the oracle's."""
    N, M = 1400, 24
    kw = dict(peers=N, seed=77)
    if case.startswith("gossip"):
        kw.update(hb_phase_ns=(T0 + int(case.split("_")[1]) * 1_000_000) % 1_000_000_000)
    p = oracle.params_for("nim", **kw) if case == "nim_self_log" else oracle.params(**kw)
    sched = _sched(M, N)
    if case == "not_lockstep":  # publish times off the heartbeat grid by different amounts
        t = np.asarray(sched[0], np.uint64) + (np.arange(M, dtype=np.uint64) * np.uint64(7_777_777))
        sched = (t, sched[1], sched[2])
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
    sim, _ = gpu_sim(p, 5, (50, 150, 40, 130), batch=8)
    sim.run(sched, collect=False)
    st = sim.stats()
    for k in ("deliveries", "relaxations", "gossip_iwant", "latency_sum_ms", "latency_max_ms"):
        assert st[k] == ref["stats"][k], k
    assert st["list_pull_batches"] >= 1
