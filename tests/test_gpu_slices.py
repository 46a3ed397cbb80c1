"""Batch slices (gs_relax.hip try_slices / run_lpull_batch's Slices): several
full batches of one shape on a small graph run as ONE list pass over copies of
the graph (slice j's rows are j * N + peer). The results must be those of the
same batches run one at a time (GS_SLICES=0) and of the CPU oracle, for every
way a run hands results out (rows, streamed blocks, latency stream, summaries,
device-resident counters), with single- and multi-fragment rows and with lazy
gossip (the eager pass's no-op proof per slice, and a phase where the proof
fails and the group is re-run as single batches).

Reference: config #2 (BASELINE.json, shadow/README.md:57: 10k peers,
FRAGMENTS=8, 1000 messages); main.rs:101-143 / 228-235 for the rules the
oracle restates."""
import numpy as np
import pytest

import gossipsim
import oracle
from test_gpu_parity import T0, _sched, compare, gpu_sim

pytestmark = pytest.mark.gpu
LINKS = (50, 150, 40, 130)
HB = 1_000_000_000


def _run(monkeypatch, slices, p, sched, batch, how):
    monkeypatch.setenv("GS_SLICES", slices)
    sim, _ = gpu_sim(p, 5, LINKS, batch=batch)
    out = {}
    if how == "rows":
        res = sim.run(sched)
        out["t"], out["h"] = res["t_complete"], res["hops"]
    elif how == "summary":
        res = sim.run(sched, summary=True)
        out["t"] = res["t_complete"]
        out.update({"summary_" + k: v for k, v in res["summary"].items()})
    elif how == "lat":
        got = []
        sim.run(sched, collect=False, on_lat=lambda first, lat: got.append((first, lat.copy())), block_msgs=7)
        out["lat"] = np.concatenate([x for _, x in sorted(got, key=lambda y: y[0])])
    else:
        sim.run(sched, collect=False)
    st = sim.stats()
    sim.close()
    return out, st


KEYS = ("deliveries", "frag_deliveries", "relaxations", "latency_sum_ms", "latency_max_ms", "messages", "batches",
        "gossip_iwant", "list_pull_batches")


@pytest.mark.parametrize("frags,gossip,how", [
    (1, 0, "rows"), (1, 1, "rows"), (8, 1, "rows"), (1, 1, "none"), (4, 0, "lat"), (1, 1, "lat"),
    (2, 1, "summary")])
def test_slices_equal_single_batches(monkeypatch, frags, gossip, how):
    """8 batches of 16 messages at 1500 peers: one sliced pass (8 copies of the
    graph) equals the 8 single batches bit for bit, with fewer window passes."""
    p = oracle.params(peers=1500, seed=300 + frags, fragments=frags, lazy_gossip=gossip)
    sched = _sched(128, 1500)
    a, sa = _run(monkeypatch, "", p, sched, 16, how)
    b, sb = _run(monkeypatch, "0", p, sched, 16, how)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for k in KEYS:
        assert sa[k] == sb[k], k
    assert sa["batches"] == 8 and sa["list_pull_batches"] == 8


def test_slices_fewer_passes_with_timing(monkeypatch):
    """The sliced group runs its passes once for all its batches."""
    p = oracle.params(peers=1200, seed=310, fragments=1)
    sched = _sched(64, 1200)
    launches = {}
    for env in ("", "0"):
        monkeypatch.setenv("GS_SLICES", env)
        sim, _ = gpu_sim(p, 5, LINKS, batch=16)
        sim.set_timing(True)
        sim.run(sched, collect=False)
        launches[env] = sim.stats()["relax_launches"]
        sim.close()
    assert launches[""] * 2 < launches["0"]


@pytest.mark.parametrize("frags", [1, 8])
def test_slices_against_oracle(monkeypatch, frags):
    """A sliced run (3 slices of 10 + a single batch of the rest) equals the oracle."""
    monkeypatch.setenv("GS_SLICES", "")
    p = oracle.params(peers=900, seed=320 + frags, fragments=frags)
    compare(p, 5, LINKS, _sched(37, 900), batch=10)


def test_slices_gossip_phase_falls_back_exactly(monkeypatch):
    """Heartbeats 120 ms after every publish: IWANTs change the result, the
    group's no-op proof fails and the group runs again with the IHAVE / IWANT
    inside its passes — still the oracle's result; the discarded eager run
    counts once as a fallback."""
    monkeypatch.setenv("GS_SLICES", "")
    p = oracle.params(peers=1200, seed=330, hb_phase_ns=(T0 + 120_000_000) % HB)
    sim, _ = compare(p, 5, LINKS, _sched(32, 1200), batch=8)
    st = sim.stats()
    # the first single batch's eager pass fails its proof (the group's counts nothing), then every
    # batch runs its gossip inside the list pass
    assert st["gossip_iwant"] > 0 and st["batches"] == 4
    assert st["gossip_fallback_batches"] == 1 and st["gossip_list_batches"] == 4


def test_slices_c2_shape_bench_path(monkeypatch):
    """bench.py's config #2 shape (10k peers, F = 8, 128-message batches) on a
    quarter of its messages: device-resident counters equal the single-batch run."""
    p = oracle.params(peers=10_000, seed=1, fragments=8)
    sched = gossipsim.shard_messages(1, 0, 1, 256, 10_000, 15000)
    _, sa = _run(monkeypatch, "", p, sched, 128, "none")
    _, sb = _run(monkeypatch, "0", p, sched, 128, "none")
    for k in KEYS:
        assert sa[k] == sb[k], k
    assert sa["gossip_noop_msgs"] == 256


@pytest.mark.parametrize("frags,slices", [(2, "0"), (8, "0"), (8, ""), (3, "")])
def test_fragment_groups_complete_from_logs(monkeypatch, frags, slices):
    """Fragmented batches complete from the final logs (k_lcomplete reduces each
    message's F fragment lanes: reassembly) unless a sink takes rows: the
    counters, the gossip no-op proof and the u16 latency stream equal the dense
    rows' k_complete (GS_LPULL_DENSE=1)."""
    p = oracle.params(peers=1300, seed=340 + frags, fragments=frags)
    sched = _sched(64, 1300)
    out = {}
    for dense in ("", "1"):
        monkeypatch.setenv("GS_LPULL_DENSE", dense)
        o, st = _run(monkeypatch, slices, p, sched, 16, "lat")
        _, st2 = _run(monkeypatch, slices, p, sched, 16, "none")
        out[dense] = (o["lat"], st, st2)
    np.testing.assert_array_equal(out[""][0], out["1"][0])
    for k in KEYS + ("gossip_noop_msgs",):
        assert out[""][1][k] == out["1"][1][k], k
        assert out[""][2][k] == out["1"][2][k], k
    assert out[""][2]["gossip_noop_msgs"] == 64


@pytest.mark.parametrize("frags,phase_ms", [(1, 55), (1, 30), (4, 120)])
def test_slices_gossip_active_equal_single_batches(monkeypatch, frags, phase_ms):
    """Gossip-active groups (the in-pass IHAVE / IWANT over slice rows: CSR and
    rng by the peer, planes and row-done bits by the slice row, each slice's
    heartbeat indices) equal the same batches run one at a time."""
    p = oracle.params(peers=1400, seed=350 + phase_ms, fragments=frags, hb_phase_ns=(T0 + phase_ms * 1_000_000) % HB)
    sched = _sched(96, 1400)
    a, sa = _run(monkeypatch, "", p, sched, 16, "rows")
    b, sb = _run(monkeypatch, "0", p, sched, 16, "rows")
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # (which batches take the in-pass gossip may differ: a single batch can prove its gossip a no-op)
    for k in ("deliveries", "frag_deliveries", "relaxations", "latency_sum_ms", "latency_max_ms", "messages",
              "batches", "gossip_iwant"):
        assert sa[k] == sb[k], k
    assert sa["gossip_iwant"] > 0 and sa["gossip_list_batches"] >= 5


def test_slices_gossip_active_against_oracle(monkeypatch):
    monkeypatch.setenv("GS_SLICES", "")
    p = oracle.params(peers=1100, seed=360, fragments=2, hb_phase_ns=(T0 + 90_000_000) % HB)
    sim, _ = compare(p, 5, LINKS, _sched(40, 1100), batch=8)
    st = sim.stats()
    assert st["gossip_iwant"] > 0 and st["gossip_list_batches"] == 5
