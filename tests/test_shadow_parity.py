"""The Shadow-parity harness (dst-libp2p-test-node_amd/shadow_parity.py) on
synthetic Shadow logs, CPU only.

A synthetic `latencies<i>` file is the grep output run.sh:61 makes, written by
the product's own log writer (gs_write_node_log, the format the reference awk
scripts are pinned to in test_host_cpu.py) from an oracle run. The harness must
read it back, rebuild the publish schedule (t_pub = tx_time, publisher = the
peer without a line), and compute the nearest-rank p50 / p95 / max that a numpy
restatement (np.percentile method="inverted_cdf") gives; a simulator summary
with the same numbers scores 0 error, a +3 % shift passes the +-5 % gate and a
+8 % shift fails it. The GPU end of the harness (Simulator.run(summary=True))
is covered by tests/test_gpu_features.py::test_shadow_parity_harness_end_to_end."""
import ctypes
import os

import numpy as np
import pytest

import gossipsim
import oracle
import shadow_parity as sp

T0 = gossipsim.T0_NS


def _oracle_run(N=300, M=6, seed=11):
    p = oracle.params(peers=N, seed=seed)
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(2_000_000_000)
    pub = ((17 + 5 * np.arange(M)) % N).astype(np.int64)
    sched = (t, pub, np.full(M, 15000))
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
    return p, sched, ref


def _write_log(path, p, sched, tc):
    cfg = gossipsim.PeerConfig(**{n: getattr(p, n) for n, _ in oracle.OrParams._fields_})
    t, pub, size = sched
    arr = (gossipsim.GsPublish * len(t))(*[gossipsim.GsPublish(int(t[i]), int(pub[i]), int(size[i]), 0, 0)
                                           for i in range(len(t))])
    tc = np.ascontiguousarray(tc, np.uint64)
    rc = gossipsim.lib().gs_write_node_log(ctypes.byref(cfg.c), str(path).encode(), arr, len(t),
                                           tc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert rc == 0


def _np_summary(sched, tc):
    out = {}
    for i, tx in enumerate(sched[0].tolist()):
        row = tc[i][(tc[i] != np.iinfo(np.uint64).max) & (np.arange(tc.shape[1]) != sched[1][i])]
        ms = ((row - np.uint64(tx)) // np.uint64(1_000_000)).astype(np.int64)
        out[int(tx)] = {"n": len(ms), "sum": int(ms.sum()), "max": int(ms.max()),
                        "p50": int(np.percentile(ms, 50, method="inverted_cdf")),
                        "p95": int(np.percentile(ms, 95, method="inverted_cdf"))}
    return out


def test_synthetic_shadow_log_round_trip(tmp_path):
    p, sched, ref = _oracle_run()
    log = tmp_path / "latencies1"
    _write_log(log, p, sched, ref["t_complete"])
    # the grep output also carries BW lines and other noise the awk scripts drop
    with open(log, "a") as f:
        f.write("shadow.data/hosts/peer3/main.1000.stdout:9:BW: in 12 out 30\n")
        f.write("shadow.data/hosts/peer3/main.1000.stderr:1:thread panicked\n")
    per = sp.read_latencies(str(log))
    assert sorted(per) == [int(x) for x in sched[0]]
    t, pub, size = sp.schedule_from_log(per, p.peers, 15000)
    np.testing.assert_array_equal(t, sched[0])
    np.testing.assert_array_equal(pub, sched[1])
    got = sp.summarize(per)
    want = _np_summary(sched, ref["t_complete"])
    assert got == want
    rep = sp.compare(got, want)
    assert rep["pass"] and rep["worst_abs_rel_err"] == {"p50": 0.0, "p95": 0.0, "max": 0.0}
    assert rep["deliveries"]["shadow"] == ref["stats"]["deliveries"]


@pytest.mark.parametrize("shift,ok", [(1.03, True), (0.97, True), (1.08, False)])
def test_shadow_gate_at_5_percent(tmp_path, shift, ok):
    """Every latency of the 'Shadow' side scaled: the harness reports the
    relative error of each percentile and gates at +-5 %."""
    p, sched, ref = _oracle_run(seed=12)
    sim = _np_summary(sched, ref["t_complete"])
    shadow = {tx: {k: (int(round(v * shift)) if k in ("p50", "p95", "max", "sum") else v) for k, v in d.items()}
              for tx, d in sim.items()}
    rep = sp.compare(shadow, sim)
    assert rep["pass"] == ok
    e = rep["worst_abs_rel_err"]
    assert abs(max(e.values()) - abs(1 / shift - 1)) < 0.01


def test_pod_host_names_and_ambiguous_publisher(tmp_path):
    """topogen names its hosts pod-<i> (defect D3); a message that another peer
    also missed has no unique publisher and takes run.sh's rule instead."""
    p, sched, ref = _oracle_run(N=200, M=3, seed=13)
    tc = ref["t_complete"].copy()
    tc[1, (sched[1][1] + 1) % p.peers] = np.iinfo(np.uint64).max  # a second silent peer for message 1
    log = tmp_path / "latencies1"
    _write_log(log, p, sched, tc)
    text = open(log).read().replace("/peer", "/pod-")
    open(log, "w").write(text)
    per = sp.read_latencies(str(log))
    assert len(per) == 3
    with pytest.raises(ValueError, match="ambiguous"):
        sp.schedule_from_log(per, p.peers, 15000)
    _, pub, _ = sp.schedule_from_log(per, p.peers, 15000, publisher_id=int(sched[1][0]), rotation=5)
    np.testing.assert_array_equal(pub, sched[1])
