"""Sensitivity of the latency percentiles to the model constants the reference
cannot pin: the handshake round trips before the subscription
epoch (hs_rtts), the heartbeat phase of a publish (the +3 ms
injector transit in gossipsim.T0_NS, §2.7) and the muxer / signing overheads
(A9, §2.4). Configs #0 and #1 of SURVEY §8(d) on the CPU oracle (the GPU is
bit-exact with it on all of these knobs); per variant the pooled nearest-rank
p50 / p95 / max of every delivery (ms) and the mean per-message max (the
"Average Max Message Dissemination Latency" of summary_latency_large.awk:63-68),
with the relative change against the baseline row.

    python scripts/sensitivity.py --json profiles/r03_sensitivity.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
import oracle  # noqa: E402  (CPU oracle)

T0 = 946684800_000_000_000 + 500_000_000_000 + 3_000_000  # gossipsim.T0_NS
HB = 1_000_000_000


def phase_for(offset_ns):
    """hb_phase_ns such that every publish at T0 + k s lands offset_ns after a heartbeat."""
    return (T0 - offset_ns) % HB


VARIANTS = [
    ("baseline: hs_rtts 3, publish 3 ms after a heartbeat, yamux, signed", {}),
    ("hs_rtts 2", dict(hs_rtts=2)),
    ("hs_rtts 4", dict(hs_rtts=4)),
    ("publish 370 ms after a heartbeat", dict(hb_phase_ns=phase_for(370_000_000))),
    ("publish 700 ms after a heartbeat", dict(hb_phase_ns=phase_for(700_000_000))),
    ("publish 0 ms after a heartbeat (no injector transit)", dict(hb_phase_ns=phase_for(0))),
    ("muxer quic", dict(muxer=1)),
    ("muxer mplex", dict(muxer=2)),
    ("unsigned messages", dict(signed_msgs=0)),
]

CONFIGS = {
    "c0_100_peers_1_msg": dict(peers=100, stages=1, links=(50, 50, 100, 100), msgs=1, pub0=4, rotation=0,
                               seeds=list(range(1, 21))),
    "c1_1k_peers_100_msgs": dict(peers=1000, stages=1, links=(50, 50, 50, 50), msgs=100, pub0=6, rotation=1,
                                 seeds=[1, 2, 3]),
    # config #1's size on config #2/#3's heterogeneous run.sh links (5 stages, 50-150 Mbit, 40-130 ms)
    "c1_1k_peers_hetero_links": dict(peers=1000, stages=5, links=(50, 150, 40, 130), msgs=100, pub0=6, rotation=1,
                                     seeds=[1, 2, 3]),
}


def nearest_rank(s, q):
    return int(s[max(1, -(-q * len(s) // 100)) - 1])


def measure(cfg, knobs):
    lat, maxes = [], []
    for seed in cfg["seeds"]:
        p = oracle.params(peers=cfg["peers"], seed=seed, **knobs)
        M = cfg["msgs"]
        t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(HB)
        pub = (cfg["pub0"] + cfg["rotation"] * np.arange(M)) % cfg["peers"]
        ref = oracle.simulate(p, cfg["stages"], cfg["links"], sched=(t, pub, np.full(M, 15000)))
        tc = ref["t_complete"]
        for i in range(M):
            row = tc[i][(tc[i] != np.iinfo(np.uint64).max) & (np.arange(cfg["peers"]) != pub[i])]
            ms = (row - t[i]) // np.uint64(1_000_000)
            lat.append(ms)
            maxes.append(int(ms.max()))
    s = np.sort(np.concatenate(lat))
    return {"p50_ms": nearest_rank(s, 50), "p95_ms": nearest_rank(s, 95), "max_ms": int(s[-1]),
            "avg_max_ms": float(np.mean(maxes)), "deliveries": int(len(s))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    args = ap.parse_args()
    out = {}
    for cname, cfg in CONFIGS.items():
        rows = []
        base = None
        for vname, knobs in VARIANTS:
            r = measure(cfg, knobs)
            if base is None:
                base = r
            r["rel"] = {k: (r[k] - base[k]) / base[k] for k in ("p50_ms", "p95_ms", "max_ms", "avg_max_ms")}
            r["variant"] = vname
            rows.append(r)
            print("%-22s %-58s p50 %5d p95 %5d max %5d avg-max %8.1f | %+6.1f%% %+6.1f%% %+6.1f%% %+6.1f%%" % (
                cname, vname, r["p50_ms"], r["p95_ms"], r["max_ms"], r["avg_max_ms"],
                100 * r["rel"]["p50_ms"], 100 * r["rel"]["p95_ms"], 100 * r["rel"]["max_ms"],
                100 * r["rel"]["avg_max_ms"]), flush=True)
        out[cname] = {"config": {k: v for k, v in cfg.items()}, "rows": rows}
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
