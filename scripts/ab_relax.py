"""A/B of k_relax variants and batch sizes in ONE process (interleaved rounds).

python scripts/ab_relax.py --peers 1000000 --rounds 5 --configs 64:1,64:4,64:5,32:4,16:4
Each config is batch:variant (variant bits: 1 read-filter, 2 tile-skip, 4 final-bitset).
Every config is first checked bit-exact against the first one on the same messages.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
import numpy as np  # noqa: E402
import gossipsim  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--peers", type=int, default=1_000_000)
ap.add_argument("--fragments", type=int, default=1)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--msgs", type=int, default=256, help="messages per timed measurement")
ap.add_argument("--configs", default="64:0,64:1,64:4,64:5,64:6,32:4,16:4,128:4")
args = ap.parse_args()
cfgs = [tuple(int(x) for x in c.split(":")) for c in args.configs.split(",")]
sims = {}
for b, _ in cfgs:
    if b not in sims:
        sim = gossipsim.Simulator(peers=args.peers, batch=b, fragments=args.fragments, seed=1)
        sim.set_topogen_links(5, 50, 150, 40, 130)
        sim.connect_gossipsub_peers()
        sim.mesh_converge()
        sims[b] = sim


def sched(i0, n):
    t, p, s = gossipsim.shard_messages(0, 0, 1, i0 + n, args.peers, 15000)
    return t[i0:], p[i0:], s[i0:]


ref = None
for b, v in cfgs:  # exactness across configs on the same 64 messages
    os.environ["GS_RELAX_VARIANT"] = str(v)
    r = sims[b].run(sched(0, 64))
    if ref is None:
        ref = r["t_complete"].copy()
    assert (r["t_complete"] == ref).all(), "config %d:%d differs" % (b, v)
res = {c: [] for c in cfgs}
for rnd in range(args.rounds):
    for b, v in cfgs:
        os.environ["GS_RELAX_VARIANT"] = str(v)
        sim = sims[b]
        sim.reset_stats()
        sim.set_timing(True)
        t0 = time.perf_counter()
        sim.run(sched(64 + rnd * args.msgs, args.msgs), collect=False)
        dt = time.perf_counter() - t0
        st = sim.stats()
        sim.set_timing(False)
        res[(b, v)].append(dict(rate=st["deliveries"] / dt, relax_ms=st["relax_ms"], run_ms=st["run_ms"],
                                launches=st["relax_launches"], relax_bytes=st["relax_bytes_alg"],
                                push_frac=st["pushes"] / max(1, st["relaxations"])))
for c in cfgs:
    rates = [x["rate"] for x in res[c]]
    rm = float(np.median([x["relax_ms"] for x in res[c]]))
    print(json.dumps(dict(batch=c[0], variant=c[1], median_rate=float(np.median(rates)),
                          min_rate=float(np.min(rates)), relax_ms=rm,
                          run_ms=float(np.median([x["run_ms"] for x in res[c]])),
                          launches=res[c][0]["launches"], push_frac=res[c][0]["push_frac"],
                          relax_alg_GBps=res[c][0]["relax_bytes"] / (rm / 1e3) / 1e9)))
