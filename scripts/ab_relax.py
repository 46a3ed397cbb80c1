"""A/B of the k_relax variants in ONE process on one graph (rule: interleaved rounds).

python scripts/ab_relax.py --peers 1000000 --rounds 5 --steps 4
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
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--fragments", type=int, default=1)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--variants", default="0,1,2,3")
args = ap.parse_args()
sim = gossipsim.Simulator(peers=args.peers, batch=args.batch, fragments=args.fragments, seed=1)
sim.set_topogen_links(5, 50, 150, 40, 130)
sim.connect_gossipsub_peers()
sim.mesh_converge()
variants = [int(v) for v in args.variants.split(",")]
ref = None
for v in variants:  # exactness across variants on one batch
    os.environ["GS_RELAX_VARIANT"] = str(v)
    r = sim.run(gossipsim.shard_messages(0, 0, 1, args.batch, args.peers, 15000))
    if ref is None:
        ref = r["t_complete"].copy()
    assert (r["t_complete"] == ref).all(), "variant %d differs" % v
res = {v: [] for v in variants}
for rnd in range(args.rounds):
    for v in variants:
        os.environ["GS_RELAX_VARIANT"] = str(v)
        sim.reset_stats()
        sim.set_timing(True)
        t0 = time.perf_counter()
        for s in range(args.steps):
            sim.run(gossipsim.shard_messages(1 + s, 0, 1, args.batch, args.peers, 15000), collect=False)
        dt = time.perf_counter() - t0
        st = sim.stats()
        res[v].append(dict(rate=st["deliveries"] / dt, relax_ms=st["relax_ms"] / args.steps,
                           launches=st["relax_launches"] / args.steps, run_ms=st["run_ms"] / args.steps))
for v in variants:
    rates = [x["rate"] for x in res[v]]
    print(json.dumps(dict(variant=v, median_rate=float(np.median(rates)), min_rate=float(np.min(rates)),
                          relax_ms_per_step=float(np.median([x["relax_ms"] for x in res[v]])),
                          run_ms_per_step=float(np.median([x["run_ms"] for x in res[v]])),
                          launches_per_step=res[v][0]["launches"])))
