"""A/B of k_pull knobs read from the environment per batch (one process,
interleaved rounds): python scripts/ab_spec.py --var GS_PULL_SPEC --values off,8,16,32
Every value must give the same counters (deliveries, relaxations, latency sums)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
import gossipsim  # noqa: E402

if os.environ.get("GS_LIB_PATH"):
    gossipsim.LIB_PATH = os.environ["GS_LIB_PATH"]

ap = argparse.ArgumentParser()
ap.add_argument("--peers", type=int, default=1_000_000)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--var", default="GS_PULL_SPEC")
ap.add_argument("--values", default="off,8,16,32,64")
args = ap.parse_args()
sim = gossipsim.Simulator(peers=args.peers, batch=1024, fragments=1, seed=1)
sim.set_topogen_links(5, 50, 150, 40, 130)
sim.connect_gossipsub_peers()
sim.mesh_converge()
vals = args.values.split(",")
best = {v: 1e9 for v in vals}
ref = None
for r in range(args.rounds):
    for v in vals:
        if v == "off":
            os.environ.pop(args.var, None)
        else:
            os.environ[args.var] = v
        sim.reset_stats()
        t0 = time.perf_counter()
        sim.run(gossipsim.shard_messages(r, 0, 1, 1024, args.peers, 15000), collect=False)
        dt = time.perf_counter() - t0
        st = sim.stats()
        key = (r, st["deliveries"], st["relaxations"], st["latency_sum_ms"], st["latency_max_ms"],
               st["frag_deliveries"])
        if v == vals[0]:
            ref = key
        assert key == ref, (v, key, ref)
        best[v] = min(best[v], dt)
        print("round %d %s=%s %.2f ms" % (r, args.var, v, dt * 1e3), flush=True)
for v in vals:
    print("BEST %s=%s %.2f ms" % (args.var, v, best[v] * 1e3))
