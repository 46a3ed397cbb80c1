"""Config #2 shape probe (bench.py CONFIGS["c2_10k_F8"]): per-pass time of the
F = 8 list pass at several peer counts with one 128-message batch, to size
what running several batches' rows in one launch would buy (a 10k-row pass is
a few rows per resident wave). Prints one line per peer count."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dst-libp2p-test-node_amd"))
import gossipsim  # noqa: E402

for N in [int(x) for x in os.environ.get("C2_PEERS", "10000,20000,40000,80000").split(",")]:
    B = int(os.environ.get("C2_BATCH", 128))
    sim = gossipsim.Simulator(peers=N, batch=B, fragments=8, seed=1)
    sim.set_topogen_links(5, 50, 150, 40, 130)
    sim.connect_gossipsub_peers()
    sim.mesh_converge(400)
    sim.run(gossipsim.shard_messages(0, 0, 1, B, N, 15000), collect=False)
    best = None
    for _ in range(3):
        sim.reset_stats()
        t0 = time.perf_counter()
        sim.run(gossipsim.shard_messages(1, 0, 1, B, N, 15000), collect=False)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    sim.reset_stats()
    sim.set_timing(True)
    sim.run(gossipsim.shard_messages(1, 0, 1, B, N, 15000), collect=False)
    sim.set_timing(False)
    st = sim.stats()
    print("c2 probe N=%d B=%d: run %.2f ms, passes %d, pass_ms %.2f (%.1f us each), %.3g deliveries/s" %
          (N, B, best * 1e3, st["relax_launches"], st["relax_ms"], st["relax_ms"] * 1e3 / max(1, st["relax_launches"]),
           st["deliveries"] / best), flush=True)
    sim.close()
