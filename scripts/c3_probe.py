"""Config #3 (bench.py CONFIGS["c3_100k_gossip_churn"]) for kernel traces:
one warm-up batch, then one timed 1024-message batch with GS_DEBUG_COUNTS-style
counters and per-bucket timing. Run under
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3 -- python scripts/c3_probe.py
and read the dispatch order with scripts/c3_trace.py."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dst-libp2p-test-node_amd"))
import gossipsim  # noqa: E402

N = int(os.environ.get("C3_PEERS", 100_000))
M = int(os.environ.get("C3_MSGS", 1024))
BATCH = int(os.environ.get("C3_BATCH", 1024))
sim = gossipsim.Simulator(peers=N, batch=BATCH, fragments=1, seed=1, lazy_gossip=1, churn_ppm=10_000, churn_down=10,
                          churn_horizon=16, heartbeat_ns=1_000_000_000,
                          hb_phase_ns=gossipsim.T0_NS - 20 * 1_000_000_000 + 370_000_000)
sim.set_topogen_links(5, 50, 150, 40, 130)
sim.connect_gossipsub_peers()
sim.mesh_converge(400)
sim.run(gossipsim.shard_messages(0, 0, 1, M, N, 15000), collect=False)
sim.reset_stats()
sim.set_timing(True)
t0 = time.perf_counter()
sim.run(gossipsim.shard_messages(1, 0, 1, M, N, 15000), collect=False)
dt = time.perf_counter() - t0
st = sim.stats()
print("c3 probe: %.1f ms, %.3g deliveries/s, %d batches, run_ms %.1f relax_ms %.1f" % (dt * 1e3, st["deliveries"] / dt, st["batches"], st["run_ms"], st["relax_ms"]))
print({k: v for k, v in st.items()})
