"""Config #3 (100k peers, hetero links, lazy gossip, 1 % churn) timing for rocprofv3."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gossipsim  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_100k_gossip_churn"
c = dict(bench.CONFIGS[name])
if len(sys.argv) > 2:
    c["batch"] = int(sys.argv[2])
if len(sys.argv) > 3:
    c["msgs"] = int(sys.argv[3])
# C3_KNOBS="lazy_gossip=0,churn_ppm=0": override config knobs (A/B of the mesh / gossip parts)
for kv in filter(None, os.environ.get("C3_KNOBS", "").split(",")):
    k, v = kv.split("=")
    c["knobs"] = dict(c["knobs"], **{k: int(v)})
sim = gossipsim.Simulator(peers=c["peers"], batch=c["batch"], fragments=c["fragments"], seed=1, **c["knobs"])
sim.set_topogen_links(c["links"][0], *c["links"][1:])
t0 = time.perf_counter()
sim.connect_gossipsub_peers()
sim.mesh_converge(400)
print("setup %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
sim.run(gossipsim.shard_messages(0, 0, 1, c["batch"], c["peers"], 15000), collect=False)
sim.reset_stats()
t0 = time.perf_counter()
sim.run(gossipsim.shard_messages(1, 0, 1, c["msgs"], c["peers"], 15000), collect=False)
dt = time.perf_counter() - t0
st = sim.stats()
print("batch %d: %.1f ms for %d msgs, %.3g deliveries/s" % (c["batch"], dt * 1e3, c["msgs"], st["deliveries"] / dt),
      {k: st[k] for k in ("deliveries", "relaxations", "gossip_iwant", "buckets", "relax_launches")})
