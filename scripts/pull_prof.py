"""Diagnostic: where the shader clocks of k_pull go, per pass (needs the
GS_PULL_PROF build, scripts/pull_prof.sh). Slots: 0 skipped rows, 1 key +
record loads and the LDS min (step 1-2), 2 dense merge (3), 3 sparse emit (4),
4 chunk minima (5), 5 active rows."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
import gossipsim  # noqa: E402

gossipsim.LIB_PATH = os.path.join(ROOT, "prof_build", "libgossipsim.so")
peers = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
L = gossipsim.lib()
L.gs_debug_pull_prof.argtypes = [ctypes.c_void_p]
B = int(os.environ.get("BATCH", 1024))  # config #2: PEERS=10000 BATCH=128 FRAGS=8
sim = gossipsim.Simulator(peers=peers, batch=B, fragments=int(os.environ.get("FRAGS", 1)), seed=1, device=0)
sim.set_topogen_links(5, 50, 150, 40, 130)
sim.connect_gossipsub_peers()
sim.mesh_converge(400)
sim.run(gossipsim.shard_messages(0, 0, 1, B, peers, 15000), collect=False)
buf = np.zeros(32 * 8, dtype=np.uint64)
L.gs_debug_pull_prof(buf.ctypes.data)
sim.set_timing(True)
sim.run(gossipsim.shard_messages(1, 0, 1, B, peers, 15000), collect=False)
L.gs_debug_pull_prof(buf.ctypes.data)
b = buf.reshape(32, 8).astype(np.float64)
print("pass  skip%  load+rec%  dense%  sparse%  cmin%  active_rows  Gclk")
for p in range(32):
    t = b[p, :5].sum()
    if t == 0:
        continue
    print("%4d %6.1f %9.1f %7.1f %8.1f %6.1f %12d %6.2f" % (
        p, *(100 * b[p, :5] / t), int(b[p, 5]), t / 1e9))
tot = b[:, :5].sum(0)
print("all  " + " ".join("%.1f" % x for x in 100 * tot / tot.sum()))
