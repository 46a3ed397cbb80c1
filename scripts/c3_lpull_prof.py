"""Diagnostic: k_lpull shader clocks per section for config #3 (churn list
pass), GS_PULL_PROF build (scripts/pull_prof.sh build). Passes >= 31 are
summed in the last row. Slots: 0 skipped rows, 1 header + entries + records,
2 IHAVE step, 3 classify, 4 list appends, 5 emit, 6 row state, 7 rows."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
import gossipsim  # noqa: E402

gossipsim.LIB_PATH = os.path.join(ROOT, "prof_build", "libgossipsim.so")
peers = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
L = gossipsim.lib()
L.gs_debug_pull_prof.argtypes = [ctypes.c_void_p]
sim = gossipsim.Simulator(peers=peers, batch=1024, fragments=1, seed=1, lazy_gossip=1, churn_ppm=10_000, churn_down=10,
                          churn_horizon=16, heartbeat_ns=1_000_000_000,
                          hb_phase_ns=gossipsim.T0_NS - 20 * 1_000_000_000 + 370_000_000)
sim.set_topogen_links(5, 50, 150, 40, 130)
sim.connect_gossipsub_peers()
sim.mesh_converge(400)
sim.run(gossipsim.shard_messages(0, 0, 1, 1024, peers, 15000), collect=False)
buf = np.zeros(32 * 8, dtype=np.uint64)
L.gs_debug_pull_prof(buf.ctypes.data)
sim.run(gossipsim.shard_messages(1, 0, 1, 1024, peers, 15000), collect=False)
L.gs_debug_pull_prof(buf.ctypes.data)
b = buf.reshape(32, 8).astype(np.float64)
names = ["skip", "ent+rec", "ihave", "classify", "append", "emit", "state"]
print("pass " + " ".join("%8s%%" % n for n in names) + "  active_rows   Gclk")
for p in range(32):
    t = b[p, :7].sum()
    if t == 0:
        continue
    print("%4d " % p + " ".join("%9.1f" % (100 * b[p, k] / t) for k in range(7)) + "  %11d %6.2f" % (int(b[p, 7]), t / 1e9))
tot = b[:, :7].sum(0)
print("all  " + " ".join("%9.1f" % x for x in 100 * tot / tot.sum()) + "  %6.2f Gclk" % (tot.sum() / 1e9))
