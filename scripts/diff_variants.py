"""Diagnostic: run the same batch with two GS_RELAX_VARIANT values (lazy gossip
off, so no push-path fallback can hide a difference) and report where the
completion times / hops differ. python scripts/diff_variants.py [peers] [batch] [vA] [vB]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
import gossipsim  # noqa: E402

peers = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
va, vb = (sys.argv[3], sys.argv[4]) if len(sys.argv) > 4 else ("45", "109")
sim = gossipsim.Simulator(peers=peers, batch=B, fragments=1, seed=1, device=0, lazy_gossip=0)
sim.set_topogen_links(5, 50, 150, 40, 130)
sim.connect_gossipsub_peers()
sim.mesh_converge(400)
sched = gossipsim.shard_messages(0, 0, 1, B, peers, 15000)
out = {}
for v in (va, vb):
    os.environ["GS_RELAX_VARIANT"] = v
    blocks = []
    sim.run(sched, on_block=lambda f, t, h: blocks.append((f, t.copy(), h.copy())), block_msgs=64)
    out[v] = blocks
    print("variant", v, sim.stats(), flush=True)
nd = 0
for (fa, ta, ha), (fb, tb, hb) in zip(out[va], out[vb]):
    bad = (ta != tb) | (ha != hb)
    if bad.any():
        m, u = np.nonzero(bad)
        nd += bad.sum()
        for k in range(min(5, len(m))):
            print("msg %d peer %d: %s t=%d h=%d | %s t=%d h=%d" % (fa + m[k], u[k], va, ta[m[k], u[k]], ha[m[k], u[k]],
                                                                  vb, tb[m[k], u[k]], hb[m[k], u[k]]))
print("differing (msg, peer) pairs:", nd)
