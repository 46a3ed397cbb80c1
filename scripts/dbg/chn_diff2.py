"""Debug: churn list pass vs push path at config #3 shape; oracle on the mismatching messages."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "dst-libp2p-test-node_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "oracle"))
import numpy as np
import gossipsim, oracle
T0 = gossipsim.T0_NS
N = int(os.environ.get("N", 10000)); M = int(os.environ.get("M", 256))
p = oracle.params(peers=N, seed=3, lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                  hb_phase_ns=T0 - 20 * 1_000_000_000 + 370_000_000)
t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
sched = (t, (6 + np.arange(M)) % N, np.full(M, 15000))
out = []
for chl in ("1", "0"):
    os.environ["GS_CHURN_LIST"] = chl
    k = {n: getattr(p, n) for n, _ in oracle.OrParams._fields_}
    k["batch"] = M
    sim = gossipsim.Simulator(**k)
    sim.set_topogen_links(5, 50, 150, 40, 130)
    sim.connect_gossipsub_peers()
    sim.mesh_converge(400)
    res = sim.run(sched)
    out.append((res, sim.stats()))
    sim.close()
(a, sa), (b, sb) = out
d = np.argwhere((a["t_complete"] != b["t_complete"]) | (a["hops"] != b["hops"]))
print("mismatches", len(d), sa["gossip_iwant"], sb["gossip_iwant"], sa["deliveries"], sb["deliveries"])
ms = sorted(set(int(m) for m, u in d))[:6]
if ms:
    sub = (t[ms], sched[1][ms], sched[2][ms])
    ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sub)
    for m, u in d[:30]:
        i = ms.index(int(m)) if int(m) in ms else None
        if i is None: continue
        tp = int(t[m]); f = lambda x: None if x == 2**64 - 1 else (int(x) - tp) / 1e6
        print(" m", m, "u", u, "list", f(a["t_complete"][m, u]), a["hops"][m, u], "push", f(b["t_complete"][m, u]),
              b["hops"][m, u], "oracle", f(ref["t_complete"][i, u]), ref["hops"][i, u])
