"""Debug: churn list pass vs oracle on one small case; prints mismatching lanes."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "dst-libp2p-test-node_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "oracle"))
import numpy as np
import gossipsim, oracle
T0 = gossipsim.T0_NS
kw = dict(churn_ppm=20000, lazy_gossip=int(os.environ.get("G", 0)), fragments=1, hb_phase_ns=gossipsim.SHADOW_START_NS)
p = oracle.params(peers=700, seed=51, **kw)
M = 24
t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
sched = (t, (6 + np.arange(M)) % 700, np.full(M, 15000))
ref = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
for chl in ("1", "0"):
    os.environ["GS_CHURN_LIST"] = chl
    k = {n: getattr(p, n) for n, _ in oracle.OrParams._fields_}
    k["batch"] = 8
    sim = gossipsim.Simulator(**k)
    sim.set_topogen_links(5, 50, 150, 40, 130)
    sim.connect_gossipsub_peers()
    sim.mesh_converge(400)
    res = sim.run(sched)
    st = sim.stats()
    d = np.argwhere(res["t_complete"] != ref["t_complete"])
    print("CHURN_LIST", chl, "mismatches", len(d), {x: st[x] for x in ("deliveries", "list_pull_batches", "relaxations")}, ref["stats"]["deliveries"], ref["stats"]["relaxations"])
    hb = p.heartbeat_ns; ph = p.hb_phase_ns
    for m, u in d[:20]:
        g, o = int(res["t_complete"][m, u]), int(ref["t_complete"][m, u])
        tp = int(t[m]); q0 = (tp - ph) // hb
        def rel(x): return None if x == 2**64 - 1 else (x - tp) / 1e6
        ea = None if g == 2**64 - 1 else (g - ph) // hb
        print(" m", m, "u", u, "gpu", rel(g), "hops", res["hops"][m, u], "oracle", rel(o), ref["hops"][m, u],
              "q0", q0, "epoch(gpu)", ea, "off(u,ea)", None if ea is None else oracle.offline(p, u, ea) if hasattr(oracle, "offline") else "?")
    sim.close()
