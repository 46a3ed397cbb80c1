"""Config #3 (100k peers, heterogeneous links, lazy gossip, churn) with
gs_set_traffic on: writes the Shadow tracker heartbeat report that
shadow/summary_shadowlog.awk reads, and the node metrics, gzipped under OUT (default
gpurun_out/c3_traffic/). Prints the traffic totals and the run time with and
without the traffic passes as one JSON line.

    python scripts/c3_traffic.py [--msgs 1024] [--out gpurun_out/c3_traffic]
"""
import argparse
import gzip
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))
sys.path.insert(0, ROOT)
import gossipsim  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1024)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c3_traffic"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    c = CONFIGS["c3_100k_gossip_churn"]
    sim = gossipsim.Simulator(peers=c["peers"], batch=c["batch"], fragments=c["fragments"], seed=1, **c["knobs"])
    sim.set_topogen_links(c["links"][0], *c["links"][1:])
    sim.connect_gossipsub_peers()
    sim.mesh_converge(400)
    sched = gossipsim.shard_messages(1, 0, 1, a.msgs, c["peers"], 15000)
    t0 = time.perf_counter()
    sim.run(sched, collect=False)
    plain = time.perf_counter() - t0
    st0 = sim.stats()
    sim.set_traffic(True)  # zeroes the counters
    sim.reset_stats()
    t0 = time.perf_counter()
    sim.run(sched, collect=False)
    with_tr = time.perf_counter() - t0
    st = sim.stats()
    tr = sim.traffic()
    assert st["deliveries"] == st0["deliveries"]
    # the reports of 100k peers are tens of MB: keep them gzipped (zcat | awk)
    for name, write in (("shadow_heartbeat.log", lambda f: gossipsim.write_shadow_heartbeat(f, tr)),
                        ("metrics.txt", sim.write_node_metrics)):
        tmp = os.path.join(a.out, name)
        write(tmp)
        with open(tmp, "rb") as fi, gzip.open(tmp + ".gz", "wb") as fo:
            shutil.copyfileobj(fi, fo)
        os.remove(tmp)
    s = lambda k: int(tr[:, gossipsim.TRAFFIC_COLS.index(k)].sum())
    print(json.dumps({
        "config": "c3_100k_gossip_churn", "msgs": a.msgs, "deliveries": int(st["deliveries"]),
        "gossip_iwant": int(st["gossip_iwant"]), "run_ms": plain * 1e3, "run_ms_with_traffic": with_tr * 1e3,
        **{k: s(k) for k in gossipsim.TRAFFIC_COLS}}), flush=True)


if __name__ == "__main__":
    main()
