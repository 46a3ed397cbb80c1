"""Shadow-parity harness: per-message latency percentiles of a Shadow run of the
reference nodes against the simulator on the same experiment (BASELINE.json
north_star's second check: p50 / p95 / max within +-5 % at 100-1k peers).

The reference pipeline is `shadow shadow.yaml` -> `grep -rne 'milliseconds\\|BW'
shadow.data/ > latencies<i>` -> `awk -f summary_latency*.awk latencies<i>`
(shadow/run.sh:58-74). This module reads that grep file:

    shadow.data/hosts/<host>/<proc>.stdout:<line>:<tx_time> milliseconds: <ms>

one line per (peer, message) completion (rust-test-node/src/main.rs:93; go
main.go:49), where <host> is `peer<id>` (what summary_latency*.awk:17 splits)
or `pod-<id>` (what shadow/topogen.py names its hosts, defect D3); BW and other
lines are skipped as the awk scripts skip them (summary_latency_large.awk:11-13).

Messages are identified by tx_time (the awk scripts' key, arr[4]); the publish
schedule is rebuilt from the log itself: t_pub = tx_time (the node stamps it at
the publish, main.rs:105-111) and the publisher is the one peer with no line
for that message (rust does not log its own message), or the injector rule of
shadow.yaml (gs_shadow_injector, topogen.py:125-136) when that is ambiguous.

Percentiles use the simulator's nearest-rank rule (gs_msg_summary: the value at
rank ceil(q * n) of the sorted latencies), so a perfect simulator scores 0.

    python shadow_parity.py --latencies latencies1 --yaml shadow.yaml \\
        --gml network_topology.gml --peers 100 --msg-size 15000 [--json out.json]

The simulation itself runs on the GPU through the C ABI (gossipsim.Simulator,
run(summary=True): the percentiles come from the device's gs_msg_summary).
"""
import argparse
import json
import re
import sys

import numpy as np

LINE = re.compile(rb"hosts/(?:peer|pod-?)(\d+)/[^:\n]*:\d+:(\d+) milliseconds: (\d+)\s*$")


def read_latencies(path):
    """grep file -> {tx_time: (peer ids int64[n], latency ms int64[n])}, lines in file order."""
    per = {}
    with open(path, "rb") as f:
        for raw in f:
            m = LINE.search(raw)
            if not m:
                continue  # BW lines, heartbeat lines, anything the awk scripts drop
            host, tx, ms = int(m.group(1)), int(m.group(2)), int(m.group(3))
            p = per.setdefault(tx, ([], []))
            p[0].append(host)
            p[1].append(ms)
    return {tx: (np.asarray(h, np.int64), np.asarray(ms, np.int64)) for tx, (h, ms) in per.items()}


def nearest_rank(sorted_ms, num, den):
    """Value at rank ceil(num/den * n) (1-based) of an ascending array (gs_msg_summary's rule)."""
    n = len(sorted_ms)
    if n == 0:
        return None
    k = (num * n + den - 1) // den
    return int(sorted_ms[max(k, 1) - 1])


def summarize(per_msg):
    """{tx: (hosts, ms)} -> {tx: {"n", "p50", "p95", "max", "sum"}}."""
    out = {}
    for tx, (_, ms) in per_msg.items():
        s = np.sort(ms)
        out[tx] = {"n": int(len(s)), "p50": nearest_rank(s, 50, 100), "p95": nearest_rank(s, 95, 100),
                   "max": int(s[-1]) if len(s) else None, "sum": int(s.sum())}
    return out


def infer_publishers(per_msg, peers, self_log=False):
    """Publisher of each message: the one peer in [0, peers) with no line for it
    (rust / nim without SELFTRIGGER: the publisher logs nothing). -> {tx: id or None}."""
    out = {}
    for tx, (hosts, _) in per_msg.items():
        if self_log:
            out[tx] = None
            continue
        seen = np.zeros(peers, bool)
        seen[hosts[(hosts >= 0) & (hosts < peers)]] = True
        miss = np.flatnonzero(~seen)
        out[tx] = int(miss[0]) if len(miss) == 1 else None
    return out


def schedule_from_log(per_msg, peers, msg_size, publisher_id=None, rotation=0, self_log=False):
    """(t_pub, publisher, msg_size) arrays, messages in tx_time order. Publishers
    the log cannot name (a self-logging node, or a peer that also missed the
    message) come from run.sh's rule publisher_id + i * rotation mod peers
    (run.sh:34-36; the injector, traffic_sync.py, is not part of the reference)."""
    txs = sorted(per_msg)
    pubs = infer_publishers(per_msg, peers, self_log)
    pub = []
    for i, tx in enumerate(txs):
        p = pubs[tx]
        if p is None:
            if publisher_id is None:
                raise ValueError("publisher of message tx_time=%d is ambiguous in the log; give --publisher-id" % tx)
            p = (publisher_id + i * rotation) % peers
        pub.append(p)
    return (np.asarray(txs, np.uint64), np.asarray(pub, np.uint32), np.full(len(txs), msg_size, np.uint32))


def sim_summary(summary, sched):
    """Simulator.run(summary=True)["summary"] -> the summarize() layout keyed by t_pub."""
    out = {}
    for i, tx in enumerate(np.asarray(sched[0]).tolist()):
        out[int(tx)] = {"n": int(summary["delivered"][i]), "p50": int(summary["p50_ms"][i]),
                        "p95": int(summary["p95_ms"][i]), "max": int(summary["max_ms"][i]),
                        "sum": int(summary["lat_sum_ms"][i])}
    return out


def compare(shadow, sim, tol=0.05):
    """Per-message relative errors (sim - shadow) / shadow of p50, p95, max (0
    when both are 0), plus the awk scripts' aggregates (mean of per-message max
    = "Average Max Message Dissemination Latency", mean latency); pass = every
    |error| <= tol."""
    rows, worst = [], {"p50": 0.0, "p95": 0.0, "max": 0.0}
    for tx in sorted(shadow):
        a, b = shadow[tx], sim.get(tx)
        if b is None:
            raise ValueError("message tx_time=%d is in the Shadow log but not simulated" % tx)
        r = {"tx_time": tx, "n_shadow": a["n"], "n_sim": b["n"]}
        for k in ("p50", "p95", "max"):
            x, y = a[k], b[k]
            e = 0.0 if x == y else (float("inf") if not x else (y - x) / x)
            r[k] = (x, y, e)
            worst[k] = max(worst[k], abs(e))
        rows.append(r)
    m = len(rows)
    avg_max_sh = sum(shadow[t]["max"] for t in shadow) / max(m, 1)
    avg_max_sim = sum(sim[t]["max"] for t in shadow) / max(m, 1)
    mean_sh = sum(shadow[t]["sum"] for t in shadow) / max(1, sum(shadow[t]["n"] for t in shadow))
    mean_sim = sum(sim[t]["sum"] for t in shadow) / max(1, sum(sim[t]["n"] for t in shadow))
    rel = lambda x, y: 0.0 if x == y else (float("inf") if not x else (y - x) / x)
    return {"messages": m, "tol": tol, "worst_abs_rel_err": worst,
            "avg_max_latency_ms": {"shadow": avg_max_sh, "sim": avg_max_sim, "rel_err": rel(avg_max_sh, avg_max_sim)},
            "mean_latency_ms": {"shadow": mean_sh, "sim": mean_sim, "rel_err": rel(mean_sh, mean_sim)},
            "deliveries": {"shadow": sum(shadow[t]["n"] for t in shadow), "sim": sum(sim[t]["n"] for t in shadow)},
            "pass": all(v <= tol for v in worst.values()),
            "per_message": rows}


def run(args):
    import gossipsim
    per = read_latencies(args.latencies)
    if not per:
        raise SystemExit("no arrival lines in %s" % args.latencies)
    inj = gossipsim.shadow_injector(args.yaml) if args.yaml else None
    msg_size = args.msg_size or (inj["msg_size"] if inj else 15000)
    kw = {"peers": args.peers, "fragments": args.fragments, "seed": args.seed, "batch": max(1, len(per))}
    if args.node:
        kw["node"] = gossipsim.NODES[args.node]
    sched = schedule_from_log(per, args.peers, msg_size, args.publisher_id, args.rotation,
                              self_log=args.node == "nim")
    sim = gossipsim.Simulator(**kw)
    if args.gml:
        sim.set_shadow_links(args.gml, args.yaml, shortest=args.shortest)
    else:
        S, bl, bh, ll, lh = [int(x) for x in args.topogen.split(",")]
        sim.set_topogen_links(S, bl, bh, ll, lh, shortest=args.shortest)
    sim.connect_gossipsub_peers()
    sim.mesh_converge()
    res = sim.run(sched, collect=False, summary=True)
    rep = compare(summarize(per), sim_summary(res["summary"], sched), args.tol)
    rep["config"] = {"peers": args.peers, "msg_size": msg_size, "fragments": args.fragments, "seed": args.seed,
                     "links": args.gml or args.topogen, "latencies": args.latencies}
    return rep


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--latencies", required=True, help="grep -rne 'milliseconds\\|BW' shadow.data/ output")
    ap.add_argument("--peers", type=int, required=True)
    ap.add_argument("--yaml", help="shadow.yaml (injector args, host placement with --gml)")
    ap.add_argument("--gml", help="Shadow network graph (topogen's GML)")
    ap.add_argument("--topogen", default="1,50,50,100,100", help="stages,bl,bh,ll,lh when no --gml")
    ap.add_argument("--shortest", action="store_true", help="Shadow use_shortest_path latencies")
    ap.add_argument("--msg-size", type=int, default=0)
    ap.add_argument("--fragments", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--node", choices=("rust", "go", "nim"), default="rust")
    ap.add_argument("--publisher-id", type=int, help="run.sh publisher_id (when the log cannot name one)")
    ap.add_argument("--rotation", type=int, default=0, help="run.sh publisher_rotation")
    ap.add_argument("--tol", type=float, default=0.05)
    ap.add_argument("--json", help="write the full report here")
    args = ap.parse_args(argv)
    rep = run(args)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rep, f, indent=1, default=float)
    short = {k: v for k, v in rep.items() if k != "per_message"}
    print(json.dumps(short, default=float))
    return 0 if rep["pass"] else 1


if __name__ == "__main__":
    sys.exit(main())
