"""Regenerate the golden fixtures under tests/golden/ (run in the build container only).

Sources of truth, all executed from /root/reference (never copied into the repo):
  * shadow/topogen.py (networkx + PyYAML): GML/YAML for several parameter sets ->
    topogen_*.json  (stage bandwidths, GML edge latencies, host -> stage map).
  * shadow/summary_latency.awk and summary_latency_large.awk: summaries of a
    synthetic arrival log in the reference's grep format -> awk_*.txt.
  * oracle/gs_oracle.c (this repo): small dissemination fixtures -> oracle_*.npz,
    a regression pin of the oracle across rounds (not a reference pin).

Usage: python tests/golden/make_golden.py
"""
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/shadow"

TOPOGEN_CASES = {
    # name: topogen flags
    "defaults": ["-n", "100"],
    "runsh_example": ["-n", "100", "-bl", "50", "-bh", "150", "-ll", "40", "-lh", "130",
                      "-st", "5", "-s", "15000", "-f", "1", "-m", "10", "-d", "1000"],
    "config1": ["-n", "1000", "-bl", "50", "-bh", "50", "-ll", "50", "-lh", "50", "-st", "1",
                "-s", "15000", "-f", "1", "-m", "100", "-d", "1000"],
    "seven_stages": ["-n", "50", "-bl", "10", "-bh", "1000", "-ll", "5", "-lh", "300",
                     "-st", "7", "-mx", "quic", "-f", "4"],
    "three_stages_tight": ["-n", "30", "-bl", "100", "-bh", "101", "-ll", "20", "-lh", "21",
                           "-st", "3"],
}


RAW_CASES = ("runsh_example", "seven_stages")


def parse_gml(path):
    """Minimal GML reader for topogen's output (nodes with bandwidth, edges with latency)."""
    text = open(path).read()
    nodes, edges = {}, []
    for blk in re.finditer(r"node \[(.*?)\]", text, re.S):
        b = blk.group(1)
        nid = int(re.search(r"id (\d+)", b).group(1))
        up = re.search(r'host_bandwidth_up "(\d+) Mbit"', b)
        dn = re.search(r'host_bandwidth_down "(\d+) Mbit"', b)
        nodes[nid] = (int(up.group(1)), int(dn.group(1)))
    for blk in re.finditer(r"edge \[(.*?)\]", text, re.S):
        b = blk.group(1)
        s = int(re.search(r"source (\d+)", b).group(1))
        t = int(re.search(r"target (\d+)", b).group(1))
        lat = int(re.search(r'latency "(\d+) ms"', b).group(1))
        loss = float(re.search(r"packet_loss ([0-9.eE+-]+)", b).group(1))
        edges.append((s, t, lat, loss))
    return nodes, edges


def topogen_fixtures():
    import yaml
    for name, flags in TOPOGEN_CASES.items():
        with tempfile.TemporaryDirectory() as d:
            subprocess.check_call([sys.executable, os.path.join(REF, "topogen.py")] + flags, cwd=d)
            nodes, edges = parse_gml(os.path.join(d, "network_topology.gml"))
            cfg = yaml.safe_load(open(os.path.join(d, "shadow.yaml")))
            if name in RAW_CASES:  # the generated files themselves, for the GML / shadow.yaml ingest tests
                for src, dst in (("network_topology.gml", "gml"), ("shadow.yaml", "yaml")):
                    with open(os.path.join(d, src)) as fi, open(os.path.join(HERE, "topogen_%s.%s" % (name, dst)),
                                                                "w") as fo:
                        fo.write(fi.read())
        hosts = cfg["hosts"]
        peers = [h for h in hosts if h != "pod-%d" % (len(hosts) - 1)]
        fx = {
            "flags": flags,
            "nodes": {str(k): v for k, v in sorted(nodes.items())},
            "edges": sorted(edges),
            "host_stage": [hosts["pod-%d" % i]["network_node_id"] for i in range(len(peers))],
            "controller": hosts["pod-%d" % len(peers)]["network_node_id"],
            "peer_env": hosts["pod-0"]["processes"][0]["environment"],
        }
        with open(os.path.join(HERE, "topogen_%s.json" % name), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
        print("wrote topogen_%s.json" % name)


# Synthetic arrivals in the format of rust-test-node/src/main.rs:93 as grep -rne prints them
# (shadow/run.sh:61). (peer, tx_time, ms). SURVEY Appendix B.5 plus a few more rows.
AWK_ARRIVALS = [
    (3, 1700000000000000000, 120),
    (7, 1700000000000000000, 230),
    (9, 1700000000000000000, 95),
    (12, 1700000001000000000, 310),
    (5, 1700000001000000000, 180),
    (5, 1700000002000000000, 1020),
    (11, 1700000002000000000, 640),
    (2, 1700000002000000000, 655),
]


def awk_fixtures():
    # the emitter groups by peer and numbers lines per peer; rebuild exactly that here
    per_peer = {}
    for peer, tx, ms in sorted(AWK_ARRIVALS, key=lambda r: (r[0], r[1])):
        per_peer.setdefault(peer, []).append((tx, ms))
    lines = []
    for peer in sorted(per_peer):
        for i, (tx, ms) in enumerate(per_peer[peer], 1):
            lines.append("shadow.data/hosts/peer%d/main.1000.stdout:%d:%d milliseconds: %d"
                         % (peer, i, tx, ms))
    bw = "shadow.data/hosts/peer3/main.1000.stdout:99:BW in 1234 out 5678"
    with open(os.path.join(HERE, "awk_arrivals.json"), "w") as f:
        json.dump(AWK_ARRIVALS, f)
    with open(os.path.join(HERE, "awk_latencies.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(HERE, "awk_latencies_bw.txt"), "w") as f:
        f.write("\n".join(lines + [bw]) + "\n")
    for script in ("summary_latency", "summary_latency_large"):
        for inp in ("awk_latencies", "awk_latencies_bw"):
            out = subprocess.check_output(["awk", "-f", os.path.join(REF, script + ".awk"),
                                           os.path.join(HERE, inp + ".txt")]).decode()
            with open(os.path.join(HERE, "%s__%s.txt" % (inp, script)), "w") as f:
                f.write(out)
            print("wrote %s__%s.txt" % (inp, script))


def oracle_fixtures():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cases = {
        # name: (params, stages, links(bl,bh,ll,lh), n_msgs, msg_size)
        "uniform_n300": (dict(peers=300, seed=1), 1, (50, 50, 50, 50), 6, 15000),
        "hetero_n400_f4": (dict(peers=400, seed=2, fragments=4), 5, (50, 150, 40, 130), 5, 15000),
        "nim_n200_cap": (dict(peers=200, seed=3, dial_extra=0, max_connections=14, d_out=3),
                         3, (20, 80, 30, 90), 4, 3000),
    }
    for name, (kw, S, links, M, size) in cases.items():
        p = oracle.params(**kw)
        # tx_time: injector start + 3 ms HTTP transit (gossipsim.T0_NS)
        t = 946684800_000_000_000 + 500_003_000_000 + np.arange(M, dtype=np.uint64) * 1_000_000_000
        pub = (6 + np.arange(M)) % p.peers
        r = oracle.simulate(p, S, links, sched=(t, pub, np.full(M, size)))
        np.savez_compressed(os.path.join(HERE, "oracle_%s.npz" % name),
                            row_ptr=r["row_ptr"], col=r["col"], flags=r["flags"], mesh=r["mesh"],
                            cnt=r["cnt"], t_complete=r["t_complete"], hops=r["hops"],
                            epochs=np.array([r["epochs"]]), sched_t=t, sched_pub=pub,
                            stats=np.array([r["stats"][k] for k in sorted(r["stats"])], np.uint64))
        with open(os.path.join(HERE, "oracle_%s.json" % name), "w") as f:
            json.dump(dict(params=kw, stages=S, links=links, n_msgs=M, msg_size=size,
                           stats=r["stats"], epochs=r["epochs"]), f, indent=1, sort_keys=True)
        print("wrote oracle_%s" % name, r["stats"])


if __name__ == "__main__":
    topogen_fixtures()
    awk_fixtures()
    oracle_fixtures()
