"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

python scripts/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
       <out_summary.json> [--traffic-json profiles/traffic_latest.json --peers N --batch B]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch. On gfx950 FETCH_SIZE reports
half the bytes of a coalesced streaming read (MI355X_MICROARCH.md, HBM
section); we calibrate that factor on a kernel of our own whose reads are
known exactly: k_complete streams every key once per batch (8 B x peers x
batch x FP, 8-byte lanes, the same access width as the pull pass's row reads),
or, on the push path, k_scan per non-empty bucket. The same factor is applied
to every kernel's FETCH_SIZE ("corrected"); WRITE_SIZE is taken as is. The
traffic json carries the relaxation kernel's bytes per launch (k_lpull,
k_pull, or k_scan + k_frontier) for bench.py's roofline.traffic. With the
list pull path, profile under GS_LPULL_DENSE=1 so that k_complete runs.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = name.split("(")[0].replace("void ", "").strip()
    return name.split("::")[-1] if "<" not in name else name[name.rfind("::", 0, name.find("<")) + 2:]


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--traffic-json")
    ap.add_argument("--peers", type=int)
    ap.add_argument("--batch", type=int)
    ap.add_argument("--buckets", type=int, help="non-empty buckets in the profiled run (k_scan calibration)")
    ap.add_argument("--fp", type=int, default=1, help="fragment lanes per message (k_complete calibration)")
    a = ap.parse_args()
    fe, wr = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    factor, calib = 2.0, "guide value (x2 on streaming reads)"
    scan = [k for k in fe if k.startswith("k_scan<")]
    comp = [k for k in fe if k.startswith("k_complete<")]
    if comp and a.peers and a.batch:
        known = 8.0 * a.peers * a.batch * a.fp * len(fe[comp[0]])
        got = sum(fe[comp[0]]) * 1024.0
        factor, calib = known / got, "k_complete: %d launches x %d peers x %d msgs x %d lanes x 8 B / FETCH_SIZE" % (
            len(fe[comp[0]]), a.peers, a.batch, a.fp)
    elif scan and a.peers and a.batch and a.buckets:
        known = 8.0 * a.peers * a.batch * a.buckets
        got = sum(fe[scan[0]]) * 1024.0
        factor, calib = known / got, "k_scan: %d buckets x %d peers x %d msgs x 8 B / FETCH_SIZE" % (
            a.buckets, a.peers, a.batch)
    out = {"read_factor": factor, "calibration": calib, "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f, w = fe.get(k, []), wr.get(k, [])
        n = max(len(f), len(w))
        fm = sum(f) / len(f) * 1024.0 if f else 0.0
        wm = sum(w) / len(w) * 1024.0 if w else 0.0
        out["kernels"][k] = {"launches": n, "fetch_bytes_raw_mean": fm, "write_bytes_mean": wm,
                             "hbm_bytes_per_launch_corrected": fm * factor + wm}
    json.dump(out, open(a.out, "w"), indent=1)
    if a.traffic_json:
        rel = [k for k in out["kernels"] if k.startswith("k_lpull<")] or \
            [k for k in out["kernels"] if k.startswith("k_pull<")] or \
            [k for k in out["kernels"] if k.startswith("k_scan<") or k.startswith("k_frontier<")]
        launches = max(out["kernels"][k]["launches"] for k in rel)
        per_launch = sum(out["kernels"][k]["hbm_bytes_per_launch_corrected"] for k in rel)
        json.dump({"peers": a.peers, "batch": a.batch, "kernels": rel, "launches": launches,
                   "hbm_bytes_per_launch": per_launch, "read_factor": factor, "calibration": calib,
                   "source": a.fetch + " + " + a.write}, open(a.traffic_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
