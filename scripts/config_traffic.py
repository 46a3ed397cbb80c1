"""Per-config HBM traffic from scripts/config_pmc.sh's counter files.

python scripts/config_traffic.py <pmc dir> <out json> [--read-factor F]

For each config of bench.py's configs_1gpu: FETCH_SIZE (x the read factor,
MI355X_MICROARCH.md's gfx950 correction; the default is the factor
calibrated on k_complete in profiles/traffic_latest.json) + WRITE_SIZE, in
bytes:
  - per launch of the window-pass kernel (every k_lpull / k_pull template of
    the run, launches pooled): bench.py's configs_1gpu roofline.traffic;
  - per batch over every kernel of the run (epoch steps, gossip senders,
    completion ...), beside the config's algorithmic bytes per batch.
Only the kernels of the config's first timed run count (bench.py config_rates
prints its CLOCK_MONOTONIC span under GS_CFG_MARK=1; rocprofv3's timestamps
are on that clock), so graph set-up, mesh convergence and warm-up stay out."""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path, counter, span=None):
    """bytes per kernel name; with span = (t0, t1) only dispatches starting inside it"""
    per = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            if span and not span[0] <= int(r["Start_Timestamp"]) <= span[1]:
                continue
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return per


def mark(log, name):
    """the first timed run's CLOCK_MONOTONIC span (bench.py config_rates under GS_CFG_MARK=1)"""
    try:
        for x in open(log):
            if x.startswith('{"mark"'):
                m = json.loads(x)
                if m["mark"] == name:
                    return m["t0_ns"], m["t1_ns"]
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--read-factor", type=float)
    a = ap.parse_args()
    factor = a.read_factor
    src = "command line"
    if factor is None:
        tj = json.load(open(os.path.join(ROOT, "profiles", "traffic_latest.json")))
        factor, src = tj["read_factor"], "profiles/traffic_latest.json (" + tj["calibration"] + ")"
    sys.path.insert(0, ROOT)
    import bench  # noqa: E402  (config shapes only; nothing runs)
    res = {"read_factor": factor, "read_factor_source": src, "configs": {}}
    for name, c in bench.CONFIGS.items():
        fdir, wdir = (os.path.join(a.dir, "%s_%s" % (name, k)) for k in ("FETCH_SIZE", "WRITE_SIZE"))
        files = []
        for d in (fdir, wdir):
            hit = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
            files.append(hit[0] if hit else None)
        if not all(files):
            continue
        spans = [mark(os.path.join(a.dir, "%s_%s.log" % (name, k)), name) for k in ("FETCH_SIZE", "WRITE_SIZE")]
        timed = all(spans)
        fe, wr = load(files[0], "FETCH_SIZE", spans[0]), load(files[1], "WRITE_SIZE", spans[1])
        kern = {}
        for k in sorted(set(fe) | set(wr)):
            f, w = fe.get(k, []), wr.get(k, [])
            kern[k] = {"launches": max(len(f), len(w)), "bytes": sum(f) * factor + sum(w)}
        rel = [k for k in kern if k.startswith("k_lpull<")] or [k for k in kern if k.startswith("k_pull<")]
        nl = sum(kern[k]["launches"] for k in rel)
        nb = -(-c["msgs"] // c["batch"])
        batches = nb if timed else 1 + (c.get("reps", 1) + 1) * nb
        tot = sum(v["bytes"] for v in kern.values())
        log = os.path.join(a.dir, "%s_FETCH_SIZE.log" % name)
        alg = None
        try:
            line = [x for x in open(log) if x.startswith("{") and not x.startswith('{"mark"')][-1]
            alg = json.loads(line)[name].get("alg_bytes_per_batch")
        except (OSError, IndexError, ValueError, KeyError):
            pass
        top = sorted(kern.items(), key=lambda kv: -kv[1]["bytes"])[:6]
        res["configs"][name] = {
            "pass_kernels": rel, "pass_launches": nl,
            "hbm_bytes_per_launch": (sum(kern[k]["bytes"] for k in rel) / nl) if nl else None,
            "scope": "the first timed run (kernels starting inside its clock span)" if timed else
                     "the whole process (setup, warm-up and every run)",
            "batches": batches, "hbm_bytes_per_batch_all_kernels": tot / batches,
            "alg_bytes_per_batch": alg, "ratio_all_kernels_to_alg": (tot / batches / alg) if alg else None,
            "top_kernels_bytes_per_batch": {k: v["bytes"] / batches for k, v in top},
            "source": os.path.relpath(files[0], ROOT) + " + " + os.path.relpath(files[1], ROOT)}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
