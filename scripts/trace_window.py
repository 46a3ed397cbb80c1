"""Kernel time inside a marked run (bench.py config_rates under GS_CFG_MARK=1).

python scripts/trace_window.py <kernel_trace.csv> <log with {"mark": ...} lines> [config name]

Prints, for the first timed run of the config: wall span, summed kernel
time per kernel (busy time on the GPU, overlapping streams counted once per
kernel), the time no kernel ran (host gaps: set-up, syncs, copies) and the
longest gaps with the kernel that preceded each."""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402


def main():
    trace, log = sys.argv[1], sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else None
    span = None
    for x in open(log):
        if x.startswith('{"mark"'):
            m = json.loads(x)
            if name is None or m["mark"] == name:
                span = (m["t0_ns"], m["t1_ns"])
                name = m["mark"]
                break
    if span is None:
        sys.exit("no mark")
    ks = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if span[0] <= t0 <= span[1]:
                ks.append((t0, t1, short(r["Kernel_Name"])))
    ks.sort()
    per = defaultdict(lambda: [0, 0])
    busy, gaps, end = 0, [], span[0]
    prev = "(start)"
    for t0, t1, k in ks:
        per[k][0] += 1
        per[k][1] += t1 - t0
        if t0 > end:
            gaps.append((t0 - end, prev, k))
            busy_start = t0
        else:
            busy_start = end
        if t1 > end:
            busy += t1 - busy_start
            end = t1
        prev = k
    wall = span[1] - span[0]
    print("%s: wall %.3f ms, kernels busy %.3f ms, no kernel running %.3f ms, %d dispatches" %
          (name, wall / 1e6, busy / 1e6, (wall - busy) / 1e6, len(ks)))
    for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:15]:
        print("  %-60s %5d x %9.1f us = %8.3f ms" % (k[:60], n, t / n / 1e3, t / 1e6))
    print("longest gaps:")
    for g, a, b in sorted(gaps, reverse=True)[:12]:
        print("  %8.1f us  after %-40s before %s" % (g / 1e3, a[:40], b[:40]))


if __name__ == "__main__":
    main()
