"""Per-dispatch durations of the last batch of a rocprofv3 kernel trace (k_seed .. k_complete)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_default/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
ks = sorted([(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows],
            key=lambda x: x[1])
seeds = [i for i, k in enumerate(ks) if "k_seed" in k[0]]
last = ks[seeds[-1]:]
KN = ("k_lpull", "k_lseed", "k_lcomplete", "k_lfinal", "k_lpub", "k_pull", "k_scan", "k_frontier", "k_complete", "k_seed")
short = lambda n: next((k for k in KN if k in n), n[:12])
print(" ".join("%s:%.0f" % (short(n).replace("k_", ""), (e - s) / 1e3) for n, s, e in last if "copyBuf" not in n))
tot = {}
for n, s, e in last:
    tot[short(n)] = tot.get(short(n), 0) + (e - s) / 1e6
print("ms:", {k: round(v, 2) for k, v in tot.items()}, "batch wall %.2f" % ((last[-1][2] - last[0][1]) / 1e6))
