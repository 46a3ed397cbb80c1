"""Per-dispatch durations of the bucket kernels from a rocprofv3 --kernel-trace CSV
(the last step of a bench run): one line per pass / bucket, in launch order."""
import csv
import sys


def main(path, pat=("k_pull", "k_scan", "k_frontier", "k_complete", "k_seed")):
    rows = list(csv.DictReader(open(path)))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
          if any(p in r["Kernel_Name"] for p in pat)]
    ks.sort(key=lambda x: x[1])
    seeds = [i for i, k in enumerate(ks) if "k_seed" in k[0]]
    last = ks[seeds[-1]:]  # the last batch
    tot = {}
    for name, s, e in last:
        short = name.split("(")[0].split("<")[0].split("::")[-1]
        tot[short] = tot.get(short, 0) + (e - s) / 1e3
        print("%-14s %9.1f us" % (short, (e - s) / 1e3))
    print("batch wall %.1f us" % ((last[-1][2] - last[0][1]) / 1e3), {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main(sys.argv[1])
