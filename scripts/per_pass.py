"""Per-pass view of the last batch: k_pull duration (kernel trace) beside its
HBM bytes (PMC FETCH_SIZE x read factor, WRITE_SIZE), in launch order.

python scripts/per_pass.py <kernel_trace.csv> <fetch.csv> <write.csv> [read_factor]
The three runs execute the same launch sequence, so the i-th k_pull of each
file is the same pass."""
import csv
import sys


def pulls_trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_pull" in r["Kernel_Name"]]


def pulls_pmc(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and "k_pull" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) * 1024.0 for r in rows]


def main():
    tr, fe, wr = pulls_trace(sys.argv[1]), pulls_pmc(sys.argv[2], "FETCH_SIZE"), pulls_pmc(sys.argv[3], "WRITE_SIZE")
    factor = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
    n = 24
    tr, fe, wr = tr[-n:], fe[-n:], wr[-n:]
    print("pass   us    read_GB  write_GB  TB/s")
    tot_t = tot_b = 0.0
    for i, (t, f, w) in enumerate(zip(tr, fe, wr)):
        b = f * factor + w
        tot_t += t
        tot_b += b
        print("%3d %8.0f %8.2f %8.2f %6.2f" % (i, t, f * factor / 1e9, w / 1e9, b / (t * 1e-6) / 1e12 if t > 0 else 0))
    print("total %.2f ms, %.1f GB, %.2f TB/s" % (tot_t / 1e3, tot_b / 1e9, tot_b / (tot_t * 1e-6) / 1e12))


if __name__ == "__main__":
    main()
