"""HBM traffic per kernel of one config #3 batch from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) over scripts/prof_c3.py or scripts/c3_probe.py:

    python scripts/c3_pmc.py <fetch counter_collection.csv> <write counter_collection.csv> [alg_bytes]

Only the timed batch is kept (dispatches from the last k_offline_range on, the
start of its churn epochs; the warm-up batch runs before it). FETCH_SIZE is
doubled (MI355X_MICROARCH.md, HBM: gfx950 reports half the bytes of a wide
coalesced read; the random 8-B reads of these kernels are uncalibrated, so the
read side is an estimate), WRITE_SIZE taken as is. Prints GB per kernel and the
total against the batch's algorithmic bytes (gs_stats.bytes_alg) when given."""
import collections
import csv
import sys


def short(n):
    return n.replace("void ", "").replace("gs::(anonymous namespace)::", "").split("(")[0]


def load(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_offline_range" in r["Kernel_Name"]]
    rows = rows[starts[-1]:] if starts else rows
    per = collections.defaultdict(float)
    for r in rows:
        per[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024.0  # KB -> B
    return per


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    alg = float(sys.argv[3]) if len(sys.argv) > 3 else None
    names = sorted(set(f) | set(w), key=lambda k: -(2 * f.get(k, 0) + w.get(k, 0)))
    tot = 0.0
    print("%-40s %10s %10s %10s" % ("kernel", "read GB", "write GB", "total GB"))
    for k in names:
        r, x = 2 * f.get(k, 0.0), w.get(k, 0.0)
        tot += r + x
        if r + x > 1e7:
            print("%-40s %10.2f %10.2f %10.2f" % (k, r / 1e9, x / 1e9, (r + x) / 1e9))
    print("total %.1f GB per batch" % (tot / 1e9) + ("" if alg is None else ", %.1fx the %.2f GB algorithmic"
                                                      % (tot / alg, alg / 1e9)))


if __name__ == "__main__":
    main()
