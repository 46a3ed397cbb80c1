"""Per-kernel totals and the per-bucket sequence of a rocprofv3 kernel trace
(scripts/c3_probe.py): which buckets cost what, and where the time goes."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("void ", "").replace("gs::(anonymous namespace)::", "").split("(")[0]
# keep the timed batch: everything after the last k_seed but one (warm-up first)
seeds = [i for i, r in enumerate(rows) if "k_seed" in r["Kernel_Name"]]
start = seeds[-1] if seeds else 0
ev = [i for i, r in enumerate(rows[:start]) if "k_offline_range" in r["Kernel_Name"]]
if ev:
    start = ev[-1]
rows = rows[start:]
tot = collections.Counter()
cnt = collections.Counter()
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[short(r["Kernel_Name"])] += d
    cnt[short(r["Kernel_Name"])] += 1
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print("span %.1f ms, kernel sum %.1f ms" % (span / 1e6, sum(tot.values()) / 1e6))
for k, v in tot.most_common(20):
    print("%-45s %6d calls %9.2f ms  avg %8.1f us" % (k, cnt[k], v / 1e6, v / cnt[k] / 1e3))
# per-bucket sequence: (scan, frontier, gossip) per launch
seq = []
cur = {}
for r in rows:
    n = short(r["Kernel_Name"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n.startswith("k_scan"):
        if cur:
            seq.append(cur)
        cur = {"scan": d}
    elif n.startswith("k_frontier"):
        cur["front"] = cur.get("front", 0) + d
    elif n.startswith("k_gossip<"):
        cur["gossip"] = cur.get("gossip", 0) + d
if cur:
    seq.append(cur)
print("buckets", len(seq))
for i, b in enumerate(seq):
    print("%4d scan %8.1f front %8.1f gossip %8.1f" % (i, b.get("scan", 0), b.get("front", 0), b.get("gossip", 0)))
