"""Wall time covered by each kernel family in a rocprofv3 kernel trace (union
of intervals), over the whole trace: which family is on the critical path of a
multi-stream (loop-back parts) run."""
import csv
import re
import sys


def union(iv):
    iv.sort()
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ((ce - cs) if ce is not None else 0)


rows = list(csv.DictReader(open(sys.argv[1])))
fam = {}
for r in rows:
    n = re.sub(r"gs::\(anonymous namespace\)::", "", r["Kernel_Name"])
    n = re.sub(r"^void ", "", n)
    n = re.split(r"[<(]", n)[0]
    fam.setdefault(n, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
allv = [x for v in fam.values() for x in v]
t0 = min(s for s, _ in allv)
t1 = max(e for _, e in allv)
print("span %.1f ms, any kernel %.1f ms" % ((t1 - t0) / 1e6, union(list(allv)) / 1e6))
for n, v in sorted(fam.items(), key=lambda kv: -union(list(kv[1]))):
    u = union(list(v))
    if u > 1e5:
        print("%-28s calls %6d  union %8.1f ms  sum %8.1f ms" % (n, len(v), u / 1e6, sum(e - s for s, e in v) / 1e6))
