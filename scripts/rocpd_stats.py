"""Kernel stats (name, calls, total ms, avg us, %) from a rocprofv3 rocpd
SQLite database (the default output format of this rocprofv3), like the
--stats CSV. Usage: python scripts/rocpd_stats.py results.db [top_n] > stats.txt"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = db.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                  "order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
print("%-90s %8s %12s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "%"))
for name, n, s, a in rows[:top]:
    short = name if len(name) <= 90 else name[:87] + "..."
    print("%-90s %8d %12.3f %10.2f %6.2f" % (short, n, s / 1e6, a / 1e3, 100.0 * s / tot))
print("total kernel time %.3f ms over %d dispatches" % (tot / 1e6, sum(r[1] for r in rows)))
