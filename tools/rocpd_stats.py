"""Kernel statistics (the rocprofv3 --stats summary: calls, total / average / min / max ns per
kernel) from a rocprofv3 SQLite results database (ROCm 7 writes results.db when no
--output-format is given).  usage: python tools/rocpd_stats.py RESULTS.db [OUT.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("""SELECT name, COUNT(*), SUM(end - start), AVG(end - start), MIN(end - start), MAX(end - start)
                     FROM kernels GROUP BY name ORDER BY SUM(end - start) DESC""").fetchall()
total = sum(r[2] for r in rows) or 1
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for name, calls, tot, avg, mn, mx in rows:
    w.writerow([name, calls, tot, f"{avg:.1f}", f"{100.0 * tot / total:.2f}", mn, mx])
