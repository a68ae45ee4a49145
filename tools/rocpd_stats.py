"""rocprofv3's SQLite output (run_results.db) -> the kernel_stats.csv columns
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs).
    python tools/rocpd_stats.py gpurun_out/TAG/prof/run_results.db > profiles/X_kernel_stats.csv
"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = list(con.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                        "from kernels group by name order by sum(duration) desc"))
total = sum(r[2] for r in rows) or 1
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for name, n, tot, avg, mn, mx in rows:
    w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 3), mn, mx])
