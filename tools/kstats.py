"""Per-step kernel summary of a rocprofv3 rocpd database (or kernel_stats CSV):
python tools/kstats.py <run_results.db> <steps-in-run> [top]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
steps = int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = db.execute("select name, count(*), sum(end-start)/1e6 from kernels group by name order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total {tot:.3f} ms, {tot / steps:.3f} ms/step over {steps} steps")
for n, c, t in rows[:top]:
    print(f"{t / steps:8.3f} ms/step {c / steps:6.1f}/step {1e3 * t / c:9.1f} us/launch  {n[:100]}")
