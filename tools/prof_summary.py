"""Summarise a rocprofv3 rocpd database (kernel-trace) into per-kernel totals per step."""
import sqlite3
import sys

db, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(duration)/1e6, avg(duration)/1e3 from kernels group by name "
                 "order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel time {tot / steps:.3f} ms per step ({steps:g} steps)")
for name, n, ms, avg in rows[:top]:
    print(f"{ms / steps:8.3f} ms/step  n/step={n / steps:6.1f}  avg={avg:8.1f}us  {name[:120]}")
