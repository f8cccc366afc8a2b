"""Per-kernel totals from a rocprofv3 SQLite output (rocpd): name, calls, total ms, mean us."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
ki = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
cols = [r[1] for r in db.execute(f"pragma table_info({ki})")]
namecol = "display_name" if "display_name" in cols else "kernel_name"
q = (f"select s.{namecol}, count(*), sum(d.end - d.start) from {kd} d join {ki} s on d.kernel_id = s.id "
     f"group by s.{namecol} order by 3 desc")
rows = list(db.execute(q))
tot = sum(r[2] for r in rows)
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for name, n, t in rows[:lim]:
    print(f"{t / 1e6:10.2f} ms {n:6d} {t / n / 1e3:10.1f} us  {100 * t / tot:5.1f}%  {name[:110]}")
