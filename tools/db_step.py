"""List the kernels of one training step from a rocprofv3 results .db (between the last two launches whose
name contains MARK), optionally filtered by a substring.  usage: python tools/db_step.py <db> [filter] [mark]"""
import sqlite3
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
mark = sys.argv[3] if len(sys.argv) > 3 else "heads384"
rows = list(c.execute("select name, duration, grid_x, queue_id, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if mark in r[0]]
s, e = idx[-2], idx[-1]
t0 = rows[s][4]
for r in rows[s:e]:
    n = short(r[0])
    if flt and not any(f in n for f in flt.split(",")):
        continue
    print("%8.1f %-44s %8.1f grid=%-8d q=%s" % ((r[4] - t0) / 1e3, n[:44], r[1] / 1e3, r[2], r[3]))
print("step span %.1f us" % ((rows[e][4] - t0) / 1e3))
