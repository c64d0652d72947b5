"""Kernels of one training step on every queue of a rocprofv3 results .db, in start order, with the gap before
each launch on its own queue.  usage: python tools/db_queue.py <db> [mark] [queue]"""
import sqlite3
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

c = sqlite3.connect(sys.argv[1])
mark = sys.argv[2] if len(sys.argv) > 2 else "heads384"
onlyq = int(sys.argv[3]) if len(sys.argv) > 3 else None
rows = list(c.execute("select name, duration, grid_x, queue_id, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if mark in r[0]]
s, e = idx[-2], idx[-1]
t0 = rows[s][4]
prev = {}
for r in rows[s:e]:
    q = r[3]
    if onlyq is not None and q != onlyq:
        continue
    gap = (r[4] - prev[q]) / 1e3 if q in prev else 0.0
    prev[q] = r[5]
    print("%8.1f q%-2d gap%7.1f %-44s %8.1f grid=%d" % ((r[4] - t0) / 1e3, q, gap, short(r[0])[:44], r[1] / 1e3, r[2]))
for q in sorted(set(r[3] for r in rows[s:e])):
    print("queue %d busy %.1f us" % (q, sum(r[5] - r[4] for r in rows[s:e] if r[3] == q) / 1e3))
print("step span %.1f us" % ((rows[e][4] - t0) / 1e3))
