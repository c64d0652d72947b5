"""Per-stream busy time and idle gaps of the last full training step in a rocprofv3 kernel_trace.csv.

usage: python tools/stream_gaps.py <kernel_trace.csv> [min_gap_us] [--queues]  (--queues: group by hardware queue,
       e.g. for a replayed graph whose branches run on several queues)
Prints, per HIP stream (Stream_Id), the kernel time, the idle time between its kernels, and the largest gaps
with the kernels on either side -- where the compute stream waits for the host or for the other stream."""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     r["Queue_Id"] if "--queues" in sys.argv else r["Stream_Id"]))
rows.sort()
idx = [i for i, r in enumerate(rows) if r[2].startswith("adam") and "tick" not in r[2]]
s, e = idx[-2] + 1, idx[-1] + 1
step = rows[s:e]
t0, t1 = step[0][0], step[-1][1]
print("step wall %.3f ms" % ((t1 - t0) / 1e6))
args = [a for a in sys.argv[1:] if not a.startswith("--")]
mg = float(args[1]) if len(args) > 1 else 5.0
for sid in sorted({r[3] for r in step}):
    ks = [r for r in step if r[3] == sid]
    busy = sum(b - a for a, b, _, _ in ks) / 1e3
    gaps = []
    for p, q in zip(ks, ks[1:]):
        g = (q[0] - p[1]) / 1e3
        gaps.append((g, p[2], q[2], (p[1] - t0) / 1e3))
    idle = sum(max(0.0, g[0]) for g in gaps)
    print("stream %s: %d kernels, busy %.1f us, idle between kernels %.1f us (%d gaps > %.0f us)"
          % (sid, len(ks), busy, idle, sum(1 for g in gaps if g[0] > mg), mg))
    for g, a, b, at in sorted(gaps, reverse=True)[:12]:
        print("   gap %7.1f us at %7.1f us: %s -> %s" % (g, at, a, b))
