"""Per-kernel stats and a step timeline from a rocprofv3 rocpd database (kernel trace).
usage: python tools/trace_timeline.py <run_results.db> [kernel-name-regex-for-timeline] [n_rows]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, stream_id, start, end, duration, grid_x, workgroup_x from kernels order by start").fetchall()
stats = {}
for name, sid, s, e, d, gx, wx in rows:
    short = re.sub(r"^_ZN3lmr\w*?\d+(k_\w+?)I.*$", r"\1", name)
    short = re.sub(r"\(.*$", "", short)[:60]
    st = stats.setdefault(short, [0, 0.0])
    st[0] += 1
    st[1] += d / 1e6
print("%-60s %6s %10s %9s" % ("kernel", "calls", "total ms", "avg ms"))
for k, (c, t) in sorted(stats.items(), key=lambda x: -x[1][1]):
    print("%-60s %6d %10.3f %9.4f" % (k, c, t, t / c))
if len(sys.argv) > 2:
    rx = re.compile(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 80
    sel = [r for r in rows if rx.search(r[0])]
    t0 = sel[-n][2] if len(sel) >= n else sel[0][2]
    print("\nlast %d matching dispatches (start/end in us from the first shown, stream)" % n)
    for name, sid, s, e, d, gx, wx in sel[-n:]:
        short = re.sub(r"^_ZN3lmr\w*?\d+(k_\w+?)I.*$", r"\1", name)[:40]
        print("%-40s stream %3d  %9.1f %9.1f  %7.1f us" % (short, sid, (s - t0) / 1e3, (e - t0) / 1e3, d / 1e3))
