"""Per-step kernel table from a rocprofv3 rocpd database: the timed steps are delimited by a
once-per-step marker kernel (substring), so warm-up work (MIOpen find, first-call tuning)
is excluded. usage: python scripts/rocpd_steps.py DB MARKER NSTEPS [TOP]"""
import sqlite3
import sys

db, marker, nsteps = sys.argv[1], sys.argv[2], int(sys.argv[3])
top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
marks = [r[1] for r in rows if marker in r[0]]
if len(marks) < nsteps + 1:
    sys.exit(f"marker {marker!r} seen {len(marks)} times, need {nsteps + 1}")
t0, t1 = marks[-nsteps - 1], marks[-1]
agg = {}
for n, s, e in rows:
    if t0 <= s < t1:
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
tot = sum(v[1] for v in agg.values())
print(f"window {(t1 - t0) / 1e6 / nsteps:.3f} ms/step wall, kernels {tot / 1e6 / nsteps:.3f} ms/step busy")
for n, (cnt, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{d / 1e6 / nsteps:8.3f} ms {cnt / nsteps:6.1f}x {100 * d / tot:5.1f}%  {n[:120]}")
