"""Per-step kernel table from a rocprofv3 --kernel-trace CSV: the steps are delimited by a
once-per-step marker kernel (name substring, its LAST NSTEPS+1 occurrences), so warm-up and
setup work is excluded. usage: python scripts/trace_steps.py TRACE.csv MARKER NSTEPS [TOP]"""
import csv
import sys


def main(path, marker, nsteps, top=40):
    rows = sorted(((r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp']))
                   for r in csv.DictReader(open(path))), key=lambda x: x[1])
    marks = [s for n, s, e in rows if marker in n]
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
    print(f"window {(t1 - t0) / 1e6 / nsteps:.3f} ms/step wall, kernels {tot / 1e6 / nsteps:.3f} ms/step busy\n")
    print("| ms/step | calls/step | % | kernel |\n|---|---|---|---|")
    for n, (cnt, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"| {d / 1e6 / nsteps:.3f} | {cnt / nsteps:.1f} | {100 * d / tot:.1f} | `{n[:110]}` |")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 40)
