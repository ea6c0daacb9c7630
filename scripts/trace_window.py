"""Per-step kernel table from a rocprofv3 kernel_trace.csv restricted to the LAST n steps (steps
delimited by a marker kernel, e.g. the optimizer launch): excludes one-time work such as MIOpen's
find-mode benchmarking in the first iterations.
    python scripts/trace_window.py TRACE.csv MARKER_SUBSTRING [n_steps] [top]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
marker, n = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
assert len(idx) > n, f'only {len(idx)} marker launches'
win = rows[idx[-n - 1] + 1: idx[-1] + 1]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in win:
    nm = r['Kernel_Name']
    k = nm[nm.find('WCfg'):nm.find('WCfg') + 90] if 'WCfg' in nm else nm[:90]
    agg[k][0] += 1
    agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
tot = sum(v[1] for v in agg.values())
span = (int(win[-1]['End_Timestamp']) - int(win[0]['Start_Timestamp'])) / 1e3
print(f'last {n} steps: kernel time {tot / n / 1e3:.2f} ms/step, wall span {span / n / 1e3:.2f} ms/step\n')
print('| ms/step | share | calls/step | avg us | kernel |\n|---|---|---|---|---|')
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f'| {v[1] / n / 1e3:.2f} | {100 * v[1] / tot:.1f}% | {v[0] / n:g} | {v[1] / v[0]:.1f} | `{k}` |')
