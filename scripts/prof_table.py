"""Print a per-step kernel table from a rocprofv3 kernel_stats.csv: python scripts/prof_table.py CSV STEPS [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"kernel time per step: {tot / 1e6 / steps:.2f} ms over {steps:g} profiled steps\n")
print("| ms/step | calls/step | avg us | kernel |\n|---|---|---|---|")
for r in rows[:n]:
    print(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.2f} | {int(r['Calls']) / steps:g} | "
          f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:100]}` |")
