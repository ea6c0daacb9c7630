"""Summarise a rocprofv3 --stats kernel CSV: per-step ms, calls/step, avg us per kernel."""
import csv
import sys


def main(path, steps, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print(f"kernel time per step: {tot / steps / 1e6:.2f} ms over {steps} profiled steps\n")
    print("| ms/step | calls/step | avg us | kernel |\n|---|---|---|---|")
    for r in rows[:top]:
        print(f"| {float(r['TotalDurationNs']) / steps / 1e6:.2f} | {int(r['Calls']) / steps:.0f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:100]}` |")


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 30)
