"""Summarise a rocprofv3 kernel_stats.csv: top kernels and per-category totals."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
n_top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
print(f'total {tot / 1e6:.1f} ms')
for r in rows[:n_top]:
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} us "
          f"{float(r['Percentage']):5.1f}%  {r['Name'][:120]}")
