"""Top kernels of a rocprofv3 --stats kernel_stats.csv.  The optional divisor is the number of
train steps the profiled command ran (warm-up + timed), to print per-step figures.

  python tools/prof_summary.py <run_kernel_stats.csv> [steps] [top]
"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    print(f"{float(r['TotalDurationNs'])/1e6/div:8.3f} ms/step {float(r['Percentage']):6.2f}% n/step={int(r['Calls'])/div:7.1f} avg={float(r['AverageNs'])/1e3:8.2f}us  {r['Name'][:100]}")
print('total ms/step', tot / 1e6 / div)
