"""Print the kernels of a rocprofv3 --stats csv by total time: python scripts/dev/top_kernels.py <dir> [n]."""
import csv
import sys

rows = list(csv.DictReader(open(f"{sys.argv[1]}/trace/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{r['Calls']:>6} {float(r['AverageNs']) / 1000:9.1f} us  {r['Name'][:100]}")
