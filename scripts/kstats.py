"""Top kernels of a rocprofv3 kernel_stats.csv: total ms, calls, average ms."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {int(r['Calls']):5d} calls avg "
          f"{float(r['AverageNs']) / 1e6:8.3f} ms  {r['Name'][:100]}")
