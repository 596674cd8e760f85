"""Summarise a rocprofv3 *_kernel_stats.csv: python scripts/kstats.py <csv> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} calls avg {float(r['AverageNs'])/1e3:8.1f} us"
          f" {100*float(r['TotalDurationNs'])/tot:5.1f}%  {r['Name'][:100]}")
print("total ms", round(tot / 1e6, 2))
