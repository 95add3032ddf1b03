"""Summarise a rocprofv3 --stats kernel_stats.csv (developer helper)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:40]:
    print(f"{float(r['TotalDurationNs'])/tot*100:6.2f}% calls={r['Calls']:>6} avg={float(r['AverageNs'])/1000:8.2f}us "
          f"per-step={float(r['TotalDurationNs'])/steps/1000:8.1f}us  {r['Name'][:90]}")
print('total kernel ms', tot / 1e6, 'per step us', tot / steps / 1000)
