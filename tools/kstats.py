"""Print a rocprofv3 kernel_stats.csv (name, calls, average / min / max duration)."""
import csv
import sys

for r in list(csv.DictReader(open(sys.argv[1])))[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>6s} avg={float(r['AverageNs']) / 1e3:8.2f}us "
          f"min={float(r['MinNs']) / 1e3:8.2f} max={float(r['MaxNs']) / 1e3:8.2f}")
