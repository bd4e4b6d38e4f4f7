"""Summarise a rocprofv3 kernel_stats.csv: name, calls, avg/min/max us, share."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        print(f"  {r['Name'][:58]:58s} calls={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:9.2f}us "
              f"min={float(r['MinNs'])/1e3:9.2f} max={float(r['MaxNs'])/1e3:9.2f} {float(r['Percentage']):5.1f}%")
