#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv: calls, total, average."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel time %.2f ms' % (tot / 1e6))
for r in rows[:n]:
    print('%-88s %7s %10.2f ms %9.4f ms avg %5.1f%%' % (r['Name'][:88], r['Calls'], float(r['TotalDurationNs']) / 1e6,
                                                      float(r['AverageNs']) / 1e6, float(r['Percentage'])))
