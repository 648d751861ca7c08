"""Top kernels of a rocprofv3 --stats run: python tools/kstats.py <dir> [top]"""
import csv
import glob
import sys

rows = []
for p in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    rows += list(csv.DictReader(open(p)))
tot = sum(float(r['TotalDurationNs']) for r in rows) or 1.0
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{r['Name'][:78]:78s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['TotalDurationNs']) / tot * 100:5.1f} %")
