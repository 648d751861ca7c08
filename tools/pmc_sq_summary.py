"""Average per-dispatch SQ/GRBM counters per kernel from tools/gpu_pmc_sq.sh output."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                acc[row['Kernel_Name']][row['Counter_Name']].append(float(row['Counter_Value']))
    for k, cs in sorted(acc.items()):
        if 'nr::' not in k:
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f'  {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})')


if __name__ == '__main__':
    main(sys.argv[1])
