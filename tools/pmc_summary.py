"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs into per-kernel HBM bytes per launch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half of the bytes of wide
(16 B/lane) coalesced streaming reads -> multiplied by 2; WRITE_SIZE is exact for 16 B/lane stores.
Units: FETCH_SIZE / WRITE_SIZE are in KB (x1024 bytes)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root, counter):
    out = defaultdict(list)
    for path in glob.glob(os.path.join(root, counter, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get('Counter_Name') != counter:
                    continue
                out[row['Kernel_Name']].append(float(row['Counter_Value']))
    return out


def main(root):
    fetch = load(root, 'FETCH_SIZE')
    write = load(root, 'WRITE_SIZE')
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024 * sum(f) / max(len(f), 1)
        wb = 1024 * sum(w) / max(len(w), 1)
        res[k] = {'launches': max(len(f), len(w)), 'fetch_bytes_per_launch_x2': fb, 'write_bytes_per_launch': wb,
                  'hbm_bytes_per_launch': fb + wb}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
