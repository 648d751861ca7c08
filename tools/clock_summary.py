"""Effective shader clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE [SQ_...] pass.

    python tools/clock_summary.py <dir> [kernel-substring]

clock = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) / dispatch wall time
(MI355X_MICROARCH.md 'DVFS give-back'); dispatches shorter than 0.3 ms read high and are skipped.
Other counters in the same pass are reported per dispatch (mean), e.g. SQ_BUSY_CU_CYCLES,
SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, sub=''):
    rows = defaultdict(dict)   # dispatch id -> {counter: value, name, t}
    times = {}
    for path in glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                times[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    for path in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                d = rows[r['Dispatch_Id']]
                d['name'] = r['Kernel_Name']
                d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
                if 'Start_Timestamp' in r and r.get('End_Timestamp'):
                    d['t'] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    agg = defaultdict(lambda: defaultdict(list))
    for did, d in rows.items():
        if sub not in d.get('name', ''):
            continue
        t = times.get(did, d.get('t'))
        if not t or t < float(os.environ.get("NR_MIN_T", "3e-4")):
            continue
        a = agg[d['name'][:90]]
        a['t'].append(t)
        for k, v in d.items():
            if k in ('name', 't'):
                continue
            a[k].append(v)
        if 'GRBM_GUI_ACTIVE' in d:
            a['clock_GHz'].append(d['GRBM_GUI_ACTIVE'] / 8 / t / 1e9)
    for name, a in agg.items():
        n = len(a['t'])
        print(f'{name}: {n} dispatches, mean {1e3 * sum(a["t"]) / n:.3f} ms')
        for k, v in sorted(a.items()):
            if k == 't':
                continue
            vs = sorted(v)
            print(f'   {k:28s} mean {sum(v) / len(v):14.4g}  median {vs[len(vs) // 2]:14.4g}')


if __name__ == '__main__':
    main(*sys.argv[1:])
