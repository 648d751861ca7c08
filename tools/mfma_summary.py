"""Matrix-pipe occupancy and effective clock per kernel from rocprofv3 --pmc passes.

    python tools/mfma_summary.py <grbm-pass-dir> <sq-pass-dir> [kernel-substring] > summary.json

Pass 1 holds GRBM_GUI_ACTIVE, pass 2 SQ_VALU_MFMA_BUSY_CYCLES (+ SQ_BUSY_CU_CYCLES), each collected
in its own rocprofv3 --pmc --kernel-trace run of the same command (MI355X_MICROARCH.md: GRBM and SQ
counters in separate passes, no other trace domains).  Per kernel name:
  clock_ghz  = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) / dispatch wall time (pass 1);
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES (cycles summed over the 1024 SIMDs) /
               (1024 x clock x dispatch wall time of pass 2), i.e. the fraction of SIMD-cycles the
               matrix pipe was busy;
  frac_decomp = mfma_busy x clock / 2.4 GHz: the fraction of the 2.4 GHz dense-MFMA peak the kernel
               would reach at full operand efficiency (the f16x3 roofline frac is this times the
               useful-product share of the issued MFMAs).
Dispatches shorter than NR_MIN_T (default 1e-4 s) are skipped (the GRBM quotient reads high on
very short dispatches, MI355X_MICROARCH.md 'DVFS give-back')."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024          # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
PEAK_CLOCK_GHZ = 2.4


def load(root):
    """{dispatch id: {'name', 't', counter: value}}"""
    times, rows = {}, defaultdict(dict)
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
    for did, d in rows.items():
        d['t'] = times.get(did)
    return rows


def main(grbm_dir, sq_dir, sub=''):
    tmin = float(os.environ.get('NR_MIN_T', '1e-4'))
    clk, busy = defaultdict(list), defaultdict(list)
    for d in load(grbm_dir).values():
        if sub in d.get('name', '') and d.get('t') and d['t'] >= tmin and 'GRBM_GUI_ACTIVE' in d:
            clk[d['name']].append((d['t'], d['GRBM_GUI_ACTIVE'] / 8 / d['t'] / 1e9))
    for d in load(sq_dir).values():
        if sub in d.get('name', '') and d.get('t') and d['t'] >= tmin and 'SQ_VALU_MFMA_BUSY_CYCLES' in d:
            busy[d['name']].append((d['t'], d['SQ_VALU_MFMA_BUSY_CYCLES'], d.get('SQ_BUSY_CU_CYCLES')))
    out = {}
    for name in sorted(set(clk) | set(busy)):
        c = clk.get(name, [])
        b = busy.get(name, [])
        rec = {'dispatches_grbm': len(c), 'dispatches_sq': len(b)}
        if c:
            rec['mean_ms_grbm_pass'] = 1e3 * sum(t for t, _ in c) / len(c)
            # time-weighted clock over the dispatches
            rec['clock_ghz'] = sum(t * g for t, g in c) / sum(t for t, _ in c)
        if b:
            rec['mean_ms_sq_pass'] = 1e3 * sum(t for t, _, _ in b) / len(b)
            rec['mfma_busy_cycles_per_dispatch'] = sum(m for _, m, _ in b) / len(b)
            if c:
                cyc = sum(t for t, _, _ in b) * rec['clock_ghz'] * 1e9 * SIMDS
                rec['mfma_busy'] = sum(m for _, m, _ in b) / cyc
                rec['frac_decomp'] = rec['mfma_busy'] * rec['clock_ghz'] / PEAK_CLOCK_GHZ
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:])
