#!/bin/bash
# r06: kernel census of the fp32 NeuS and SIREN VolSDF training steps (no hipBLASLt kernel left), then the
# training bench legs after the Adam version-counter fix
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06j}; mkdir -p $O
for w in ${WHICH:-neus32 siren32}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/census_$w -o run -- python3 tools/train_census.py --which $w > $O/census_$w.log 2>&1 \
    || { echo "census $w failed"; tail -5 $O/census_$w.log; exit 1; }
  grep "ms per step" $O/census_$w.log
  python3 - $O/census_$w <<'PY'
import csv, glob, sys
rows = []
for p in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    rows += list(csv.DictReader(open(p)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
blas = [r for r in rows if 'nr::' not in r['Name'] and any(s in r['Name'] for s in ('Cijk', 'hipblaslt', 'Tensile', 'rocblas', 'gemm'))]
print(f"{sys.argv[1]}: {len(rows)} kernels, vendor GEMM kernels {len(blas)} = {100 * sum(float(r['TotalDurationNs']) for r in blas) / tot:.2f} % of device time")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(__import__("os").environ.get("TOPK", "8"))]:
    print(f"   {r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['TotalDurationNs']) / tot * 100:5.1f} %")
PY
done
[ -n "$NO_TRAIN" ] && exit 0
for extra in "" "--train-nerfpp"; do
  timeout -k 10 400 python3 bench.py --workload train $extra --steps 20 --warmup 3 > $O/train$extra.json 2> $O/train$extra.err || { echo "train bench failed"; tail -5 $O/train$extra.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/train$extra.json').read().strip().splitlines()[-1]); print('train$extra', round(d['value']), d['unit'], d['ms_per_step'])"
done
