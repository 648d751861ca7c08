#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of tools/mlp_driver.py per library variant (NR_LIB), one rocprofv3 pass per
# counter; summaries in gpurun_out/pmcd_<variant>/summary.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  O=gpurun_out/pmcd_$v
  mkdir -p $O
  for C in FETCH_SIZE WRITE_SIZE; do
    NR_LIB=neurecon_amd/_exp/libnrhip_$v.so timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv \
      -d $O/$C -o run -- python3 tools/mlp_driver.py --iters 2 ${DRIVER_ARGS} > $O/$C.log 2>&1 || { echo "pmc $v $C failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $O > $O/summary.json
  echo "== $v"; python3 - $O/summary.json <<'PY'
import json, sys
for k, r in json.load(open(sys.argv[1])).items():
    if 'sdf4' in k:
        print(k[:48], r['launches'], 'fetch', round(r['fetch_bytes_per_launch_x2'] / 1e6), 'MB write', round(r['write_bytes_per_launch'] / 1e6), 'MB')
PY
done
