#!/bin/bash
# HBM traffic per kernel launch: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
# (they do not fit one TCC pass on gfx950), kernel-trace only, no other trace domains.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${T_PROF:-420} rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-eval --no-frame ${BENCH_ARGS} > $OUT/$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
