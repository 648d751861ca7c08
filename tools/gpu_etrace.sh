#!/bin/bash
# r06: per-launch kernel trace of config (e) (UNISURF 4096 rays), 2 steps after 1 warm-up
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-etrace}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/bench_frameworks.py --configs --only e --steps 2 --warmup 1 > $O/run.log 2>&1 || { echo "trace failed"; tail -5 $O/run.log; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1); cp $f $O/kernel_trace.csv; echo done
