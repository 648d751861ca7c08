#!/bin/bash
# Round-3 profile set: rocprofv3 --kernel-trace --stats of the default bench (f16x3 and fp32), the
# config-(d) frame and training workloads, and tools/bench_frameworks.py --configs (VolSDF / UNISURF
# and configs (c), (d), (e)); then the FETCH_SIZE / WRITE_SIZE passes of the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
ONLY=${ONLY:-}
run() {  # tag, timeout, command...  (ONLY="b b_full": just those tags)
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $1 "* ]]; then return 0; fi
  local tag=$1 t=$2; shift 2
  mkdir -p $O/$tag
  timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- "$@" > $O/$tag/stdout.log 2>&1
  local rc=$?
  echo "$tag rc=$rc"; tail -2 $O/$tag/stdout.log | cut -c1-300
  return $rc
}
run b 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full-eval --no-frame &&
run b_full 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-frame &&
run b_fp32 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-eval --no-frame --precision fp32 &&
run frame_d 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --workload frame_d &&
run train 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --workload train &&
run configs 500 python3 tools/bench_frameworks.py --steps 3 --warmup 1 --configs &&
[ -n "$ONLY" ] || TAG=r03 bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 && echo pmc ok
