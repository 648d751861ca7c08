#!/bin/bash
# Round-4 profile set: rocprofv3 --kernel-trace --stats of the default bench (config b, without the
# frame / configs legs), its full-evaluation loop, the training workload and the config-(d) frame; then
# FETCH_SIZE / WRITE_SIZE passes (each its own run, kernel-trace only) of config (b) and of training.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
ONLY=${ONLY:-}
run() {  # tag, timeout, command...
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $1 "* ]]; then return 0; fi
  local tag=$1 t=$2; shift 2
  mkdir -p $O/$tag
  timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- "$@" > $O/$tag/stdout.log 2>&1
  local rc=$?
  echo "$tag rc=$rc"; tail -1 $O/$tag/stdout.log | cut -c1-300
  return $rc
}
pmc() {  # tag, counter, command...
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" pmc_$1 "* ]]; then return 0; fi
  local tag=$1 c=$2; shift 2
  mkdir -p $O/pmc_$tag
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$tag/$c -o run -- "$@" > $O/pmc_$tag/$c.log 2>&1
  local rc=$?; echo "pmc $tag $c rc=$rc"; return $rc
}
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-frame --no-configs"
run b 300 $B --no-full-eval &&
run b_full 300 $B &&
run train 300 python3 bench.py --workload train --steps 5 --warmup 2 &&
run frame_d 400 python3 bench.py --workload frame_d --steps 2 --warmup 1 &&
pmc b FETCH_SIZE $B --steps 3 --warmup 1 --no-full-eval &&
pmc b WRITE_SIZE $B --steps 3 --warmup 1 --no-full-eval &&
pmc train FETCH_SIZE python3 bench.py --workload train --steps 3 --warmup 1 &&
pmc train WRITE_SIZE python3 bench.py --workload train --steps 3 --warmup 1 &&
python3 tools/pmc_summary.py $O/pmc_b > $O/f16x3_pmc_summary.json &&
python3 tools/pmc_summary.py $O/pmc_train > $O/train_pmc_summary.json && echo pmc ok
