#!/bin/bash
# training-workload profile set (after the blocked layout): rocprofv3 kernel stats, then FETCH_SIZE and
# WRITE_SIZE passes (each its own run, kernel-trace only) -> train_pmc_summary.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04pt
mkdir -p $O/train $O/pmc_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- python3 bench.py --workload train --steps 5 --warmup 2 > $O/train/stdout.log 2>&1 || exit $?
echo "train rc=0"; grep '^{"metric"' $O/train/stdout.log | cut -c1-200
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_train/$c -o run -- python3 bench.py --workload train --steps 3 --warmup 1 > $O/pmc_train/$c.log 2>&1 || exit $?
  echo "pmc $c rc=0"
done
python3 tools/pmc_summary.py $O/pmc_train > $O/train_pmc_summary.json && echo pmc ok
