#!/bin/bash
# nr_wgrad with the one-launch reduction: parity, kernel split, the fp32 training-batch bar, the full
# default bench (configs + training), then the same-box A/B of the 24-bit slab
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w4
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED|nr_wgrad" $O/wg_pytest.log | tail -14; [ $rc = 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/wgrad_bench.py > $O/prof.log 2>&1 || exit $?
grep "nr_wgrad\|hipBLAS" $O/prof.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_raybatch.py -v -rA -s --timeout 300 --timeout-method thread -k random_batch > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst|weight_v" $O/pytest.log | tail -14; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || exit $?
tail -c 3000 $O/bench.log
bash tools/ab_slab.sh
