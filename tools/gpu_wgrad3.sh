#!/bin/bash
# nr_wgrad after the buffer-load rewrite: parity tests, timing, kernel split under rocprof, then the
# training tests and the same-box A/B of the 24-bit slab
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w3
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED|nr_wgrad" $O/wg_pytest.log | tail -14; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb.log 2>&1 || exit $?; grep -v amdgpu.ids $O/wb.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/wgrad_bench.py > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | head -12
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_raybatch.py tests/test_gpu_train.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst" $O/pytest.log | tail -14; [ $rc = 0 ] || exit $rc
bash tools/ab_slab.sh
