#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w9
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED|nr_wgrad|max \|hip" $O/wg_pytest.log | tail -24; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb.log 2>&1 || exit $?; grep -v amdgpu.ids $O/wb.log
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/p1 -o run -- python3 tools/wgrad_bench.py > $O/p1.log 2>&1 || exit $?
python3 tools/pmc_sq_summary.py $O | grep -A9 wgrad_kernel
