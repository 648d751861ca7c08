#!/bin/bash
# nr_wgrad bring-up: its parity tests, the training parity tests, then the training bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r04w}
mkdir -p $O
if [ -x tools/probes/ldsdma_x3 ]; then timeout -k 5 60 tools/probes/ldsdma_x3 > $O/probe_x3.log 2>&1; echo "probe rc=$?"; cat $O/probe_x3.log; fi
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -x -v -rA -s --timeout 120 --timeout-method thread > $O/pytest_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; grep -E "max \||nr_wgrad|passed|failed|Error" $O/pytest_wgrad.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_raybatch.py -x -v -rA -s --timeout 300 --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $O/pytest_train.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --workload train --steps 20 --warmup 3 > $O/bench_train.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_train.log | cut -c1-400
exit $rc
