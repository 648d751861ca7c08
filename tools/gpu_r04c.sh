#!/bin/bash
# r04 combined check: LDS-DMA dwordx3 probe, smoke (build ID), nr_wgrad tests, the whole -m gpu suite,
# then the default bench line.  Logs under gpurun_out/$TAG/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04c}
mkdir -p $O
if [ -x tools/probes/ldsdma_x3 ]; then timeout -k 5 60 tools/probes/ldsdma_x3 > $O/probe_x3.log 2>&1; echo "probe rc=$?"; cat $O/probe_x3.log; fi
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -x -v -rA -s --timeout 120 --timeout-method thread > $O/pytest_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; grep -E "max \||nr_wgrad" $O/pytest_wgrad.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${T_TEST:-900} python3 -u -m pytest tests -m gpu -v -rA -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1
rb=$?; echo "bench rc=$rb"; tail -1 $O/bench.log | cut -c1-700
exit $rc
