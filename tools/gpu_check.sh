#!/bin/bash
# GPU-box check: parity tests, then (unless a test run crashed) a short bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q -s ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest crashed/timed out"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${T_BENCH:-600} python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rb=$?
echo "bench rc=$rb"; tail -3 gpurun_out/bench.log
exit $rb
