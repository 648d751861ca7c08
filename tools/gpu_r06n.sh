#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06n}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_unisurf.py tests/test_gpu_dist.py} > $O/pytest.log 2>&1; rc=$?
tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head; exit 1; }
timeout -k 10 300 python3 -u tools/bench_frameworks.py --configs --only ${ONLY:-e} --steps 10 > $O/bench.txt 2>&1 || { tail -5 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt | cut -c1-1500
