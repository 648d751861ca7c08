#!/bin/bash
# r06: VolSDF lane-segmented passes -- the VolSDF parity suite, then config (c) timing with per-kernel times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_volsdf.py} > $O/pytest.log 2>&1; rc=$?
tail -n 3 $O/pytest.log; grep -E "iter_usage|rays pass|worst" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "^E |FAILED" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python3 -u tools/bench_frameworks.py --configs --only c --steps 10 > $O/bench_c.txt 2>&1 || { echo "bench failed"; tail -20 $O/bench_c.txt; exit 1; }
tail -30 $O/bench_c.txt
