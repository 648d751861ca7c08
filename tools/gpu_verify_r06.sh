#!/bin/bash
# r06 verification: selected GPU tests (TESTS), then the full default bench line (one JSON line).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06v}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TEST:-600} python3 -u -m pytest -x -q -rA --timeout 120 --timeout-method thread -m gpu $TESTS > $O/pytest.log 2>&1
  rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${T_BENCH:-400} python3 bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -n 20 $O/bench.err; exit 1; }
  tail -c 3000 $O/bench.json
fi
