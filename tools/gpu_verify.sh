#!/bin/bash
# One verification pass on the GPU box: smoke(), the whole -m gpu suite with every test's name and
# printed pass rates (-rA -s), then the default bench line.  Logs under gpurun_out/$TAG/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04}
mkdir -p $O
git_head=$(cat .git_head 2>/dev/null || echo "?")
echo "tree build id: $(python3 -c 'from neurecon_amd import build; print(build.source_hash())')" | tee $O/build_id.txt
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 ${T_TEST:-1200} python3 -u -m pytest tests -m gpu -x -v -rA -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
fi
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 ${T_BENCH:-600} python3 -u bench.py ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-600
exit $rc
