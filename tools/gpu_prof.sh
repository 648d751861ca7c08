#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench (no CPU leg); summaries land in gpurun_out/prof_<tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_$TAG/bench_stdout.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_$TAG/bench_stdout.log
find gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
