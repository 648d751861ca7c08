cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04b
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04b/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r04b/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/shard_balance.py > gpurun_out/r04b/shard.log 2>&1; rc=$?; echo "shard rc=$rc"; tail -4 gpurun_out/r04b/shard.log
exit $rc
