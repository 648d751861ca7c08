#!/bin/bash
# Round-6 final verification of the tree as committed: smoke, the whole -m gpu suite, the default bench
# line, then the profile set (rocprofv3 --kernel-trace --stats of config (b) and of training; the
# matrix-pipe passes; FETCH_SIZE / WRITE_SIZE passes), each step under its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06f}
mkdir -p $O
python3 -c "from neurecon_amd import build as b; print('build_id', b.lib_build_id(), 'tree', b.source_hash())" > $O/build_id.txt
cat $O/build_id.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -n 20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${T_TEST:-1100} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.txt | head -20; exit 1; }
  tail -n 1 $O/pytest_gpu.txt
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -n 20 $O/bench.err; exit 1; }
  tail -c 400 $O/bench.json
fi
if [ -n "$PROFILES" ]; then
  TAG=${TAG}_m STEPS=20 bash tools/gpu_mfma_r05.sh > $O/mfma.log 2>&1 || { echo "mfma passes failed"; tail -n 5 $O/mfma.log; exit 1; }
  B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-frame --no-configs --no-scaling-legs --no-fp32-mode"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b_full -o run -- $B > $O/b_full.log 2>&1 || { echo "b_full prof failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- python3 bench.py --workload train --steps 5 --warmup 2 > $O/train.log 2>&1 || { echo "train prof failed"; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_b/$C -o run -- $B --steps 3 --warmup 1 --no-full-eval > $O/pmc_b_$C.log 2>&1 || { echo "pmc b $C failed"; exit 1; }
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_train/$C -o run -- python3 bench.py --workload train --steps 3 --warmup 1 > $O/pmc_train_$C.log 2>&1 || { echo "pmc train $C failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $O/pmc_b > $O/f16x3_pmc_summary.json && python3 tools/pmc_summary.py $O/pmc_train > $O/train_pmc_summary.json && echo "profiles ok"
fi
