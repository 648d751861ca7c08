#!/bin/bash
# A/B of the default library against variant builds (NR_LIB), alternated on one box:
#   TESTS="tests/test_gpu_parity.py ..." VARIANTS="neurecon_amd/_ab/libnrhip_x.so ..." bash tools/gpu_ab.sh
# 1) the listed GPU tests on the default library; 2) ROUNDS x (default, each variant) of the config-(b)
# bench (per-launch-type averages) and, with DRIVER_MODES, tools/mlp_driver.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TEST:-400} python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $O/pytest.log 2>&1
  rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
fi
B="python3 bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-frame --no-configs ${BENCH_ARGS:---no-full-eval}"
for r in $(seq ${ROUNDS:-2}); do
  for lib in default $VARIANTS; do
    tag=$(basename $lib .so)
    if [ "$lib" = default ]; then env_lib=""; else env_lib="NR_LIB=$lib"; fi
    env $env_lib timeout -k 10 120 $B > $O/bench_${tag}_$r.json 2> $O/bench_${tag}_$r.err || { echo "bench $tag failed"; tail -n 5 $O/bench_${tag}_$r.err; exit 1; }
    python3 - $O/bench_${tag}_$r.json $tag <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
pl = d['roofline']['per_launch_type']
fe = d.get('full_evaluation', {})
print(f"{sys.argv[2]:24s} {d['value']:10.1f} rays/s {d['ms_per_step']:7.3f} ms  frac {d['roofline']['frac']:.4f}  " +
      '  '.join(f"{k[10:]} {v['avg_launch_ms']:.4f}" for k, v in pl.items()) +
      (f"  full {fe['value']:.1f}" if fe else ''))
EOF
    for m in $DRIVER_MODES; do
      echo -n "   driver $m: "; env $env_lib timeout -k 10 120 python3 tools/mlp_driver.py --mode $m --iters 20 2>&1 | tail -n 1
    done
  done
done
