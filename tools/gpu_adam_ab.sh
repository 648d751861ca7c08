set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "adam or neus_train_step_vs_oracle" > gpurun_out/adam_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for a in fused nr; do
    timeout -k 10 180 python bench.py --workload train --adam $a --steps 30 --warmup 5 > gpurun_out/adam_bench_${a}_$i.json 2> gpurun_out/adam_bench_${a}_$i.err || exit 1
  done
done
