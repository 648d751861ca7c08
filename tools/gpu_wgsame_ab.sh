# nr_wgrad with 32-bit k-step indices, the vector row as a template parameter and one lane-offset set
# for same-geometry pairs (in-tree build) vs the previous build (neurecon_amd/_ab/libnrhip_wgold.so):
# parity tests first, then alternated timing (wgrad at the training layout; the NeuS training step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad.py tests/test_gpu_train.py > gpurun_out/wgsame_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export NR_LIB=neurecon_amd/_ab/libnrhip_wgold.so; else unset NR_LIB; fi
    timeout -k 10 120 python tools/wgrad_bench.py --points 130560 --no-blas --blocked > gpurun_out/wgsame_wg_${v}_$i.txt 2>&1 || exit 1
    timeout -k 10 180 python bench.py --workload train --steps 30 --warmup 5 > gpurun_out/wgsame_train_${v}_$i.json 2> gpurun_out/wgsame_train_${v}_$i.err || exit 1
  done
done
unset NR_LIB
