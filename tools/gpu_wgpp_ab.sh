# nr_wgrad phase split between the two waves of a SIMD (variants wg_pp4: waves w & 4 split first;
# wg_pp1: odd waves), after the r05 loop-head drain fix, vs the in-tree build: parity of the variants
# (tests/test_gpu_wgrad.py), then alternated timing (wgrad at the training layout; the NeuS training step)
set -o pipefail
mkdir -p gpurun_out
for v in wg_pp4 wg_pp1; do
  NR_LIB=neurecon_amd/_ab/libnrhip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad.py > gpurun_out/wgpp_tests_$v.txt 2>&1 || exit 1
done
for i in 1 2; do
  for v in base wg_pp4 wg_pp1; do
    export NR_LIB=neurecon_amd/_ab/libnrhip_$v.so
    timeout -k 10 120 python tools/wgrad_bench.py --points 130560 --no-blas --blocked > gpurun_out/wgpp_wg_${v}_$i.txt 2>&1 || exit 1
    timeout -k 10 180 python bench.py --workload train --steps 30 --warmup 5 > gpurun_out/wgpp_train_${v}_$i.json 2> gpurun_out/wgpp_train_${v}_$i.err || exit 1
  done
done
unset NR_LIB
