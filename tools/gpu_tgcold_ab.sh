# tgemm_kernel without the compiler's tile-start vmcnt(0) on the prefetched path (in-tree build) vs the
# previous build (neurecon_amd/_ab/libnrhip_tgold.so): parity tests first, then alternated timing
# (tools/tg_driver.py per epilogue mode; the NeuS training step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_raybatch.py > gpurun_out/tgcold_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export NR_LIB=neurecon_amd/_ab/libnrhip_tgold.so; else unset NR_LIB; fi
    timeout -k 10 120 python tools/tg_driver.py --iters 30 > gpurun_out/tgcold_tg_${v}_$i.txt 2>&1 || exit 1
    timeout -k 10 180 python bench.py --workload train --steps 30 --warmup 5 > gpurun_out/tgcold_train_${v}_$i.json 2> gpurun_out/tgcold_train_${v}_$i.err || exit 1
  done
done
unset NR_LIB
