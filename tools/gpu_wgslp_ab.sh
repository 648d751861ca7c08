# A/B: nr_wgrad.hip with and without -fno-slp-vectorize (neurecon_amd/_ab/libnrhip_wgnoslp.so),
# alternated: the wgrad timing tool at the training shapes, then the NeuS training step
set -o pipefail
mkdir -p gpurun_out
V=neurecon_amd/_ab/libnrhip_wgnoslp.so
for i in 1 2; do
  for lib in base noslp; do
    if [ $lib = base ]; then unset NR_LIB; else export NR_LIB=$V; fi
    timeout -k 10 120 python tools/wgrad_bench.py --points 130560 --no-blas > gpurun_out/wgslp_wg_${lib}_$i.txt 2>&1 || exit 1
    timeout -k 10 180 python bench.py --workload train --steps 30 --warmup 5 > gpurun_out/wgslp_train_${lib}_$i.json 2> gpurun_out/wgslp_train_${lib}_$i.err || exit 1
  done
done
unset NR_LIB
