# tgemm_kernel per-phase shader-clock split on the current schedule (stamps variant build; timing of
# the variant is not the product's), then the product build's per-mode launch times
set -o pipefail
mkdir -p gpurun_out
NR_LIB=neurecon_amd/_ab/libnrhip_stamps.so timeout -k 10 120 python tools/tg_driver.py --iters 10 --stamps > gpurun_out/tgstamps.txt 2>&1 || exit 1
timeout -k 10 120 python tools/tg_driver.py --iters 30 > gpurun_out/tgstamps_product.txt 2>&1 || exit 1
