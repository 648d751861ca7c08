# r06: tgemm_kernel launch times of the product build (tools/tg_driver.py).  The r06 run also timed a
# no-weight-DMA variant (profiles/r06/tgemm_nodma_bound.txt): that variant breaks tgemm_kernel's counted
# waits and faulted, so it is not run from here again.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/tg_driver.py --iters 30 > gpurun_out/tgb_product.txt 2>&1 || exit 1
