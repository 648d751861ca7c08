# nr_wgrad cost split at the training step's layout (P = 130560, 16 x 16 blocked operands, 256 x 256):
# the full kernel, loads only, no MFMA, no split + LDS store (variant builds in neurecon_amd/_ab; timing only)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base wg_loadonly wg_nomfma wg_nostore; do
    if [ $v = base ]; then unset NR_LIB; else export NR_LIB=neurecon_amd/_ab/libnrhip_$v.so; fi
    timeout -k 10 120 python tools/wgrad_bench.py --points 130560 --no-blas --blocked > gpurun_out/wgsplit_${v}_$i.txt 2>&1 || exit 1
  done
done
