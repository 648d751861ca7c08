#!/bin/bash
# same-box A/B of the config-(b) bench: A = neurecon_amd/_exp/abA.so (fp32 slabs, the build before the
# 24-bit slab), B = neurecon_amd/libnrhip.so; alternated; both with an 8 GiB workspace (one chunk each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=neurecon_amd/_exp/abA.so; else lib=neurecon_amd/libnrhip.so; fi
    NR_LIB=$lib timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-frame --no-configs \
      --workspace-gb 8 "$@" > gpurun_out/ab/slab_$v$r.log 2>&1 || exit $?
    echo "$v$r $(grep -o '"value": [0-9.]*' gpurun_out/ab/slab_$v$r.log | head -1) $(grep -o '"frac": [0-9.]*' gpurun_out/ab/slab_$v$r.log | head -1)"
  done
done
