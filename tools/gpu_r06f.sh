#!/bin/bash
# r06: config (c) timing, alternating the current library and an A/B variant library (NR_LIB)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06f}; mkdir -p $O
for r in 1 2; do
  for L in neurecon_amd/libnrhip.so ${ALT:-neurecon_amd/_ab/libnr_oldvs.so}; do
    NR_LIB=$PWD/$L timeout -k 10 300 python3 -u tools/bench_frameworks.py --configs --only c --steps 10 > $O/bench_c_$r_$(basename $L).txt 2>&1 || { echo "bench failed"; exit 1; }
    echo "$L: $(tail -1 $O/bench_c_$r_$(basename $L).txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["c_volsdf_2048x256"]; print(round(d["rays_per_s"]), {k: round(v[1]/10,3) for k,v in d["kernels"].items()})')"
  done
done
