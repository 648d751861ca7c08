#!/bin/bash
# r06: every forward-only SDF launch on 64-point tiles (NR_NARROW_FWD=1) vs the size threshold, configs
# (c) and (e) alternated
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06w}; mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    NR_NARROW_FWD=$v timeout -k 10 300 python3 -u tools/bench_frameworks.py --configs --only ce --steps 10 > $O/ce_${r}_$v.txt 2>&1 || { echo "bench failed"; tail -5 $O/ce_${r}_$v.txt; exit 1; }
    echo "narrow=$v: $(tail -1 $O/ce_${r}_$v.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v["rays_per_s"]) for k,v in d.items()})')"
  done
done
