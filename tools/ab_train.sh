#!/bin/bash
# A/B of the training bench on one box: A = neurecon_amd/_exp/head.so (the committed build), B = the
# working-tree build; alternated so box-to-box variance cancels.  Extra args go to both runs.
# head.so: compile the changed .hip files of `git archive HEAD neurecon_amd/csrc include` with
# neurecon_amd/build.py's flags and link them with the other objects of neurecon_amd/_build/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then lib=neurecon_amd/_exp/head.so; else lib=neurecon_amd/libnrhip.so; fi
    NR_LIB=$lib timeout -k 10 150 python bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline "$@" \
      > gpurun_out/ab_$v$r.log 2>&1 || exit $?
    echo "$v$r $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v$r.log)"
  done
done
