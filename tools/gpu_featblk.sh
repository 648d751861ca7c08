#!/bin/bash
# (record of an r04 measurement: the experiment build it compares was removed after it was measured;
#  results and reading in profiles/r04/ and DESIGN.md -- rerunning needs that variant restored)
# blocked geometry feature (sdf4 -> rad4) experiment: config-(b) bench, default build vs featblk, alternated;
# then the render parity tests on the featblk build (its results are valid: producer and consumer agree)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04fb
mkdir -p $O
for r in 1 2 3; do for v in base featblk; do
  lib=neurecon_amd/_exp/libnrhip_$v.so; [ $v = base ] && lib=neurecon_amd/libnrhip.so
  NR_LIB=$lib timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-frame --no-configs > $O/b_$v.log 2>&1 || exit $?
  python3 -c "
import json; s=open('$O/b_$v.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
r=j['roofline']; print('$v', j['value'], j['ms_per_step'], r['frac'], {k: v['avg_launch_ms'] for k, v in r['per_launch_type'].items()})"
done; done
NR_LIB=neurecon_amd/_exp/libnrhip_featblk.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "featblk parity rc=$rc"; tail -2 $O/parity.log
