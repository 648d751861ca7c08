#!/bin/bash
# (record of an r04 measurement: both the built-out change and the comparison library were removed after
#  it was measured; results in profiles/r04/feat_blocked_experiment.txt)
# blocked geometry feature between the render's SDF and radiance launches: render parity suites, then
# the config-(b) bench against the previous build (neurecon_amd/prev_cmp.so), alternated
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04fb2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nerf.py tests/test_gpu_volsdf.py tests/test_gpu_unisurf.py tests/test_gpu_surface.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/parity.log; [ $rc = 0 ] || exit $rc
for r in 1 2 3; do for v in prev new; do
  lib=neurecon_amd/prev_cmp.so; [ $v = new ] && lib=neurecon_amd/libnrhip.so
  NR_LIB=$lib timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-frame --no-configs > $O/b_$v.log 2>&1 || exit $?
  python3 -c "
import json; s=open('$O/b_$v.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
r=j['roofline']; print('$v', j['value'], j['ms_per_step'], r['frac'], {k: v['avg_launch_ms'] for k, v in r['per_launch_type'].items()})"
done; done
