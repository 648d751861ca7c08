#!/bin/bash
# (record of an r04 measurement: the experiment build it compares was removed after it was measured;
#  results and reading in profiles/r04/ and DESIGN.md -- rerunning needs that variant restored)
# tgemm epilogue access-pattern experiment: training bench with the default build vs NR_EXP_TG_LINEAR
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04tgl
mkdir -p $O
for r in 1 2; do for v in base tglinear; do
  lib=neurecon_amd/_exp/libnrhip_$v.so; [ $v = base ] && lib=neurecon_amd/libnrhip.so
  NR_LIB=$lib timeout -k 10 200 python3 -u bench.py --workload train --steps 10 --warmup 2 > $O/train_$v.log 2>&1 || exit $?
  python3 -c "
import json; s=open('$O/train_$v.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
r=j.get('roofline') or {}
print('$v', j['value'], j['ms_per_step'], r.get('avg_launch_ms'), r.get('achieved'))"
done; done
