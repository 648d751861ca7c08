#!/bin/bash
# 16 x 16 blocked training tensors: wgrad blocked-operand bit identity, training parity + the blocked vs
# row-major bit identity, then the training bench (blocked default vs NR_TRAIN_BLOCKED=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04merge}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "^FAILED|passed|failed|Error" $O/wg_pytest.log | tail -6; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_raybatch.py tests/test_gpu_siren.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst|Error" $O/pytest.log | tail -8; [ $rc = 0 ] || exit $rc
for r in 1 2; do for v in 1 0; do
  NR_TRAIN_BLOCKED=$v timeout -k 10 200 python3 -u bench.py --workload train --steps 10 --warmup 2 > $O/train_$v.log 2>&1 || exit $?
  python3 -c "
import json; s=open('$O/train_$v.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
r=j.get('roofline') or {}; w=r.get('wgrad') or {}
print('blocked=$v', j['value'], j['ms_per_step'], 'tgemm', r.get('avg_launch_ms'), 'wgrad', w.get('avg_launch_ms'))"
done; done
