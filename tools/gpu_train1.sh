#!/bin/bash
# training-path change check: the training parity tests, then the bench's training config (+ (b))
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04t1}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_raybatch.py tests/test_gpu_siren.py tests/test_gpu_wgrad.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst" $O/pytest.log | tail -8; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame --config-steps 10 > $O/bench.log 2>&1 || exit $?
python3 -c "
import json; s=open('$O/bench.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
print(j['value'], {k: (v['value'], v.get('ms_per_step')) for k, v in j['configs'].items()})
t=j['configs']['train_neus_512']; print(t.get('device_time_by_group')); print(t.get('top_kernels'))"
