#!/bin/bash
# nr_wgrad with running per-quad exponents: parity, timing, training tests, bench configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w7
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED|nr_wgrad|max \|hip" $O/wg_pytest.log | tail -24; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb.log 2>&1 || exit $?; grep -v amdgpu.ids $O/wb.log
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_raybatch.py tests/test_gpu_train.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst" $O/pytest.log | tail -8; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame --config-steps 10 > $O/bench.log 2>&1 || exit $?
python3 -c "
import json,sys; s=open('$O/bench.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
print(j['value'], {k: (v['value'], v.get('ms_per_step')) for k, v in j['configs'].items()})
t=j['configs']['train_neus_512']; print(t.get('device_time_by_group')); print(t.get('library_kernels'))"
