#!/bin/bash
# chunked UNISURF march: UNISURF render / training parity, then config (e) via the default bench configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04march
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_unisurf.py tests/test_gpu_train.py -x -v -rA -s --timeout 300 --timeout-method thread -k "unisurf or UNISURF" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -4; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame --config-steps 10 > $O/bench.log 2>&1 || exit $?
python3 -c "
import json; s=open('$O/bench.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
e=j['configs']['e_unisurf_4096']; print(j['value'], e['value'], e['ms_per_step'], e.get('roofline'), str(e.get('kernels'))[:400])"
