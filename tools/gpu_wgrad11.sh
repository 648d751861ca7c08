#!/bin/bash
# (record of an r04 measurement: the experiment build it compares was removed after it was measured;
#  results and reading in profiles/r04/ and DESIGN.md -- rerunning needs that variant restored)
# nr_wgrad ping-pong phase split: base (waves w & 4 split first) vs none vs adjacent waves; parity
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w11
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED" $O/wg_pytest.log | tail -4; [ $rc = 0 ] || exit $rc
for r in 1 2; do for v in base wg_pp0 wg_pp1; do
  lib=neurecon_amd/_exp/libnrhip_$v.so; [ $v = base ] && lib=neurecon_amd/libnrhip.so
  NR_LIB=$lib timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb_$v.log 2>&1 || exit $?
  echo "$v: $(grep nr_wgrad $O/wb_$v.log | cut -d, -f1 | tr '\n' ' ')"
done; done
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_raybatch.py tests/test_gpu_train.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst" $O/pytest.log | tail -8; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame --config-steps 10 > $O/bench.log 2>&1 || exit $?
python3 -c "import json; s=open('$O/bench.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0]); print(j['value'], {k: (v['value'], v.get('ms_per_step')) for k, v in j['configs'].items()})"
