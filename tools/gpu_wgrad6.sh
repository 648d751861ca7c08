#!/bin/bash
# nr_wgrad: parity + cost split after the unconditional prefetch and the DPP quad max
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w6
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest.log 2>&1
rc=$?; echo "wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED|nr_wgrad" $O/wg_pytest.log | tail -14; [ $rc = 0 ] || exit $rc
for v in base wg_nomfma wg_nostore wg_loadonly; do
  lib=neurecon_amd/_exp/libnrhip_$v.so; [ $v = base ] && lib=neurecon_amd/libnrhip.so
  NR_LIB=$lib timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb_$v.log 2>&1 || exit $?
  echo "$v: $(grep nr_wgrad $O/wb_$v.log | cut -d, -f1 | tr '\n' ' ')"
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame --config-steps 10 > $O/bench.log 2>&1 || exit $?
python3 -c "
import json,sys; s=open('$O/bench.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
print(j['value'], {k: (v['value'], v.get('ms_per_step')) for k, v in j['configs'].items()})
print(j['configs']['train_neus_512'].get('device_time_by_group'))"
