#!/bin/bash
# (record of an r04 measurement: the experiment build it compares was removed after it was measured;
#  results and reading in profiles/r04/ and DESIGN.md -- rerunning needs that variant restored)
# nr_wgrad 256-wide n tile vs 128 (NR_WGRAD_NB), parity of both, training bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w12
mkdir -p $O
for nb in 256 128; do
  NR_WGRAD_NB=$nb timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad.py -v -rA -s --timeout 120 --timeout-method thread > $O/wg_pytest_$nb.log 2>&1
  rc=$?; echo "NB=$nb wgrad pytest rc=$rc"; grep -E "passed|failed|FAILED|nr_wgrad" $O/wg_pytest_$nb.log | tail -4; [ $rc = 0 ] || exit $rc
done
for r in 1 2; do for nb in 256 128; do
  NR_WGRAD_NB=$nb timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb_$nb.log 2>&1 || exit $?
  echo "NB=$nb: $(grep nr_wgrad $O/wb_$nb.log | cut -d, -f1 | tr '\n' ' ')"
done; done
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_raybatch.py tests/test_gpu_train.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst" $O/pytest.log | tail -6; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-frame --config-steps 10 > $O/bench.log 2>&1 || exit $?
python3 -c "
import json; s=open('$O/bench.log').read(); j=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
print(j['value'], {k: (v['value'], v.get('ms_per_step')) for k, v in j['configs'].items()})
t=j['configs']['train_neus_512']; print(t.get('library_kernels'))"
