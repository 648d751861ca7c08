#!/bin/bash
# nr_wgrad cost split (experiment builds), the fp32 training-batch bar, the default bench, slab A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w5
mkdir -p $O
for v in base wg_nomfma wg_nostore wg_loadonly wg_noload; do
  lib=neurecon_amd/_exp/libnrhip_$v.so; [ $v = base ] && lib=neurecon_amd/libnrhip.so
  NR_LIB=$lib timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb_$v.log 2>&1 || exit $?
  echo "$v: $(grep nr_wgrad $O/wb_$v.log | cut -d, -f1 | tr '\n' ' ')"
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_raybatch.py -v -rA -s --timeout 300 --timeout-method thread -k random_batch > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|batch, worst" $O/pytest.log | tail -6; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || exit $?
tail -c 2500 $O/bench.log
bash tools/ab_slab.sh
