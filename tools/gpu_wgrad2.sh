#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w2
mkdir -p $O
timeout -k 10 120 python3 -u tools/wgrad_bench.py > $O/wb.log 2>&1; echo "wb rc=$?"; cat $O/wb.log | grep -v amdgpu.ids
for S in 64 32; do NR_WGRAD_SLICES=$S timeout -k 10 120 python3 -u tools/wgrad_bench.py 2>&1 | grep nr_wgrad; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/wgrad_bench.py > $O/prof.log 2>&1; echo "prof rc=$?"
find $O/prof -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | head -12
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_raybatch.py tests/test_gpu_train.py -v -rA -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|fp32 envelope" $O/pytest.log | grep -E "FAILED|passed|failed|layers.0.weight_v" | tail -12
exit $rc
