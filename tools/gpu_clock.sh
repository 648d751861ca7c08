#!/bin/bash
# Effective clock (GRBM_GUI_ACTIVE / 8 / wall) and MFMA-busy cycles of the SDF kernel under load:
# tools/mlp_driver.py back to back for >= 2 s, one rocprofv3 --pmc pass per counter group.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/clock_${TAG:-base}
mkdir -p $O
i=0
for C in "GRBM_GUI_ACTIVE" "SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/p$i -o run \
    -- python3 tools/mlp_driver.py --iters ${ITERS:-500} ${DRIVER_ARGS} > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  python3 tools/clock_summary.py $O/p$i sdf4 | tee $O/p$i.txt
done
