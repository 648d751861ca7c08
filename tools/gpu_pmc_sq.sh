#!/bin/bash
# SQ/GRBM counter passes (<= 8 SQ counters per pass, kernel-trace only) over tools/mlp_driver.py
# (DRIVER=tools/wgrad_bench.py for another driver script).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-sq}
OUT=gpurun_out/pmcsq_$TAG
mkdir -p $OUT
i=0
for SET in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F16 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM" \
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS" ; do
  i=$((i+1))
  timeout -k 10 ${T_PROF:-300} rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $OUT/p$i -o run \
    -- python3 ${DRIVER:-tools/mlp_driver.py} ${DRIVER_ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_sq_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
