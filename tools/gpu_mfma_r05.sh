#!/bin/bash
# Round-5 matrix-pipe evidence for the nabla kernel's three launch types on the bench itself:
# rocprofv3 --kernel-trace --stats of config (b), then one --pmc pass for GRBM_GUI_ACTIVE and one for
# SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CU_CYCLES (each its own run, kernel-trace only), summarised per
# device kernel by tools/mfma_summary.py (clock_ghz, mfma_busy).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05m}
mkdir -p $O
B="python3 bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-frame --no-configs --no-full-eval ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/stats.log 2>&1 \
  || { echo "stats pass failed"; tail -5 $O/stats.log; exit 1; }
tail -1 $O/stats.log | cut -c1-400
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/grbm -o run -- $B > $O/grbm.log 2>&1 \
  || { echo "grbm pass failed"; tail -5 $O/grbm.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 \
  || { echo "sq pass failed"; tail -5 $O/sq.log; exit 1; }
python3 tools/mfma_summary.py $O/grbm $O/sq sdf4_kernel > $O/mfma_summary.json && cat $O/mfma_summary.json
