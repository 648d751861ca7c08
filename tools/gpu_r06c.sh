#!/bin/bash
# r06: sdf5 (32x32x16) forward kernel A/B against sdf4 with experiment variants, then matrix-pipe
# occupancy and clock of both (rocprofv3 --pmc passes, each alone; tools/mfma_summary.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c}; mkdir -p $O
NR_SDF5=1 timeout -k 10 300 python3 -u tools/sdf5_ab.py --variants ${VARIANTS:-0,1,2,3,4,5,6} ${AB_ARGS} > $O/sdf5_ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/sdf5_ab.txt; exit 1; }
grep -v amdgpu.ids $O/sdf5_ab.txt
[ -n "$NO_PMC" ] && exit 0
export NR_SDF5=1; B="python3 tools/sdf5_ab.py --variants 0,1 --rounds 1 --iters 10"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/grbm -o run -- $B > $O/grbm.log 2>&1 \
  || { echo "grbm pass failed"; tail -5 $O/grbm.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 \
  || { echo "sq pass failed"; tail -5 $O/sq.log; exit 1; }
python3 tools/mfma_summary.py $O/grbm $O/sq sdf > $O/mfma_summary.json && cat $O/mfma_summary.json
