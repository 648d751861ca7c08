#!/bin/bash
# rocprofv3 --kernel-trace --stats of one command (CMD), then its top kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ks}; mkdir -p $O
timeout -k 10 ${T:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- $CMD > $O/log.txt 2>&1 || { echo "run failed"; tail -5 $O/log.txt; exit 1; }
tail -2 $O/log.txt | cut -c1-400
python3 tools/kstats.py $O/st ${TOP:-15}
