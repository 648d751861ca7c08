#!/bin/bash
# r06: VolSDF early-exit bound decisions: the VolSDF GPU tests, then config (c) alternated with the
# library built from the previous nr_volsdf.hip (ALT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06v}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_volsdf.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest_volsdf.txt 2>&1 \
  || { echo "volsdf tests failed"; grep -E "FAILED|Error" $O/pytest_volsdf.txt | head; exit 1; }
tail -n 1 $O/pytest_volsdf.txt
TAG=${TAG:-r06v} ALT=${ALT:-neurecon_amd/_ab/libnr_prevs.so} bash tools/gpu_r06f.sh
