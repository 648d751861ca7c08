#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06h}; mkdir -p $O
for m in base wgrad64 mm64 both64; do
  timeout -k 10 300 python3 -u tools/train_error_probe.py $m > $O/probe_$m.txt 2>&1 || { echo "probe $m failed"; tail -5 $O/probe_$m.txt; exit 1; }
  grep -E "== mode|layers.0.weight_v|layers.4.weight_v|layers.0.weight_g|layers.4.weight_g|512-ray|assertion" $O/probe_$m.txt
done
