#!/bin/bash
# r06: point-level compaction of the deferred reverse pass (sdf4_kernel STAGE 4): the NeuS parity, frame,
# NeRF++ and option tests, then config (b) alternated with the library built from the previous sources (ALT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06k}; mkdir -p $O
ALT=${ALT:-neurecon_amd/_ab/libnr_tiles.so}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest_parity.txt 2>&1 \
  || { echo "parity tests failed"; grep -E "FAILED|Error" $O/pytest_parity.txt | head; exit 1; }
tail -n 1 $O/pytest_parity.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_frame.py tests/test_gpu_nerf.py tests/test_gpu_options.py tests/test_gpu_perturb.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest_more.txt 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest_more.txt | head; exit 1; }
tail -n 1 $O/pytest_more.txt
for r in 1 2 3; do
  for L in neurecon_amd/libnrhip.so $ALT; do
    b=$(basename $L .so)
    NR_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-frame --no-configs --no-scaling-legs --no-fp32-mode > $O/b_${r}_$b.json 2> $O/b_${r}_$b.err || { echo "bench failed"; tail -5 $O/b_${r}_$b.err; exit 1; }
    echo "b $b: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(d["value"], d["ms_per_step"], {k: v["avg_launch_ms"] for k, v in r["per_launch_type"].items()}, d["full_evaluation"]["value"] if "full_evaluation" in d else "")' $O/b_${r}_$b.json)"
  done
done
