#!/bin/bash
# r06: compaction without the 671 072-slot limit (16-aligned list segments, per-wave slab base): tests,
# then config (b) and the config-(d) frame alternated with the library of the previous sources (ALT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06k2}; mkdir -p $O
ALT=${ALT:-neurecon_amd/_ab/libnr_limit.so}
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_nerf.py tests/test_gpu_options.py tests/test_gpu_perturb.py tests/test_gpu_dist.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.txt | head; exit 1; }
tail -n 1 $O/pytest.txt
for r in 1 2; do
  for L in neurecon_amd/libnrhip.so $ALT; do
    b=$(basename $L .so)
    NR_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-frame --no-configs --no-scaling-legs --no-fp32-mode --no-full-eval > $O/b_${r}_$b.json 2> $O/b_${r}_$b.err || { echo "bench failed"; tail -5 $O/b_${r}_$b.err; exit 1; }
    echo "b $b: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["per_launch_type"]["sdf_nabla_bwd"]["avg_launch_ms"])' $O/b_${r}_$b.json)"
    NR_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --workload frame_d --steps 3 --warmup 1 > $O/d_${r}_$b.json 2> $O/d_${r}_$b.err || { echo "bench d failed"; tail -5 $O/d_${r}_$b.err; exit 1; }
    echo "d $b: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' $O/d_${r}_$b.json)"
  done
done
