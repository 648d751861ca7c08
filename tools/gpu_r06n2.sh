#!/bin/bash
# r06: narrow 64-point tiles for small forward-only SDF launches: parity tests, then config (e) and the
# NeuS training step alternated with the library built from the previous nr_mlp.hip (ALT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06n2}; mkdir -p $O
ALT=${ALT:-neurecon_amd/_ab/libnr_wide.so}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf5.py tests/test_gpu_unisurf.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.txt | head; exit 1; }
tail -n 1 $O/pytest.txt
for r in 1 2; do
  for L in neurecon_amd/libnrhip.so $ALT; do
    b=$(basename $L .so)
    NR_LIB=$PWD/$L timeout -k 10 300 python3 -u tools/bench_frameworks.py --configs --only e --steps 10 > $O/e_${r}_$b.txt 2>&1 || { echo "bench e failed"; tail -5 $O/e_${r}_$b.txt; exit 1; }
    echo "e $b: $(tail -1 $O/e_${r}_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["e_unisurf_4096"]; print(round(d["rays_per_s"]), {k: round(v[1]/10,3) for k,v in d["kernels"].items() if k.startswith("sdf")})')"
    NR_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --workload train --steps 20 --warmup 3 > $O/t_${r}_$b.json 2> $O/t_${r}_$b.err || { echo "bench train failed"; tail -5 $O/t_${r}_$b.err; exit 1; }
    echo "train $b: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' $O/t_${r}_$b.json)"
  done
done
