#!/bin/bash
# r06: pack batches of 20 ops (one batch per SDF pack) vs 8: training tests, then the NeuS training step
# alternated with the library built from the previous nr_mlp.hip (ALT)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06p2}; mkdir -p $O
ALT=${ALT:-neurecon_amd/_ab/libnr_pack8.so}
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.txt | head; exit 1; }
tail -n 1 $O/pytest.txt
for r in 1 2 3; do
  for L in neurecon_amd/libnrhip.so $ALT; do
    b=$(basename $L .so)
    NR_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --workload train --steps 20 --warmup 3 > $O/t_${r}_$b.json 2> $O/t_${r}_$b.err || { echo "bench train failed"; tail -5 $O/t_${r}_$b.err; exit 1; }
    echo "train $b: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' $O/t_${r}_$b.json)"
  done
done
