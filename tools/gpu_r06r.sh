#!/bin/bash
# r06: the training sampler without the radiance render pack (and RadianceTG without it): training
# tests, then the NeuS training step alternated with a copy of the previous tree (_abtree: its package
# and library)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r06r}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_raybatch.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/pytest.txt | head; exit 1; }
tail -n 1 $O/pytest.txt
for r in 1 2 3; do
  for T in . _abtree; do
    b=$([ "$T" = "." ] && echo new || echo old)
    (cd $T && timeout -k 10 300 python3 bench.py --workload train --steps 20 --warmup 3 > $O/t_${r}_$b.json 2> $O/t_${r}_$b.err) || { echo "bench train failed"; tail -5 $O/t_${r}_$b.err; exit 1; }
    echo "train $b: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' $O/t_${r}_$b.json)"
  done
done
