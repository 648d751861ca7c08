cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 300 python3 -u tools/sdf5_ab.py > $O/sdf5_ab.txt 2>&1; echo "ab rc=$?"; cat $O/sdf5_ab.txt | tail -12
timeout -k 10 900 python3 -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py tests/test_gpu_train.py::test_adam_matches_torch_adam tests/test_gpu_train.py::test_neus_training_with_nr_adam_matches_torch_adam tests/test_gpu_parity.py::test_neus_workspace_bound_by_rayschunk > $O/pytest.log 2>&1; rc=$?; tail -n 3 $O/pytest.log; echo "tests rc=$rc"
