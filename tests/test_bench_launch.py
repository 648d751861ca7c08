"""bench.py's multi-GPU launch contract, rehearsed on the CPU (gloo, stub step).

`python bench.py --gpus N` outside torchrun must start N rank processes that join one process
group (the driver's scaling runs), and torchrun's own layout must give the same result: one JSON
line from rank 0 with n_gpus taken from the process group."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', OMP_NUM_THREADS='1')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_n_ranks():
    out = _run([sys.executable, 'bench.py', '--gpus', '2', '--steps', '2', '--warmup', '1', '--stub-cpu'])
    assert out['n_gpus'] == 2 and sorted(out['ranks']) == [0, 1]
    assert out['steps'] == 2 and out['warmup'] == 1
    # the weak-scaling legs of the default N-GPU line: config (e)'s sharded render with its window
    # all-reduce in the step, and the DDP training step
    for leg in ('weak_scaling_e', 'weak_scaling_train'):
        assert out[leg]['n_gpus'] == 2 and out[leg]['scaling'] == 'weak' and out[leg]['value'] > 0, out[leg]
        assert out[leg]['collective_in_step'], leg


def test_bench_single_process_default():
    out = _run([sys.executable, 'bench.py', '--steps', '2', '--warmup', '1', '--stub-cpu'])
    assert out['n_gpus'] == 1 and out['ranks'] == [0]
    assert out['weak_scaling_e']['n_gpus'] == 1 and not out['weak_scaling_e']['collective_in_step']


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_under_torchrun():
    out = _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), 'bench.py', '--gpus', '2', '--steps', '2',
                '--warmup', '1', '--stub-cpu'])
    assert out['n_gpus'] == 2 and sorted(out['ranks']) == [0, 1]
