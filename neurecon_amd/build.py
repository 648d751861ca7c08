"""Build libnrhip.so (gfx950) in-tree with hipcc.

    python -m neurecon_amd.build [--force] [--jobs N]

Every .hip under neurecon_amd/csrc is compiled for --offload-arch=gfx950 into an object in
neurecon_amd/_build/, then linked into neurecon_amd/libnrhip.so (git-ignored; it travels to the
GPU box with the repo snapshot).  Rebuilds only when a source/header is newer than the library.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, '_build')
LIB = os.path.join(HERE, 'libnrhip.so')
INC = os.path.join(os.path.dirname(HERE), 'include')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('NR_OFFLOAD_ARCH', 'gfx950')
FLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-I', CSRC, '-I', INC,
         '-munsafe-fp-atomics', '-Wno-unused-result']


# per-file extra flags: the MLP kernels keep scalar fp32 VALU beside their MFMAs (the SLP vectoriser
# would pack adjacent f32 ops into v_pk_*, which cost ~22 extra cycles there, MI355X_MICROARCH.md)
FILE_FLAGS = {'nr_mlp.hip': ['-fno-slp-vectorize']}


def flags_for(src):
    return FLAGS + FILE_FLAGS.get(os.path.basename(src), [])


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')))


def _deps():
    return _sources() + glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(INC, '*.h'))


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in _deps())


def _compile(src):
    obj = os.path.join(OUT, os.path.basename(src) + '.o')
    cmd = [HIPCC] + flags_for(src) + ['-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stderr}')
    return obj, r.stderr


def build(force=False, jobs=None, verbose=False):
    if not force and up_to_date():
        return LIB
    os.makedirs(OUT, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4) // 2), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(_compile, srcs))
    for obj, err in results:
        if verbose and err.strip():
            print(err, file=sys.stderr)
    tmp = LIB + '.tmp'
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', tmp] + [o for o, _ in results]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed:\n{r.stderr}')
    os.replace(tmp, LIB)
    return LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--jobs', type=int, default=None)
    ap.add_argument('-v', '--verbose', action='store_true')
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.jobs, verbose=a.verbose))
