"""Build libnrhip.so (gfx950) in-tree with hipcc.

    python -m neurecon_amd.build [--force] [--jobs N]

Every .hip under neurecon_amd/csrc is compiled for --offload-arch=gfx950 into an object in
neurecon_amd/_build/, then linked into neurecon_amd/libnrhip.so (git-ignored; it travels to the
GPU box with the repo snapshot).

Build ID: `source_hash()` is a sha256 over the names and bytes of every csrc source/header, the
public header and the compiler flags.  It is compiled into the library (`nr_build_id()`), and the
library is rebuilt whenever the ID it carries differs from the tree's (not by file times: a copied
tree or a reverted edit keeps or changes the hash, never the mtime order).  smoke() and bench.py
print it and smoke() asserts it equals the tree's.
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
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


def source_hash():
    """16 hex digits identifying the library's sources: csrc/*.hip, csrc/*.h, include/*.h (names and
    bytes, in name order) and the compile flags (without absolute paths)."""
    h = hashlib.sha256()
    for p in sorted(_deps(), key=lambda q: (os.path.basename(os.path.dirname(q)), os.path.basename(q))):
        h.update(os.path.basename(os.path.dirname(p)).encode() + b'/' + os.path.basename(p).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
        h.update(b'\0')
    h.update(repr([f for f in FLAGS if f not in (CSRC, INC)]).encode())
    h.update(repr(sorted(FILE_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def lib_build_id(path=LIB):
    """The build ID compiled into a library file (read from its bytes; no dlopen), or None."""
    if not os.path.exists(path):
        return None
    with open(path, 'rb') as f:
        data = f.read()
    i = data.find(b'NR_BUILD_ID=')
    if i < 0:
        return None
    return data[i + 12:i + 28].decode('ascii', 'replace')


def up_to_date():
    return lib_build_id() == source_hash()


ID_SOURCE = 'nr_capi.hip'  # the one object that carries the build ID (nr_build_id)


def _obj_key(src, build_id):
    """what an object depends on: its source, every header, its flags (and the ID for ID_SOURCE)"""
    h = hashlib.sha256()
    for p in [src] + sorted(glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(INC, '*.h'))):
        with open(p, 'rb') as f:
            h.update(os.path.basename(p).encode() + b'\0' + f.read())
    h.update(repr([f for f in flags_for(src) if f not in (CSRC, INC)] + [HIPCC]).encode())
    if os.path.basename(src) == ID_SOURCE:
        h.update(build_id.encode())
    return h.hexdigest()


def _compile(src, build_id):
    """compile one source unless its object was built from the same inputs (sidecar key file)"""
    obj = os.path.join(OUT, os.path.basename(src) + '.o')
    key = _obj_key(src, build_id)
    kfile = obj + '.key'
    if os.path.exists(obj) and os.path.exists(kfile) and open(kfile).read() == key:
        return obj, ''
    defs = [f'-DNR_BUILD_ID="{build_id}"'] if os.path.basename(src) == ID_SOURCE else []
    cmd = [HIPCC] + flags_for(src) + defs + ['-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stderr}')
    with open(kfile, 'w') as f:
        f.write(key)
    return obj, r.stderr


def build(force=False, jobs=None, verbose=False):
    if not force and up_to_date():
        return LIB
    os.makedirs(OUT, exist_ok=True)
    srcs = _sources()
    bid = source_hash()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4) // 2), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, bid), srcs))
    for obj, err in results:
        if verbose and err.strip():
            print(err, file=sys.stderr)
    tmp = LIB + '.tmp'
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', tmp] + [o for o, _ in results]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed:\n{r.stderr}')
    if lib_build_id(tmp) != bid:
        raise RuntimeError(f'linked library does not carry build ID {bid}')
    os.replace(tmp, LIB)
    return LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--jobs', type=int, default=None)
    ap.add_argument('-v', '--verbose', action='store_true')
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.jobs, verbose=a.verbose), source_hash())
