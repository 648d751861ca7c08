"""Build timing-experiment variants of libnrhip.so into neurecon_amd/_exp/ (select one at run time
with NR_LIB=...).  Variants switch off parts of the MLP kernels (results are NOT valid) to measure
what each part costs: NR_EXP_NO_DMA, NR_EXP_NO_ESTORE, NR_EXP_NO_ELOAD."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neurecon_amd import build as B  # noqa: E402

VARIANTS = {
    'base': [],
    'nodma': ['-DNR_EXP_NO_DMA'],
    'noestore': ['-DNR_EXP_NO_ESTORE'],
    'noeload': ['-DNR_EXP_NO_ELOAD'],
    'noslab': ['-DNR_EXP_NO_ESTORE', '-DNR_EXP_NO_ELOAD'],
}


def main(names):
    out_dir = os.path.join(ROOT, 'neurecon_amd', '_exp')
    os.makedirs(out_dir, exist_ok=True)
    for name in names:
        objs = []
        for src in B._sources():
            obj = os.path.join(out_dir, f'{name}_{os.path.basename(src)}.o')
            subprocess.check_call([B.HIPCC] + B.FLAGS + VARIANTS[name] + ['-c', src, '-o', obj])
            objs.append(obj)
        lib = os.path.join(out_dir, f'libnrhip_{name}.so')
        subprocess.check_call([B.HIPCC, '-shared', '-fPIC', f'--offload-arch={B.ARCH}', '-o', lib] + objs)
        print(lib)


if __name__ == '__main__':
    main(sys.argv[1:] or list(VARIANTS))
