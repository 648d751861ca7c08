"""Build timing-experiment variants of libnrhip.so into neurecon_amd/_exp/ (select one at run time
with NR_LIB=...).  Variants switch off parts of the MLP kernels (results are NOT valid) to measure
what each part costs: NR_EXP_NO_DMA, NR_EXP_NO_ESTORE, NR_EXP_NO_ELOAD, NR_EXP_NO_EPI, NR_EXP_NO_MFMA,
NR_EXP_NO_TRANS (epilogue transcendentals), NR_EXP_NO_EPISPLIT (next-operand split),
NR_EXP_SHARED_W (backward ops re-stream the forward weights: half the weight footprint).
NR_SDF4_NC=1 is a layout choice, not an experiment: its results are valid."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neurecon_amd import build as B  # noqa: E402

VARIANTS = {
    'base': [],
    # NOT for tgemm_kernel: its counted vmcnt waits include the DMA pieces, so without them asm loads
    # land after their registers are reused (r06: an illegal address, profiles/r06/tgemm_nodma_bound.txt)
    'nodma': ['-DNR_EXP_NO_DMA'],
    'noestore': ['-DNR_EXP_NO_ESTORE'],
    'noeload': ['-DNR_EXP_NO_ELOAD'],
    'noslab': ['-DNR_EXP_NO_ESTORE', '-DNR_EXP_NO_ELOAD'],
    'nosoftplus': ['-DNR_EXP_NO_SOFTPLUS'],
    'nosplit': ['-DNR_EXP_NO_SPLIT'],
    'nobarrier': ['-DNR_EXP_NO_BARRIER'],
    'novalu': ['-DNR_EXP_NO_SOFTPLUS', '-DNR_EXP_NO_SPLIT'],
    'unroll': ['-DNR_EXP_UNROLL'],
    'nopp': ['-DNR_EXP_NO_PINGPONG'],
    'v3nodma': ['-DNR_EXP_NO_DMA'],
    'v3nobar': ['-DNR_EXP_NO_BARRIER'],
    'v3noepi': ['-DNR_EXP_NO_EPI'],
    'v3nomfma': ['-DNR_EXP_NO_MFMA'],
    'v3noslab': ['-DNR_EXP_NO_ESTORE', '-DNR_EXP_NO_ELOAD'],
    'unroll_nosplit': ['-DNR_EXP_UNROLL', '-DNR_EXP_NO_SPLIT'],
    'v3notrans': ['-DNR_EXP_NO_TRANS'],
    'sharedw': ['-DNR_EXP_SHARED_W'],
    'v3noepisplit': ['-DNR_EXP_NO_EPISPLIT'],
    'v3nomfma_noepi': ['-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI'],
    # sdf4_kernel layouts (valid results): nc2 = 32-point waves, one per SIMD (the r02 default)
    'nc2': ['-DNR_SDF4_NC=2'],
    'ld4': ['-DNR_DMA_LOADERS=4'],
    'ld4s': ['-DNR_DMA_LOADERS=4', '-DNR_DMA_SPREAD'],
    'ld2': ['-DNR_DMA_LOADERS=2'],
    # per-phase shader-clock totals (tools/mlp_driver.py --stamps)
    'stamps': ['-DNR_EXP_STAMPS'],
    'stamps_nc2': ['-DNR_EXP_STAMPS', '-DNR_SDF4_NC=2'],
    'stamps_s': ['-DNR_EXP_STAMPS', '-DNR_DMA_SPREAD', '-DNR_VMEM_SPREAD'],
    'vs': ['-DNR_DMA_SPREAD', '-DNR_VMEM_SPREAD'],
    'ds': ['-DNR_DMA_SPREAD'],
    'prio': ['-DNR_SDF4_PRIO'],
    'mid': ['-DNR_MID_FLIP'],
    'mid_nc2': ['-DNR_MID_FLIP', '-DNR_SDF4_NC=2'],
    'nc1': ['-DNR_SDF4_NC=1'],
    'nc1nodma': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_DMA'],
    'nc1nobar': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_BARRIER'],
    'nc1noepi': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_EPI'],
    'nc1nomfma': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA'],
    'nc1nomfma_noepi': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI'],
    'nc1noslab': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_ESTORE', '-DNR_EXP_NO_ELOAD'],
    'nc1notrans': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_TRANS'],
    # skeleton decomposition (no MFMA, no epilogue): DMA only / fragment reads only / no barrier
    'nc1sk_noaread': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI', '-DNR_EXP_NO_AREAD'],
    'nc1sk_nodma': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI', '-DNR_EXP_NO_DMA'],
    'nc1sk_nobar': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI', '-DNR_EXP_NO_BARRIER'],
    'nc1sk_noslab': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI', '-DNR_EXP_NO_ESTORE', '-DNR_EXP_NO_ELOAD'],
    'nc1sk_dmaonly': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_MFMA', '-DNR_EXP_NO_EPI', '-DNR_EXP_NO_AREAD',
                      '-DNR_EXP_NO_ESTORE', '-DNR_EXP_NO_ELOAD'],
    'nc1noaread': ['-DNR_SDF4_NC=1', '-DNR_EXP_NO_AREAD'],
    # B operands in VGPRs (no AGPR moves; valid results)
    'nc1v': ['-DNR_SDF4_NC=1', '-DNR_SPLIT_VGPR'],
    # weight DMA pieces spread over the k-step regions (valid results)
    'nc1vs': ['-DNR_SDF4_NC=1', '-DNR_SPLIT_VGPR', '-DNR_DMA_SPREAD'],
    'nc2s': ['-DNR_DMA_SPREAD'],
    'nc1vnoepi': ['-DNR_SDF4_NC=1', '-DNR_SPLIT_VGPR', '-DNR_EXP_NO_EPI'],
    'nc2noepi': ['-DNR_EXP_NO_EPI'],
    # slab stores with the default cache policy instead of nt (valid results)
    'slabt': ['-DNR_SLAB_NT=false'],
    'sldnt': ['-DNR_SLAB_LD_POL=" nt"'],      # the default since r03
    'sldt': ['-DNR_SLAB_LD_POL=""'],          # slab loads with the default policy (the r02 build)
    'sldnt_fnt': ['-DNR_SLAB_LD_POL=" nt"', '-DNR_FEAT_NT=true'],
    # nr_wgrad cost split (results NOT valid): no MFMA / no split+LDS store / no global loads
    'wg_nomfma': ['-DNR_WG_EXP_NO_MFMA'],
    'wg_nostore': ['-DNR_WG_EXP_NO_STORE'],
    'wg_loadonly': ['-DNR_WG_EXP_NO_MFMA', '-DNR_WG_EXP_NO_STORE'],
    'wg_noload': ['-DNR_WG_EXP_NO_LOAD'],
    # nr_wgrad phase split between the two waves of a SIMD (valid results): waves w & 4 / adjacent waves
    'wg_pp4': ['-DNR_WG_PP_BIT=4'],
    'wg_pp1': ['-DNR_WG_PP_BIT=1'],
    # r05: the forward-only sdf4_kernel launches with the r04 3-slot weight ring (valid results)
    'ring3': ['-DNR_FWD_RING=3'],
    # r05: fp32 magic-number slab codes (one fma to write, one fma + mul to read; 8 instead of 6 KB / point)
    'slab32': ['-DNR_SLAB32'],
    'slab32prio': ['-DNR_SLAB32', '-DNR_SDF4_PRIO'],
    # r05: tgemm_kernel without the next-tile input prefetch (the r04 schedule; valid results)
    'tgxpf0': ['-DNR_TG_XPF=0'],
    'tgxpf4': ['-DNR_TG_XPF_PER=4'],
    'tgxpf_p4s12': ['-DNR_TG_XPF_PER=4', '-DNR_TG_XPF_SPADJ=12'],
    # r05: tgemm weight ring of 4 slots (three chunks in flight) / 3 slots drained at every barrier (r04)
    'tgring4': ['-DNR_TG_RING=4'],
    'tgdrain': ['-DNR_TG_DRAIN=1'],
    # nr_wgrad slice count from $NR_WGRAD_SLICES (tools/wgrad_bench.py)
    'wg_slices_env': ['-DNR_WG_EXP_SLICES_ENV'],
    # r05: nr_wgrad.hip built with -fno-slp-vectorize (VARIANT_FILE_FLAGS; valid results)
    'wgnoslp': [],
}
# flags for one source file of a variant only
VARIANT_FILE_FLAGS = {'wgnoslp': {'nr_wgrad.hip': ['-fno-slp-vectorize']}}


def one(name):
    out_dir = os.environ.get('NR_EXP_DIR', os.path.join(ROOT, 'neurecon_amd', '_exp'))
    objs = []
    for src in B._sources():
        obj = os.path.join(out_dir, f'{name}_{os.path.basename(src)}.o')
        extra = VARIANT_FILE_FLAGS.get(name, {}).get(os.path.basename(src), [])
        subprocess.check_call([B.HIPCC] + B.flags_for(src) + ['-DNR_VARIANT_BUILD'] + VARIANTS[name] + extra +
                              ['-c', src, '-o', obj])
        objs.append(obj)
    lib = os.path.join(out_dir, f'libnrhip_{name}.so')
    subprocess.check_call([B.HIPCC, '-shared', '-fPIC', f'--offload-arch={B.ARCH}', '-o', lib] + objs)
    return lib


def main(names):
    import concurrent.futures as cf
    os.makedirs(os.environ.get('NR_EXP_DIR', os.path.join(ROOT, 'neurecon_amd', '_exp')), exist_ok=True)
    with cf.ThreadPoolExecutor(4) as ex:
        for lib in ex.map(one, names):
            print(lib)


if __name__ == '__main__':
    main(sys.argv[1:] or list(VARIANTS))
