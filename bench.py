"""Benchmark: NeuS volume rendering, 4096 rays x 128 samples, 8x256 SDF MLP (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...   (same layout)

A step = one `volume_render` call (render mode: torch.no_grad, perturb=False, calc_normal=True,
detailed_output=False) over one 4096-ray batch of the synthetic config-(b) camera (64x64 pixels,
f=160, camera at distance 3 looking at a radius-0.5 geometric-init sphere; random-init weights of
the configs/neus.yaml architecture -- no datasets offline).  Rays are already resident in HBM.

Multi-GPU: one process per GPU over RCCL.  Under torchrun the ranks come from its environment;
`python bench.py --gpus N` alone spawns the N rank processes itself (before any GPU call) with the
same environment.  n_gpus is the process group's size (asserted equal to --gpus).
  * `value`: every rank renders its own 4096-ray batch (weak scaling, no data-path collective);
    value = all ranks' rays / max-over-ranks time of K steps.
  * `strong_scaling_frame_d`: one config-(d) 800x600 NeuS+NeRF++ frame per step, its rays split
    over the ranks (neurecon_amd.dist.render_sharded) and the maps all-gathered inside the timed
    region; rays/s of the frame at this N (strong scaling).
  * `weak_scaling_e`: config (e) UNISURF, 4096 rays per rank as the rank's contiguous share of one
    N x 4096-ray batch row: the windowed F.normalize spans ranks, so every render all-reduces the
    per-window sums of nabla^2 (RCCL) inside the timed region.
  * `weak_scaling_train`: the NeuS training step, 512 rays per rank, DDP (RCCL gradient all-reduce
    in backward) at N > 1.
Prints one JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X dense fp32 matrix (MI355X_MICROARCH.md)
F16_MFMA_PEAK_TFLOPS = 2500.0     # MI355X dense fp16/bf16 matrix (MI355X_MICROARCH.md; sparsity excluded)
# f16x3 spends 3 fp16 MFMA products (hi*hi + hi*lo + lo*hi) per algorithmic fp32 MAC
F16X3_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 3
MAC_SDF_FWD = 524_544             # SURVEY §8(a) A5 (incl. the 257-row last layer)
MAC_SDF_FWD_NOFEAT = 459_008      # the same without the 256 geometry-feature rows (sdf row only)
MAC_SDF_BWD = 459_008             # SURVEY §8(a) A6 (reverse pass for the nablas)
MAC_RAD = 271_360                 # SURVEY §8(a) A7, NeuS radiance input 289
# NeRF++ background net (base.py:395-424, neus.py:38: input 4 -> 84 embedded, view 27, D=8 W=256,
# skip at layer 5): 84*256 + 6*256*256 + 340*256 + feature 256*256 + alpha 256 + views 283*128 + rgb 128*3
MAC_NERF = 604_160
# reference algorithm per ray: 128 no-grad SDF + 255 SDF-with-nabla + 127 radiance.
# This path evaluates each of the 128 samples once (SDF + nabla when it is drawn):
# 128 + 127 SDF-with-nabla + 127 radiance; step_tflops counts that executed work.
RAY_FLOP_REF = 704.8e6
RAY_FLOP = 2.0 * (255 * (MAC_SDF_FWD + MAC_SDF_BWD) + 127 * MAC_RAD)
# HBM-side bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 --pmc passes of this bench,
# tools/gpu_pmc.sh); counters cannot be read live, so the latest committed summary is reported.
PMC_SUMMARY = {'f16x3': 'profiles/r06/f16x3_pmc_summary.json'}  # tools/gpu_final_r06.sh PROFILES=1 (PMC passes of the default bench)
# matrix-pipe occupancy and effective clock per nabla launch type (rocprofv3 GRBM_GUI_ACTIVE and
# SQ_VALU_MFMA_BUSY_CYCLES passes of this bench, tools/gpu_mfma_r05.sh -> tools/mfma_summary.py)
MFMA_SUMMARY = 'profiles/r06/mfma_summary.json'
MFMA_KERNEL = {'sdf_nabla_fwd': 'void nr::sdf4_kernel<true, false, 1>(nr::SdfKArgs)',
               'sdf_nabla_bwd': 'void nr::sdf4_kernel<true, false, 4>(nr::SdfKArgs)',  # r06: the compacted pass
               'sdf_nabla_feat': 'void nr::sdf4_kernel<true, true, 0>(nr::SdfKArgs)'}
# device kernels behind each merged library kernel name (sdf_nabla = samples + mid-points launches)
PMC_KERNEL = {('sdf_nabla', 'f16x3'): ('void nr::sdf4_kernel<true, false>(nr::SdfKArgs)',       # r02 names
                                       'void nr::sdf4_kernel<true, true>(nr::SdfKArgs)',
                                       # r03: deferred sample nablas (forward + slabs, reverse pass), mid-points
                                       'void nr::sdf4_kernel<true, false, 1>(nr::SdfKArgs)',
                                       'void nr::sdf4_kernel<true, false, 2>(nr::SdfKArgs)',
                                       'void nr::sdf4_kernel<true, true, 0>(nr::SdfKArgs)',
                                       # r06: the reverse pass over listed samples (chunks <= 671 072 slots)
                                       'void nr::sdf4_kernel<true, false, 4>(nr::SdfKArgs)'),
              ('sdf_nabla', 'fp32'): ('void nr::sdf_kernel<0, true>(nr::SdfKArgs)',)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='number of GPUs (one process each); outside torchrun, N > 1 spawns the N rank processes')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--rays', type=int, default=4096)
    ap.add_argument('--precision', default=os.environ.get('NR_PRECISION', 'f16x3'), choices=['f16x3', 'fp32'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-full-eval', action='store_true',
                    help='skip the second timed loop that evaluates every mid-point (profiling runs)')
    ap.add_argument('--workload', default='b', choices=['b', 'frame_d', 'train'],
                    help="b: the BASELINE metric (default); frame_d: config (d) full frame sharded over the GPUs; "
                         "train: NeuS training step")
    ap.add_argument('--train-rays', type=int, default=512)
    ap.add_argument('--train-nerfpp', action='store_true',
                    help='--workload train with the NeRF++ background (configs/neus_nomask_blended.yaml)')
    ap.add_argument('--adam', default='nr', choices=['nr', 'fused', 'foreach'],
                    help="the training workload's Adam: nr = neurecon_amd.optim.Adam (one nr_adam_step launch), "
                         "fused / foreach = torch.optim.Adam's implementations")
    ap.add_argument('--cpu-rays', type=int, default=1024)
    ap.add_argument('--no-frame', action='store_true',
                    help='skip the strong-scaling config-(d) frame leg of the default workload')
    ap.add_argument('--frame-steps', type=int, default=3)
    ap.add_argument('--workspace-gb', type=float, default=None,
                    help="config-(b) render workspace budget (volume_render's max_workspace_gb); default: the "
                         "library's 4 GiB, within which the 4096-ray batch renders as one chunk")
    ap.add_argument('--frame-workspace-gb', type=float, default=16.0,
                    help="workspace budget of the 480,000-ray config-(d) frame render (chunks of up to 16384 rays "
                         "keep the per-ray kernels on the whole chip; the caller's choice on a 288 GB GPU)")
    ap.add_argument('--no-configs', action='store_true',
                    help='skip the BASELINE configs (c), (e) and the training step in the default line')
    ap.add_argument('--config-steps', type=int, default=5)
    ap.add_argument('--no-scaling-legs', action='store_true',
                    help='skip the weak-scaling config-(e) and DDP-training legs of the default workload')
    ap.add_argument('--leg-steps', type=int, default=5)
    ap.add_argument('--no-fp32-mode', action='store_true',
                    help='skip the exact-fp32 rate of config (b) beside the f16x3 headline')
    ap.add_argument('--stub-cpu', action='store_true', help=argparse.SUPPRESS)
    return ap.parse_args()


def make_model(device, precision, outside=False):
    from neurecon_amd.frameworks.neus import NeuS
    torch.manual_seed(0)
    surf = dict(use_siren=False, embed_multires=6, radius_init=0.5, geometric_init=True, D=8, W=256, skips=[4],
                precision=precision)
    rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=4, use_view_dirs=True, D=4, W=256, skips=[],
               precision=precision)
    m = NeuS(variance_init=0.05, speed_factor=10.0, W_geo_feat=256, use_outside_nerf=outside, obj_bounding_radius=1.0,
             surface_cfg=surf, radiance_cfg=rad)
    return m.to(device).eval()


def camera(device):
    """config (b): c2w = look_at((0,0,-3) -> origin, up (0,-1,0)), K = [[160,0,32],[0,160,32],[0,0,1]]"""
    import numpy as np
    cam = np.array([0.0, 0.0, -3.0])
    fwd = -cam / np.linalg.norm(cam)
    x = np.cross([0.0, -1.0, 0.0], fwd); x /= np.linalg.norm(x)
    y = np.cross(fwd, x)
    c2w = np.eye(4); c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = x, y, fwd, cam
    K = np.eye(4); K[0, 0] = K[1, 1] = 160.0; K[0, 2] = K[1, 2] = 32.0
    return (torch.tensor(c2w, dtype=torch.float32, device=device)[None],
            torch.tensor(K, dtype=torch.float32, device=device)[None])


def render_kwargs():
    return dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, perturb=False,
                N_samples=64, N_importance=64, N_outside=0, upsample_algo='official_solution', N_upsample_iters=4)


def host_cpu():
    """model name and logical CPU count from lscpu (the box's CPU, of which we use `threads`)"""
    import subprocess
    info = {}
    try:
        for line in subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout.splitlines():
            k, _, v = line.partition(':')
            if k.strip() in ('Model name', 'CPU(s)', 'Socket(s)', 'Core(s) per socket'):
                info[k.strip()] = v.strip()
    except Exception:
        pass
    return info


def cpu_baseline(n_rays, reps=3):
    """Oracle (clean-room CPU restatement, parity-pinned to the reference) timed on the host cores:
    warm-up, then the median of `reps` runs over a bounded sample of the config-(b) rays
    (BASELINE.md §3)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    from oracle.neus import NeuSOracle
    from oracle import rays as orays
    threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
    threads = max(1, min(threads, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    m = make_model('cpu', 'fp32')
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    orc = NeuSOracle(sd)
    c2w, K = camera('cpu')
    ro, rd, _ = orays.get_rays(c2w, K, 64, 64)
    if n_rays < 4096:
        idx = torch.linspace(0, 4095, n_rays).round().long()
        ro, rd = ro[:, idx], rd[:, idx]
    times = []
    with torch.no_grad():
        orc.render(ro[:, :64], rd[:, :64])  # warm-up
        for _ in range(reps):
            t = time.perf_counter()
            orc.render(ro, rd)
            times.append(time.perf_counter() - t)
    dt = sorted(times)[len(times) // 2]
    cpu = host_cpu()
    return {'value': round(n_rays / dt, 2), 'unit': 'rays/s', 'cores': threads, 'kind': 'port',
            'host_cpu': cpu,
            'cores_note': 'BASELINE.md section 3 asks for all host cores; the GPU lease grants one GPU\'s CPU share '
                          f'(OMP_NUM_THREADS={os.environ.get("OMP_NUM_THREADS", "unset")} is set by the box, which '
                          'forbids using more: the other cores belong to the other GPUs\' jobs), so the oracle runs '
                          'on that many threads; lscpu\'s count is the whole machine',
            'sample': f'{n_rays} of the 4096 config-(b) rays (evenly spaced), oracle/neus.py, torch {torch.__version__} '
                      f'CPU fp32, {threads} threads of {cpu.get("CPU(s)", "?")} logical CPUs '
                      f'({cpu.get("Model name", "?")}), warm-up + median of {reps}: {dt:.2f} s per run'}


def eager_gpu_baseline(dev, n_rays, reps=3):
    """The same oracle (op-for-op the reference's eager PyTorch sequence, fp32) run on the GPU with
    PyTorch-ROCm: the north star's "reference single-GPU PyTorch-ROCm" denominator,
    since the reference itself cannot travel to the box.  Part of the baseline leg, never the product."""
    from oracle.neus import NeuSOracle
    from neurecon_amd import rend_util
    m = make_model(dev, 'fp32')
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    c2w, K = camera(dev)
    ro, rd, _ = rend_util.get_rays(c2w, K, 64, 64)
    ro, rd = ro[:, :n_rays].contiguous(), rd[:, :n_rays].contiguous()
    prev = torch.get_default_device()
    torch.set_default_device(dev)   # the oracle's linspace/ones tables follow the rays' device
    try:
        orc = NeuSOracle(sd)
        times = []
        with torch.no_grad():
            orc.render(ro, rd)  # warm-up
            for _ in range(reps):
                torch.cuda.synchronize()
                t = time.perf_counter()
                orc.render(ro, rd)
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t)
    finally:
        torch.set_default_device(prev)
    dt = sorted(times)[len(times) // 2]
    return {'value': round(n_rays / dt, 1), 'unit': 'rays/s', 'kind': 'port', 'device': torch.cuda.get_device_name(dev),
            'sample': f'{n_rays} config-(b) rays in one chunk, oracle/neus.py eager fp32 on 1 GPU, median of {reps}, '
                      f'{dt * 1e3:.1f} ms'}


# MACs per unit (point) that each library kernel executes (SURVEY.md §8(a) layer shapes): launches
# without the geometry feature skip its 256 rows of the last layer
KERNEL_MAC = {'sdf_fwd': MAC_SDF_FWD_NOFEAT, 'sdf_feat': MAC_SDF_FWD, 'sdf_nabla': MAC_SDF_FWD_NOFEAT + MAC_SDF_BWD,
              'sdf_nabla_feat': MAC_SDF_FWD + MAC_SDF_BWD, 'radiance': MAC_RAD, 'nerf': MAC_NERF,
              # deferred sample nablas: forward of every sample, reverse pass of the samples of non-zero
              # weight (units = listed samples; r03-r05 and chunks past 671 072 slots: their 16-point tiles)
              'sdf_nabla_fwd': MAC_SDF_FWD_NOFEAT, 'sdf_nabla_bwd': MAC_SDF_BWD,
              # training GEMMs report MACs (padded 16x16 blocks) as their units
              'train_gemm': 1}


def pmc_traffic(kernel, precision):
    """HBM bytes per launch of `kernel`, averaged over the launches of every device kernel behind it
    (the same launch mix the live HIP-event average covers)."""
    path = os.path.join(ROOT, PMC_SUMMARY.get(precision, '-'))
    names = PMC_KERNEL.get((kernel, precision))
    if not names or not os.path.exists(path):
        return None, None
    with open(path) as f:
        summary = json.load(f)
    recs = [summary[n] for n in names if n in summary]
    n = sum(r['launches'] for r in recs)
    if not n:
        return None, None
    return sum(r['hbm_bytes_per_launch'] * r['launches'] for r in recs) / n, PMC_SUMMARY[precision]


# L2 -> LDS weight stream of sdf4_kernel: every 128-point tile streams the whole packed network
# (nr_mlp.h kSdfKB / kSdfNBO: 3.93 MB without the feature op, 4.20 MB with it), by LDS-DMA, whose
# chip-wide fill rate is ~6.4 TB/s (MI355X_MICROARCH.md, 'ldsdma-fill'); f16x3 only
SDF_TILE_POINTS = 128
# (r03 deferred nablas: the sample launches stream F0..F7 only, the reverse-pass launch B7..B0 per
# 8 x 16-point tiles = 128 points; nr_sdf_op_info offsets)
SDF_PACKED_BYTES = {'sdf_nabla': 3_926_016, 'sdf_nabla_feat': 4_196_352, 'sdf_nabla_fwd': 1_965_056,
                    'sdf_nabla_bwd': 1_962_752}
LDSDMA_FILL_TBPS = 6.4


def weight_stream(kstats):
    """bytes the nabla launches (every launch type) streamed into LDS / their device time"""
    nb, ms = 0.0, 0.0
    for name, (n, t, units) in kstats.items():
        if name in SDF_PACKED_BYTES and n:
            nb += math.ceil(units / n / SDF_TILE_POINTS) * n * SDF_PACKED_BYTES[name]
            ms += t
    if not ms:
        return None
    tbps = nb / (ms * 1e-3) / 1e12
    return {'bytes_per_launch_avg': nb / sum(kstats[k][0] for k in SDF_PACKED_BYTES if k in kstats),
            'achieved_TBps': round(tbps, 2), 'ldsdma_fill_TBps': LDSDMA_FILL_TBPS,
            'frac': round(tbps / LDSDMA_FILL_TBPS, 3)}


def roofline(kstats, precision, census=None):
    """Dominant kernel (largest device time): executed FLOPs per launch / mean launch duration, both
    launch types of the nabla kernel merged (sample launches without the feature rows, the
    mid-point launch with them), plus each launch type on its own.  kstats: the timed steps (the
    dominant kernel's launches); census: every library kernel (per-kernel table, device-time share)."""
    peak = FP32_MFMA_PEAK_TFLOPS if precision == 'fp32' else F16X3_PEAK_TFLOPS
    per_type = {}
    for name, (n, ms, units) in kstats.items():
        if name.startswith('sdf_nabla') and n:
            fl = units * 2.0 * KERNEL_MAC[name]
            per_type[name] = {'launches': n, 'avg_launch_ms': round(ms / n, 4),
                              'achieved': round(fl / (ms * 1e-3) / 1e12, 2),
                              'frac': round(fl / (ms * 1e-3) / 1e12 / peak, 4)}
    # the sdf_kernel<nabla> launch types (samples, reverse pass, mid-points) are one kernel
    def merge(ks):
        merged = {}
        for name, (n, ms, units) in ks.items():
            key = 'sdf_nabla' if name.startswith('sdf_nabla') else name
            a = merged.setdefault(key, [0, 0.0, 0.0])
            a[0] += n; a[1] += ms; a[2] += units * 2.0 * KERNEL_MAC.get(name, 0)
        return merged
    table = merge(census if census is not None else kstats)
    total_ms = sum(v[1] for v in table.values())
    for name, (n, ms, fl) in sorted(table.items(), key=lambda kv: -kv[1][1]):
        print(f'[bench] {name:16s} launches {n:5d}  {ms:9.3f} ms ({100 * ms / max(total_ms, 1e-9):5.1f}%)  '
              f'{fl / max(ms, 1e-9) / 1e9:8.2f} TFLOP/s', file=sys.stderr)
    dom, (n, ms, fl) = max(merge(kstats).items(), key=lambda kv: kv[1][1])
    share = table[dom][1] / total_ms if dom in table and total_ms else 1.0
    per_launch_ms = ms / n
    achieved = fl / n / (per_launch_ms * 1e-3) / 1e12
    traffic, src = pmc_traffic(dom, precision)
    ev = mfma_evidence(per_type) if precision == 'f16x3' else None
    return {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': peak, 'unit': 'TFLOP/s',
            'frac': round(achieved / peak, 4), 'traffic': traffic, 'traffic_unit': 'bytes/launch',
            'traffic_source': src, 'kernel': dom,
            'avg_launch_ms': round(per_launch_ms, 4), 'launches': n,
            'flop_per_launch': fl / n, 'share_of_device_time': round(share, 4),
            'mfma_busy': ev['mfma_busy'] if ev else None, 'clock_ghz': ev['clock_ghz'] if ev else None,
            'mfma_evidence': ev,
            'per_launch_type': per_type,
            'weight_stream': weight_stream(kstats) if precision == 'f16x3' else None}


def mfma_evidence(per_type):
    """per launch type: mfma_busy (fraction of SIMD-cycles the matrix pipe was busy) and clock_ghz from
    the committed counter summary; the merged kernel's values weighted by each type's device time"""
    path = os.path.join(ROOT, MFMA_SUMMARY)
    if not os.path.exists(path) or not per_type:
        return None
    with open(path) as f:
        summary = json.load(f)
    out, wsum, busy, clk = {}, 0.0, 0.0, 0.0
    for name, rec in per_type.items():
        r = summary.get(MFMA_KERNEL.get(name, '-'))
        if not r or 'mfma_busy' not in r:
            continue
        out[name] = {'mfma_busy': round(r['mfma_busy'], 4), 'clock_ghz': round(r['clock_ghz'], 3)}
        w = rec['avg_launch_ms'] * rec['launches']
        wsum += w
        busy += w * r['mfma_busy']
        clk += w * r['clock_ghz']
    if not wsum:
        return None
    return {'mfma_busy': round(busy / wsum, 4), 'clock_ghz': round(clk / wsum, 3), 'per_launch_type': out,
            'source': MFMA_SUMMARY,
            'note': 'rocprofv3 --pmc passes of this bench (GRBM_GUI_ACTIVE; SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x '
                    'cycles)); counters cannot be read inside the timed run, so the committed summary of the same '
                    'build is reported'}


HBM_PEAK_TBPS = 8.0  # MI355X HBM3E (MI355X_MICROARCH.md)


TRAIN_PMC_SUMMARY = 'profiles/r06/train_pmc_summary.json'  # tools/gpu_final_r06.sh PROFILES=1 (PMC passes of --workload train)


def train_pmc_traffic(prefix):
    """HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE) averaged over the training bench's launches
    of every device kernel whose name contains `prefix`, from the committed PMC summary"""
    path = os.path.join(ROOT, TRAIN_PMC_SUMMARY)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        summary = json.load(f)
    recs = [r for k, r in summary.items() if prefix in k]
    n = sum(r['launches'] for r in recs)
    if not n:
        return None, None
    return sum(r['hbm_bytes_per_launch'] * r['launches'] for r in recs) / n, TRAIN_PMC_SUMMARY


def train_roofline(kstats, dt, steps, census=None):
    """Training step: the dominant library kernel is the layer GEMM (nr_train_gemm), whose launches
    stream [P, <=288] fp32 activations: HBM-bound.  achieved = algorithmic bytes of its calls (inputs,
    outputs, epilogue operands; training.TG_BYTES, counted per call by the host) / their device time.
    share_of_step: the library kernels' device time / the step time (the rest: torch elementwise and
    the losses, Adam; r05: no hipBLASLt GEMM is left in the step)."""
    from neurecon_amd import training as T
    n, ms, _ = kstats.get('train_gemm', (0, 0.0, 0.0))
    lib_ms = sum(v[1] for v in (census if census is not None else kstats).values())
    if not n:
        return None
    by = T.TG_BYTES['bytes'] / max(T.TG_BYTES['calls'], 1) * n  # bytes of the timed launches
    tbps = by / (ms * 1e-3) / 1e12
    traffic, src = train_pmc_traffic('tgemm_kernel')
    out = {'bound': 'hbm', 'achieved': round(tbps, 3), 'peak': HBM_PEAK_TBPS, 'unit': 'TB/s',
           'frac': round(tbps / HBM_PEAK_TBPS, 4), 'traffic': traffic, 'traffic_unit': 'bytes/launch',
           'traffic_source': src, 'kernel': 'train_gemm',
           'avg_launch_ms': round(ms / n, 4), 'launches': n, 'bytes_per_launch': by / n,
           'share_of_library_time': round(ms / max(lib_ms, 1e-9), 4),
           'library_share_of_step': round(lib_ms * 1e-3 / max(dt, 1e-12), 4)}
    # the weight-gradient kernel (nr_wgrad): units = operand bytes (npairs P (m + n) 4), HBM-bound
    wc = (census if census is not None else kstats).get('wgrad')
    if wc and wc[0]:
        nw, msw, byw = wc
        wtraffic, wsrc = train_pmc_traffic('wgrad_kernel')
        out['wgrad'] = {'bound': 'hbm', 'achieved': round(byw / (msw * 1e-3) / 1e12, 3), 'peak': HBM_PEAK_TBPS,
                        'unit': 'TB/s', 'frac': round(byw / (msw * 1e-3) / 1e12 / HBM_PEAK_TBPS, 4),
                        'launches_per_step': round(nw / steps, 1), 'avg_launch_ms': round(msw / nw, 4),
                        'bytes_per_launch': byw / nw, 'traffic': wtraffic, 'traffic_source': wsrc,
                        'share_of_library_time': round(msw / max(lib_ms, 1e-9), 4)}
    return out


def frame_d_inputs(dev, precision, workspace_gb=None):
    """config (d)'s model, rays [1, 480000, 3] and volume_render kwargs (frame_d_setup; also the
    full-frame test, tests/test_gpu_frame.py)."""
    import numpy as np
    from neurecon_amd import rend_util
    from neurecon_amd.frameworks.neus import NeuS
    torch.manual_seed(0)
    surf = dict(use_siren=False, embed_multires=6, radius_init=0.5, geometric_init=True, D=8, W=256, skips=[4],
                precision=precision)
    rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=4, use_view_dirs=True, D=4, W=256, skips=[],
               precision=precision)
    model = NeuS(variance_init=0.05, speed_factor=10.0, W_geo_feat=256, use_outside_nerf=True, obj_bounding_radius=1.0,
                 surface_cfg=surf, radiance_cfg=rad).to(dev).eval()
    H, W, f, dist = 600, 800, 800.0, 2.0
    cam = np.array([0.0, 0.0, -dist])
    fwd = -cam / np.linalg.norm(cam)
    x = np.cross([0.0, -1.0, 0.0], fwd); x /= np.linalg.norm(x)
    y = np.cross(fwd, x)
    c2w = np.eye(4); c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = x, y, fwd, cam
    K = np.eye(4); K[0, 0] = K[1, 1] = f; K[0, 2] = W / 2; K[1, 2] = H / 2
    ro, rd, _ = rend_util.get_rays(torch.tensor(c2w, dtype=torch.float32, device=dev)[None],
                                   torch.tensor(K, dtype=torch.float32, device=dev)[None], H, W)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, perturb=False,
              N_samples=64, N_importance=64, N_outside=32, upsample_algo='official_solution', N_upsample_iters=4,
              max_workspace_gb=workspace_gb)
    return model, ro, rd, kw, H * W


def frame_d_setup(dev, precision, workspace_gb=None):
    """config (d): NeuS + NeRF++ (N_outside=32), full 800x600 frame of the config-(d) camera (H=600,
    W=800, f=800, camera at distance 2), rays sharded over the ranks; the frame's maps are
    all-gathered (RCCL) inside the timed step."""
    from neurecon_amd import dist as nd
    from neurecon_amd.frameworks.neus import volume_render
    model, ro, rd, kw, n = frame_d_inputs(dev, precision, workspace_gb)

    def step():
        with torch.no_grad():
            return nd.render_sharded(volume_render, ro, rd, model, gather=True, **kw)
    return step, n


def train_setup(dev, precision, n_rays, world, adam='nr', nerfpp=False):
    """NeuS training step (configs/neus.yaml: N_rays=512 per rank, perturb=True, with_mask): random
    rays of a synthetic 64x64 image, render with the autograd graph (neurecon_amd.training), the
    reference's losses, backward (DDP gradient all-reduce over RCCL when world > 1), Adam.
    nerfpp=True: configs/neus_nomask_blended.yaml's model (NeRF++ background, N_outside 32, no mask loss)."""
    import types
    from neurecon_amd.frameworks.neus import Trainer
    model = make_model(dev, precision, outside=nerfpp)
    model.train()
    trainer = Trainer(model, device_ids=[dev.index or 0])
    if world > 1:
        from torch.nn.parallel import DistributedDataParallel as DDP
        trainer = DDP(trainer, device_ids=[dev.index or 0])
    # the reference's optimizer (torch.optim.Adam, models/base.py:488): by default neurecon_amd.optim.Adam,
    # the same update in one nr_adam_step launch (torch's fused form: two multi-tensor launches, ~90 us;
    # its default foreach form costs ~0.3 ms of Python per step here)
    if adam == 'nr':
        from neurecon_amd.optim import Adam
        opt = Adam(model.parameters(), lr=5e-4)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=5e-4, fused=(adam == 'fused'))
    c2w, K = camera(dev)
    g = torch.Generator().manual_seed(1)
    mi = {'intrinsics': K, 'c2w': c2w, 'object_mask': (torch.rand(1, 4096, generator=g) > 0.5).to(dev)}
    gt = {'rgb': torch.rand(1, 4096, 3, generator=g).to(dev)}
    a = types.SimpleNamespace(data=types.SimpleNamespace(N_rays=n_rays),
                              training=types.SimpleNamespace(w_eikonal=0.1, w_mask=0.0 if nerfpp else 1.0,
                                                             with_mask=not nerfpp))
    kw = dict(H=64, W=64, upsample_algo='official_solution', N_nograd_samples=2048, N_upsample_iters=4,
              N_outside=32 if nerfpp else 0, obj_bounding_radius=1.0, batched=True, perturb=True, white_bkgd=False)

    def step():
        ret = trainer(a, None, mi, gt, kw, 0, device=dev)
        opt.zero_grad()
        ret['losses']['total'].backward()
        opt.step()
    return step


def camera_for(device, H, W, f, dist):
    """SURVEY §8(d) synthetic camera: look_at((0,0,-dist) -> origin, up (0,-1,0)), K = [[f,0,W/2],[0,f,H/2]]"""
    import numpy as np
    from neurecon_amd import rend_util
    cam = np.array([0.0, 0.0, -dist])
    fwd = -cam / np.linalg.norm(cam)
    x = np.cross([0.0, -1.0, 0.0], fwd); x /= np.linalg.norm(x)
    y = np.cross(fwd, x)
    c2w = np.eye(4); c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = x, y, fwd, cam
    K = np.eye(4); K[0, 0] = K[1, 1] = f; K[0, 2] = W / 2; K[1, 2] = H / 2
    return rend_util.get_rays(torch.tensor(c2w, dtype=torch.float32, device=device)[None],
                              torch.tensor(K, dtype=torch.float32, device=device)[None], H, W)[:2]


def _census(fn, steps, warmup, sync):
    """wall time per step of `steps` calls, then one more pass with every library launch timed by HIP
    events: ({kernel: (launches, ms, units)} per step)"""
    from neurecon_amd import _lib as L
    for _ in range(warmup):
        fn()
    sync()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    dt = (time.perf_counter() - t) / steps
    L.profile_read()
    L.profile_enable(True)
    try:
        fn()
        sync()
    finally:
        L.profile_enable(False)
    return dt, L.profile_read()


def _kernel_summary(ks, precision, rad_in):
    """per library kernel: ms per step and share; the dominant MLP kernel's executed-FLOP roofline"""
    peak = FP32_MFMA_PEAK_TFLOPS if precision == 'fp32' else F16X3_PEAK_TFLOPS
    mac = dict(KERNEL_MAC, radiance=rad_in * 256 + 3 * 256 * 256 + 3 * 256)
    total = sum(v[1] for v in ks.values()) or 1e-9
    table = {k: {'launches': n, 'ms': round(ms, 4), 'share': round(ms / total, 4)}
             for k, (n, ms, u) in sorted(ks.items(), key=lambda kv: -kv[1][1])}
    mlp = {k: v for k, v in ks.items() if k in mac and k != 'train_gemm' and v[0]}
    dom = None
    if mlp:
        k, (n, ms, units) = max(mlp.items(), key=lambda kv: kv[1][1])
        tf = units * 2.0 * mac[k] / (ms * 1e-3) / 1e12
        dom = {'kernel': k, 'bound': 'mfma', 'launches': n, 'avg_launch_ms': round(ms / n, 4),
               'achieved': round(tf, 2), 'peak': peak, 'unit': 'TFLOP/s', 'frac': round(tf / peak, 4),
               'share_of_device_time': round(ms / total, 4)}
    return table, dom


def config_c(dev, precision, steps, warmup, sync):
    """BASELINE config (c): VolSDF (configs/volsdf.yaml architecture, beta_init 1e-3 so the error-bounded
    loop runs), 2048 rays of the 32x64 camera (f 80, distance 2.7), N_samples 128 + N_importance 128,
    max_upsample_iter 6, render mode"""
    from neurecon_amd.frameworks.volsdf import VolSDF, volume_render
    torch.manual_seed(0)
    surf = dict(use_siren=False, embed_multires=6, radius_init=1.0, geometric_init=True, D=8, W=256, skips=[4],
                precision=precision)
    rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=-1, use_view_dirs=True, D=4, W=256, skips=[],
               precision=precision)
    m = VolSDF(beta_init=1e-3, speed_factor=10.0, W_geo_feat=256, obj_bounding_radius=3.0, surface_cfg=surf,
               radiance_cfg=rad).to(dev).eval()
    ro, rd = camera_for(dev, 32, 64, 80.0, 2.7)
    kw = dict(near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, calc_normal=True, detailed_output=False,
              N_samples=128, N_importance=128, max_upsample_steps=6, use_nerfplusplus=False)

    def step():
        with torch.no_grad():
            return volume_render(ro, rd, m, **kw)
    dt, ks = _census(step, steps, warmup, sync)
    with torch.no_grad():
        _, _, ex = volume_render(ro, rd, m, **dict(kw, detailed_output=True))
    it = ex['iter_usage'].flatten()
    table, dom = _kernel_summary(ks, precision, 265)
    n = ro.shape[1]
    return {'workload': 'VolSDF render, 2048 rays x (128 + 128) error-bounded samples, beta 1e-3, max_upsample_iter 6',
            'value': round(n / dt, 1), 'unit': 'rays/s', 'ms_per_step': round(dt * 1e3, 3), 'steps': steps,
            'iter_usage': {str(int(k)): int((it == k).sum()) for k in it.unique().tolist()},
            'roofline': dom, 'kernels': table}


def config_e(dev, precision, steps, warmup, sync):
    """BASELINE config (e): UNISURF (configs/unisurf.yaml architecture, tau 0.5 -> logit 0, radius of
    interest 4), 4096 rays of the 64x64 camera (f 80, distance 3): 256-step march + 8 secant steps,
    64 interval + 32 free-space samples, render mode"""
    from neurecon_amd.frameworks.unisurf import UNISURF, volume_render
    torch.manual_seed(0)
    surf = dict(use_siren=False, embed_multires=6, radius_init=1.0, geometric_init=True, D=8, W=256, skips=[4],
                precision=precision)
    rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=-1, use_view_dirs=True, D=4, W=256, skips=[],
               precision=precision)
    m = UNISURF(W_geo_feat=256, surface_cfg=surf, radiance_cfg=rad).to(dev).eval()
    ro, rd = camera_for(dev, 64, 64, 80.0, 3.0)
    kw = dict(batched=True, calc_normal=True, detailed_output=False, logit_tau=0.0, radius_of_interest=4.0,
              method='secant', N_query=64, N_freespace=32)

    def step():
        with torch.no_grad():
            return volume_render(ro, rd, m, **kw)
    dt, ks = _census(step, steps, warmup, sync)
    with torch.no_grad():
        _, _, ex = volume_render(ro, rd, m, **dict(kw, detailed_output=True))
    table, dom = _kernel_summary(ks, precision, 265)
    n = ro.shape[1]
    out = {'workload': 'UNISURF render, 4096 rays: 256-step march + 8 secant steps, 64 + 32 samples',
           'value': round(n / dt, 1), 'unit': 'rays/s', 'ms_per_step': round(dt * 1e3, 3), 'steps': steps,
           'roofline': dom, 'kernels': table}
    if 'mask_surface' in ex:
        out['secant_hit_frac'] = round(float(ex['mask_surface'].float().mean()), 4)
    return out


def e_sharded_setup(dev, precision, world):
    """config (e) at N ranks (weak scaling): the 4096 rays of the config-(e) camera repeated N times as
    one batch row of N x 4096 rays; each rank renders its contiguous 4096-ray share
    (neurecon_amd.dist.render_sharded; UNISURF's windowed F.normalize spans the ranks, so the render
    all-reduces the per-window sums of nabla^2 over the process group, RCCL, inside the step)"""
    from neurecon_amd import dist as nd
    from neurecon_amd.frameworks.unisurf import UNISURF, volume_render
    torch.manual_seed(0)
    surf = dict(use_siren=False, embed_multires=6, radius_init=1.0, geometric_init=True, D=8, W=256, skips=[4],
                precision=precision)
    rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=-1, use_view_dirs=True, D=4, W=256, skips=[],
               precision=precision)
    m = UNISURF(W_geo_feat=256, surface_cfg=surf, radiance_cfg=rad).to(dev).eval()
    ro, rd = camera_for(dev, 64, 64, 80.0, 3.0)
    ro, rd = ro.repeat(1, world, 1).contiguous(), rd.repeat(1, world, 1).contiguous()
    kw = dict(batched=True, calc_normal=True, detailed_output=False, logit_tau=0.0, radius_of_interest=4.0,
              method='secant', N_query=64, N_freespace=32)

    def step():
        with torch.no_grad():
            return nd.render_sharded(volume_render, ro, rd, m, gather=False, layout='contiguous', **kw)
    return step, ro.shape[1]


def scaling_legs(args, dev, world, sync, barrier, max_over_ranks):
    """the weak-scaling legs of the default N-GPU line: config (e) with its window all-reduce, and the
    DDP training step (gradient all-reduce in backward); barrier + sync around K steps, max over ranks"""
    legs = {}
    estep, e_rays = e_sharded_setup(dev, args.precision, world)
    edt = max_over_ranks(timed(estep, args.leg_steps, 1, sync, barrier))
    legs['weak_scaling_e'] = {
        'metric': 'rays/sec, config (e): UNISURF 4096 rays per GPU (256-step march + 8 secant steps, 64 + 32 samples)',
        'value': round(e_rays * args.leg_steps / edt, 1), 'unit': 'rays/s', 'n_gpus': world, 'steps': args.leg_steps,
        'warmup': 1, 'ms_per_step': round(edt / args.leg_steps * 1e3, 3), 'scaling': 'weak',
        'rays_per_step': e_rays, 'rays_per_gpu': e_rays // world,
        'parallelism': f'contiguous ray shares x{world}' + (' + per-window nabla^2 all-reduce (RCCL) per render'
                                                            if world > 1 else ''),
        'collective_in_step': world > 1}
    tsteps = 2 * args.leg_steps
    tstep = train_setup(dev, args.precision, args.train_rays, world, args.adam)
    tdt = max_over_ranks(timed(tstep, tsteps, 2, sync, barrier))
    legs['weak_scaling_train'] = {
        'metric': 'training rays/sec, NeuS (configs/neus.yaml: 512 rays per GPU, forward + double backward + Adam)',
        'value': round(args.train_rays * world * tsteps / tdt, 1), 'unit': 'rays/s', 'n_gpus': world,
        'steps': tsteps, 'warmup': 2, 'ms_per_step': round(tdt / tsteps * 1e3, 3), 'scaling': 'weak',
        'rays_per_gpu': args.train_rays,
        'parallelism': f'DDP x{world} (RCCL gradient all-reduce in backward)' if world > 1 else 'single GPU',
        'collective_in_step': world > 1}
    return legs


def fp32_mode(args, dev, sync):
    """config (b) in the exact-fp32 precision mode (v_mfma_f32_16x16x4_f32): rays/s, ms/step, and the
    nabla kernel's fraction of the 157.3 TF/s fp32 MFMA peak (HIP events of the timed steps)"""
    from neurecon_amd import _lib as L
    from neurecon_amd import rend_util
    from neurecon_amd.frameworks.neus import volume_render
    model = make_model(dev, 'fp32')
    c2w, K = camera(dev)
    ro, rd, _ = rend_util.get_rays(c2w, K, 64, 64)
    kw = render_kwargs()

    def step():
        with torch.no_grad():
            return volume_render(ro, rd, model, **kw)
    steps = args.leg_steps
    for _ in range(2):
        step()
    sync()
    L.profile_read()
    L.profile_enable(True, 'sdf_nabla')
    try:
        dt = timed(step, steps, 0, sync, lambda: None)
    finally:
        L.profile_enable(False)
    ks = L.profile_read()
    roof = roofline(ks, 'fp32')
    return {'workload': 'config (b), precision fp32 (exact fp32 MFMA v_mfma_f32_16x16x4_f32; same render and kernels)',
            'value': round(ro.shape[1] * steps / dt, 1), 'unit': 'rays/s', 'ms_per_step': round(dt / steps * 1e3, 3),
            'steps': steps, 'dtype': 'f32',
            'roofline': {k: roof[k] for k in ('kernel', 'achieved', 'peak', 'unit', 'frac', 'avg_launch_ms',
                                               'launches', 'per_launch_type')}}


def config_train(dev, precision, n_rays, steps, warmup, sync, adam='nr', nerfpp=False):
    """NeuS training step, 512 rays (train_setup): wall rays/s, the library's kernel census, and every
    device kernel of one step by name from torch.profiler (the hipBLASLt `Cijk_*` share included)"""
    step = train_setup(dev, precision, n_rays, 1, adam, nerfpp)
    dt, ks = _census(step, steps, warmup, sync)
    table, _ = _kernel_summary(ks, precision, 289)
    wl = ('NeuS Trainer.forward + backward (double backward through the nablas) + Adam, 512 rays x 128 samples' +
          (' + NeRF++ background (configs/neus_nomask_blended.yaml: N_outside 32, no mask loss)' if nerfpp else ''))
    out = {'workload': wl, 'value': round(n_rays / dt, 1), 'unit': 'rays/s', 'ms_per_step': round(dt * 1e3, 3),
           'steps': steps, 'library_kernels': table,
           # the dominant kernel (the layer GEMM, HBM-bound) and nr_wgrad, from the census step's HIP events
           'roofline': train_roofline(ks, dt, 1, ks) if precision == 'f16x3' else None}
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(2):
                step()
            sync()
        groups, by_name = {}, {}
        for ev in prof.key_averages():
            t = getattr(ev, 'self_device_time_total', None)
            if t is None:
                t = getattr(ev, 'self_cuda_time_total', 0)
            if not t:
                continue
            nm = ev.key
            if nm.startswith('Cijk_') or 'hipblaslt' in nm.lower():
                grp = 'hipBLASLt (Cijk_*)'
            elif 'tgemm_kernel' in nm:
                grp = 'nr_train_gemm (tgemm_kernel)'
            elif 'nr::' in nm:
                grp = 'other libnrhip kernels'
            else:
                grp = 'torch / other'
            groups[grp] = groups.get(grp, 0.0) + t / 2e3   # us over 2 steps -> ms per step
            by_name[nm] = by_name.get(nm, 0.0) + t / 2e3
        tot = sum(groups.values()) or 1e-9
        out['device_time_per_step_ms'] = round(tot, 3)
        out['device_time_by_group'] = {k: {'ms': round(v, 3), 'share': round(v / tot, 4)}
                                       for k, v in sorted(groups.items(), key=lambda kv: -kv[1])}
        top = sorted(by_name.items(), key=lambda kv: -kv[1])[:6]
        out['top_kernels'] = [{'name': k[:90], 'ms': round(v, 3), 'share': round(v / tot, 4)} for k, v in top]
        out['device_time_source'] = 'torch.profiler (ROCm kernel trace), 2 steps'
    except Exception as e:  # the profiler is a diagnostic: its absence does not void the timing
        out['device_time_by_group'] = f'unavailable: {type(e).__name__}: {e}'
    return out


def executed_flop(kstats):
    """fp32-equivalent FLOPs the MLP launches executed (units = points actually evaluated)"""
    return sum(units * 2.0 * KERNEL_MAC.get(name, 0) for name, (n, ms, units) in kstats.items())


def mid_frac(kstats, rays, steps):
    """fraction of the 127 mid-points per ray that went through the SDF + radiance nets"""
    if 'sdf_nabla_feat' not in kstats:
        return None
    return round(kstats['sdf_nabla_feat'][2] / (127.0 * rays * steps), 4)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawned_rank(rank, argv, world, port):
    """worker process of `launch`: the torchrun environment for one rank, then the normal bench"""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + list(argv)
    run(parse())


def launch(args):
    """`python bench.py --gpus N` outside torchrun: start N rank processes (spawn: fresh interpreters,
    started before this parent makes any GPU call) that join one process group, the same layout
    torchrun gives (one process per GPU, LOCAL_RANK = GPU index).  A failing rank fails the launch."""
    import torch.multiprocessing as mp
    mp.start_processes(_spawned_rank, args=(sys.argv[1:], args.gpus, _free_port()), nprocs=args.gpus, join=True,
                       start_method='spawn')


def timed(step, steps, warmup, sync, barrier):
    """W untimed steps, then K steps bracketed by barrier + device sync on both sides"""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    return time.perf_counter() - t0


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and (args.gpus or 1) > 1:
        return launch(args)
    run(args)


def run(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = world > 1
    if args.stub_cpu:
        return run_stub(args, world, rank)
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group('nccl', device_id=torch.device('cuda', local))
        world = tdist.get_world_size()
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f'bench: --gpus {args.gpus} but the process group has {world} ranks')
    dev = torch.device('cuda', local)
    sync = torch.cuda.synchronize
    barrier = tdist.barrier if dist else (lambda: None)

    def max_over_ranks(x):
        if not dist:
            return x
        t = torch.tensor([x], device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        return float(t.item())

    from neurecon_amd import rend_util
    from neurecon_amd.frameworks.neus import volume_render
    if args.workload == 'frame_d':
        step, rays_per_step = frame_d_setup(dev, args.precision, args.frame_workspace_gb)  # one frame, all ranks
        n_rays = rays_per_step
    elif args.workload == 'train':
        step = train_setup(dev, args.precision, args.train_rays, world, args.adam, nerfpp=args.train_nerfpp)
        n_rays = args.train_rays * world
    else:
        model = make_model(dev, args.precision)
        c2w, K = camera(dev)
        ro, rd, _ = rend_util.get_rays(c2w, K, 64, 64)
        if args.rays != 4096:
            reps = math.ceil(args.rays / 4096)
            ro = ro.repeat(1, reps, 1)[:, :args.rays].contiguous()
            rd = rd.repeat(1, reps, 1)[:, :args.rays].contiguous()
        kw = render_kwargs()
        kw['max_workspace_gb'] = args.workspace_gb

        def step():
            with torch.no_grad():
                return volume_render(ro, rd, model, **kw)

        def step_full():  # every mid-point through the nets, as the reference (same outputs bit for bit)
            with torch.no_grad():
                return volume_render(ro, rd, model, skip_zero_alpha=False, **kw)
        n_rays = ro.shape[1] * world

    from neurecon_amd import _lib as L

    # HIP events of the timed region bracket only the dominant kernel's launches (the roofline's):
    # every recorded launch costs two event markers on the stream, ~10 us of idle GPU each at the
    # kernel boundary, so events around every library launch slowed the step by ~3 %.  The other
    # library kernels' times (the per-kernel table, the dominant kernel's share, executed FLOPs of the
    # whole step) come from a census of a few more steps with every launch recorded, after the timing.
    dom_prefix = 'train_gemm' if args.workload == 'train' else 'sdf_nabla'

    def profiled(fn):
        """(max-over-ranks time of the timed steps, dominant-kernel stats of the timed steps, every
        library kernel's stats of a census pass scaled to the timed step count)"""
        for _ in range(args.warmup):
            fn()
        sync()
        L.profile_read()           # drop warm-up records
        L.profile_enable(True, dom_prefix)
        try:
            dt = timed(fn, args.steps, 0, sync, barrier)
        finally:
            L.profile_enable(False)
        kdom = L.profile_read()
        n_census = min(3, args.steps)
        L.profile_enable(True)
        try:
            for _ in range(n_census):
                fn()
            sync()
        finally:
            L.profile_enable(False)
        f = args.steps / n_census
        census = {k: (round(n * f), ms * f, u * f) for k, (n, ms, u) in L.profile_read().items()}
        return max_over_ranks(dt), kdom, census

    dt, kstats, census = profiled(step)
    full = None
    if args.workload not in ('frame_d', 'train') and not args.no_full_eval:  # every mid-point evaluated
        full = profiled(step_full)
    frame = None
    if args.workload == 'b' and not args.no_frame:
        # strong scaling: one config-(d) 800x600 frame per step split over all ranks, all_gather timed
        fstep, frame_rays = frame_d_setup(dev, args.precision, args.frame_workspace_gb)
        fdt = max_over_ranks(timed(fstep, args.frame_steps, 1, sync, barrier))
        frame = {'metric': 'rays/sec, config (d): NeuS+NeRF++ full 800x600 frame per step, rays sharded over '
                           'the GPUs (render_sharded + all_gather of the maps inside the timed region)',
                 'value': round(frame_rays * args.frame_steps / fdt, 1), 'unit': 'rays/s', 'n_gpus': world,
                 'steps': args.frame_steps, 'warmup': 1, 'ms_per_step': round(fdt / args.frame_steps * 1e3, 3),
                 'scaling': 'strong', 'rays_per_step': frame_rays, 'rays_per_gpu': frame_rays // world,
                 'parallelism': f'ray-sharded x{world} + all_gather'}
    legs = None
    if args.workload == 'b' and not args.no_scaling_legs:
        legs = scaling_legs(args, dev, world, sync, barrier, max_over_ranks)
    f32 = None
    if args.workload == 'b' and args.precision == 'f16x3' and not args.no_fp32_mode and world == 1:
        f32 = fp32_mode(args, dev, sync)
    cfgs = None
    if args.workload == 'b' and not args.no_configs and world == 1:
        cs, cw = args.config_steps, 1
        cfgs = {'c_volsdf_2048x256': config_c(dev, args.precision, cs, cw, sync),
                'e_unisurf_4096': config_e(dev, args.precision, cs, cw, sync),
                'train_neus_512': config_train(dev, args.precision, args.train_rays, 2 * cs, 2, sync, args.adam),
                'train_neus_nerfpp_512': config_train(dev, args.precision, args.train_rays, 2 * cs, 2, sync, args.adam,
                                                      nerfpp=True)}
    total_rays = n_rays * args.steps
    value = total_rays / dt
    if rank == 0:
        ms = dt / args.steps * 1e3
        roof = roofline(kstats, args.precision, census)
        dtype = 'f32' if args.precision == 'fp32' else args.precision
        if args.workload == 'frame_d':
            out = {'metric': 'rays/sec, config (d): NeuS+NeRF++ full 800x600 frame, rays sharded over the GPUs',
                   'value': round(value, 1), 'unit': 'rays/s', 'n_gpus': world, 'steps': args.steps,
                   'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True,
                   'scaling': 'strong', 'vs_baseline': None, 'dtype': dtype,
                   'data': 'synthetic (config-(d) camera rays, seeded init weights)',
                   'config': {'workload': 'NeuS + NeRF++ (N_outside 32) render of one 800x600 frame per step, '
                                          '64 + 4x16 + 32 samples, maps all-gathered in the step',
                              'rays_per_step': n_rays, 'precision': args.precision,
                              'parallelism': f'ray-sharded x{world} + all_gather'},
                   'roofline': roof}
        elif args.workload == 'train':
            roof = train_roofline(kstats, dt, args.steps, census)
            out = {'metric': ('training rays/sec, NeuS + NeRF++ (configs/neus_nomask_blended.yaml: 512 rays per GPU, '
                              'fwd+bwd+Adam)' if args.train_nerfpp else
                              'training rays/sec, NeuS (configs/neus.yaml: 512 rays per GPU, fwd+bwd+Adam)'),
                   'value': round(value, 1), 'unit': 'rays/s', 'n_gpus': world, 'steps': args.steps,
                   'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True,
                   'scaling': 'weak', 'vs_baseline': None, 'dtype': (dtype + ' layer GEMMs (nr_train_gemm) and weight gradients (nr_wgrad); radiance forward fp32 MFMA'
                             if args.precision == 'f16x3' else 'f32'),
                   'data': 'synthetic (random 64x64 targets, config-(b) camera, seeded geometric-init weights)',
                   'config': {'workload': 'NeuS Trainer.forward + backward (double backward through the nablas) + '
                                          'Adam step', 'rays_per_gpu': args.train_rays, 'samples_per_ray': 128,
                              'parallelism': f'DDP x{world}' if world > 1 else 'single GPU',
                              'optimizer': 'neurecon_amd.optim.Adam (nr_adam_step)' if args.adam == 'nr' else
                              f'torch.optim.Adam ({args.adam})'},
                   'roofline': roof}
        else:
            out = {
                'metric': 'rays/sec (4096 rays x 128 samples, 8-layer x256 SDF MLP)',
                'value': round(value, 1), 'unit': 'rays/s', 'n_gpus': world, 'steps': args.steps,
                'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
                'vs_baseline': None, 'dtype': dtype,
                'data': 'synthetic (config-(b) camera rays, seeded geometric-init weights)',
                'config': {'workload': 'NeuS render, configs/neus.yaml architecture, 64x64 camera = 4096 rays x '
                                       '(64 coarse + 4x16 upsampled) samples, render mode',
                           'rays_per_gpu': n_rays // world, 'samples_per_ray': 128, 'precision': args.precision,
                           'parallelism': f'ray-sharded x{world}'},
                'roofline': roof,
                # executed MLP FLOPs (fp32-equivalent) per second over the whole step
                'step_tflops': round(executed_flop(census) / args.steps / (dt / args.steps) / 1e12, 2),
                'mid_points_evaluated_frac': mid_frac(kstats, n_rays // world, args.steps),
            }
            if full is not None:
                dtf, kf, kfc = full
                out['full_evaluation'] = {
                    'note': 'same rays, same outputs bit for bit (tests/test_gpu_parity.py); every mid-point through '
                            'the SDF + radiance nets as the reference does, including the ones whose alpha is exactly 0',
                    'value': round(total_rays / dtf, 1), 'ms_per_step': round(dtf / args.steps * 1e3, 3),
                    'step_tflops': round(executed_flop(kfc) / dtf / 1e12, 2),
                    'roofline': roofline(kf, args.precision, kfc)}
            if frame is not None:
                out['strong_scaling_frame_d'] = frame
            if legs is not None:
                out.update(legs)
            if f32 is not None:
                out['fp32_mode'] = f32
            if cfgs is not None:
                out['configs'] = cfgs
            out['config']['zero_alpha_skip'] = ('mid-points whose alpha is exactly 0 (no SDF decrease between the '
                                                'two samples, neus.py:28-35) get weight 0 and skip the nets; '
                                                'rgb/depth/mask/normals bit-identical to full evaluation')
            if not args.no_cpu_baseline and world == 1:
                out['cpu_baseline'] = cpu_baseline(args.cpu_rays)
                eg = eager_gpu_baseline(dev, n_rays)
                eg['speedup'] = round(value / eg['value'], 2)
                out['cpu_baseline']['eager_gpu_reference'] = eg
        out['config']['build_id'] = L.build_id()  # source hash compiled into libnrhip.so (neurecon_amd/build.py)
        out['config']['workspace_gb'] = args.workspace_gb if args.workspace_gb is not None else 'library default (4 GiB)'
        if args.workload == 'b' and not args.no_frame:
            out['strong_scaling_frame_d']['workspace_gb'] = args.frame_workspace_gb
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


def run_stub(args, world, rank):
    """CPU rehearsal of the launcher and the timing protocol (tests/test_bench_launch.py): gloo process
    group, a small matmul as the step, the same barrier / max-over-ranks / one-line JSON contract."""
    import torch.distributed as tdist
    dist = world > 1
    if dist:
        tdist.init_process_group('gloo')
        world = tdist.get_world_size()
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f'bench: --gpus {args.gpus} but the process group has {world} ranks')
    a = torch.randn(64, 64)
    barrier = tdist.barrier if dist else (lambda: None)

    def max_over_ranks(x):
        if not dist:
            return x
        t = torch.tensor([x])
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        return float(t.item())
    dt = max_over_ranks(timed(lambda: a @ a, args.steps, args.warmup, lambda: None, barrier))
    ranks = [rank]
    if dist:
        got = [None] * world
        tdist.all_gather_object(got, rank)
        ranks = got
    out = {'metric': 'stub', 'value': args.steps * world / dt, 'unit': 'steps/s', 'n_gpus': world,
           'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3,
           'ranks': ranks, 'pid': os.getpid()}
    if not args.no_scaling_legs:
        out.update(stub_legs(args, world, barrier, max_over_ranks))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


def stub_legs(args, world, barrier, max_over_ranks):
    """CPU rehearsal of scaling_legs(): the same sharding driver and collectives with stand-in compute.
    weak_scaling_e: render_sharded over a window-sharded stand-in render whose step all-reduces its
    per-window partial sums (as UNISURF's window_reduce does); weak_scaling_train: a DDP-wrapped linear
    model's forward + backward (gradient all-reduce) + Adam."""
    import torch.distributed as tdist
    from neurecon_amd import dist as nd
    n_per = 64
    ro = torch.randn(1, n_per * world, 3)
    rd = torch.randn(1, n_per * world, 3)
    seen = {}

    def fake_unisurf(o, d, model, shard=None, **kw):
        ss = (o * d).sum(dim=(0, 1)).double()          # this share's partial window sums
        if shard is not None and tdist.is_initialized():
            tdist.all_reduce(ss, op=tdist.ReduceOp.SUM)
        seen['shard'] = shard is not None
        rgb = o * ss.float().norm()
        return rgb, rgb[..., 0], {'rgb': rgb}
    fake_unisurf.window_sharded = True
    estep = lambda: nd.render_sharded(fake_unisurf, ro, rd, None, gather=False, layout='contiguous', batched=True)
    edt = max_over_ranks(timed(estep, args.leg_steps, 1, lambda: None, barrier))
    net = torch.nn.Linear(16, 16)
    model = torch.nn.parallel.DistributedDataParallel(net) if world > 1 else net
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    x = torch.randn(32, 16)

    def tstep():
        loss = model(x).square().mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    tdt = max_over_ranks(timed(tstep, 2 * args.leg_steps, 2, lambda: None, barrier))
    return {'weak_scaling_e': {'value': n_per * world * args.leg_steps / edt, 'unit': 'rays/s', 'n_gpus': world,
                               'scaling': 'weak', 'rays_per_gpu': n_per, 'steps': args.leg_steps,
                               'collective_in_step': bool(seen.get('shard'))},
            'weak_scaling_train': {'value': 32 * world * 2 * args.leg_steps / tdt, 'unit': 'rays/s', 'n_gpus': world,
                                   'scaling': 'weak', 'steps': 2 * args.leg_steps,
                                   'collective_in_step': world > 1}}


if __name__ == '__main__':
    main()
