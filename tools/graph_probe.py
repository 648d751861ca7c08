"""Capture one config-(b) render step (volume_render, no host syncs inside) in a HIP graph and
replay it: checks the replayed maps are bit-identical to the eager call and times eager vs replay."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from neurecon_amd import rend_util
    from neurecon_amd.frameworks.neus import volume_render
    dev = torch.device('cuda', 0)
    model = bench.make_model(dev, 'f16x3')
    c2w, K = bench.camera(dev)
    ro, rd, _ = rend_util.get_rays(c2w, K, 64, 64)
    kw = bench.render_kwargs()

    def step():
        with torch.no_grad():
            return volume_render(ro, rd, model, **kw)

    for _ in range(3):
        ref = step()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step()
    g.replay()
    torch.cuda.synchronize()
    ok = all(torch.equal(a, b) for a, b in [(out[0], ref[0]), (out[1], ref[1]),
                                             (out[2]['mask_volume'], ref[2]['mask_volume']),
                                             (out[2]['normals_volume'], ref[2]['normals_volume'])])
    print('graph replay bit-identical:', ok)
    for name, fn in [('eager', step), ('graph', g.replay), ('eager', step), ('graph', g.replay)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 30
        print(f'{name}: {dt * 1e3:.3f} ms/step, {4096 / dt:.0f} rays/s')
    if not ok:
        sys.exit(1)


if __name__ == '__main__':
    main()
