import sys, os, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo/tests/golden')
import weightgen as wg
from helpers import neus_model, to_gpu
g = dict(np.load('/root/repo/tests/golden/sdf_net.npz'))
m = neus_model(wg.neus_state(seed=int(g['seed'])), precision='f16x3')
pts = to_gpu(g['pts'])
with torch.no_grad():
    s, h = m.implicit_surface.forward(pts, return_h=True)
h = h[:64].cpu().numpy(); ref = g['h_nograd']
bad = ~(np.abs(h - ref) <= 1e-4 * np.abs(ref) + 1e-5)
print('bad points', np.where(bad.any(1))[0])
print('bad feats', np.where(bad.any(0))[0])
print(h[0, :8], ref[0, :8])
