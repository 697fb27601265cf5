"""Per-phase cycle census of k_render_bwd_mf (diagnostic variant: the stamps
live in tools/variants/bwd_stamps.patch, out of the product source --
`python tools/variant.py stamps --patch tools/variants/bwd_stamps.patch`, then
run this script on langsplatv2_amd/_build/var_stamps/liblsr.so).
Runs cfg3 fwd+bwd a few times and prints, per phase, the s_memtime cycles summed
over waves, per group and per chunk.  Usage: python tools/bwd_stamps.py [LIB]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

lib = _lib.load(sys.argv[1] if len(sys.argv) > 1 else "langsplatv2_amd/_build/var_stamps/liblsr.so")
_lib._lib = lib
lib.lsr_dbg_bwd_stamps.argtypes = [ctypes.c_void_p]
cfg = CONFIGS[3]
dev = torch.device("cuda:0")
cam = make_camera(cfg["W"], cfg["H"])
g0 = make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=16)
keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
g = {k: g0[k].to(dev).requires_grad_(True) for k in keys}
g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
r = GaussianRasterizer(bench.settings(cam, dev, 3, True))
dc = torch.randn(3, cfg["H"], cfg["W"], device=dev)
dl = torch.randn(16, cfg["H"], cfg["W"], device=dev)
buf = (ctypes.c_ulonglong * 16)()


def step():
    c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                language_feature_precomp=g["language_feature_precomp"], scales=g["scales"], rotations=g["rotations"])
    torch.autograd.grad([c, l], [g[k] for k in keys] + [g["means2D"]], [dc, dl])


for _ in range(3):
    step()
torch.cuda.synchronize()
lib.lsr_dbg_bwd_stamps(buf)
n = 5
for _ in range(n):
    step()
torch.cuda.synchronize()
lib.lsr_dbg_bwd_stamps(buf)
v = [buf[i] / n for i in range(10)]
names = ["prologue", "stage(chunk)", "feat+phase1", "dot mfma", "phase2", "phase3", "rows+atomics", "carry",
         "chunks", "groups"]
groups, chunks = v[9], v[8]
tot = sum(v[:8])
print(f"per launch: groups {groups:.0f}, chunks {chunks:.0f}, wave-cycles {tot:.3e}")
for i in range(8):
    per = v[i] / (groups if i in (2, 3, 4, 5, 6) else chunks)
    print(f"  {names[i]:14s} {v[i]:.3e} wave-cyc  {100 * v[i] / tot:5.1f} %  {per:8.1f} per {'group' if i in (2, 3, 4, 5, 6) else 'chunk'}")
