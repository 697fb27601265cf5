"""Census of the tile instances the binning emits at cfg3 (analysis only, torch on the GPU).

For every (Gaussian, tile) instance of the reference's binning (the 3-sigma
radius rect, A.2) evaluates the render's conservative cut-ellipse test at
16x16-tile granularity (the cut extents' box, then the exact ellipse-vs-
rectangle test of lsr_device.h: rect_overlap_exact) and counts the instances
that can contribute to some pixel of their tile.  Usage: python tools/bin_cull_census.py
(LSR_CFG=3 default)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import layout, rasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
dev = torch.device("cuda:0")
W, H, N, D = cfg["W"], cfg["H"], cfg["N"], cfg["lang_dim"]
cam = make_camera(W, H)
g0 = make_gaussians(N, cam, seed=0, sh_degree=3, lang_dim=D)
g = {k: v.to(dev) for k, v in g0.items() if isinstance(v, torch.Tensor)}
rs = bench.settings(cam, dev, 3, D > 0)
e = torch.empty(0, device=dev)
with torch.no_grad():
    _, _, radii, M, bufs, _, _, _ = rasterizer._run_forward(
        g["means3D"], g["shs"], e, g.get("language_feature_precomp", e), e, e, g["opacities"], g["scales"],
        g["rotations"], e, rs)
dec = layout.decode(bufs, N, W, H, M)
gx = (W + 15) // 16
ts = dec["tile_start"].long()
cnt = ts[1:] - ts[:-1]
tile = torch.repeat_interleave(torch.arange(cnt.numel(), device=dev), cnt)
pl = dec["point_list"].long()
xy, co, cut = dec["xy"][pl], dec["conic_opacity"][pl], dec["cut"][pl]
bx = ((tile % gx) * 16).float()
by = ((tile // gx) * 16).float()
ca, cb, cc = co[:, 0], co[:, 1], co[:, 2]
x, y = xy[:, 0], xy[:, 1]
thr = (-2.0 * cut) * 1.001 + 1e-3
u1, v1 = x - bx, y - by
u0, v0 = u1 - 15.0, v1 - 15.0
inside = (u0 <= 0) & (u1 >= 0) & (v0 <= 0) & (v1 >= 0)


def q(u, v):
    return ca * u * u + 2.0 * cb * u * v + cc * v * v


va = torch.clamp(-cb * u0 / cc, min=v0, max=v1)
vb = torch.clamp(-cb * u1 / cc, min=v0, max=v1)
ua = torch.clamp(-cb * v0 / ca, min=u0, max=u1)
ub = torch.clamp(-cb * v1 / ca, min=u0, max=u1)
qmin = torch.minimum(torch.minimum(q(u0, va), q(u1, vb)), torch.minimum(q(ua, v0), q(ub, v1)))
degenerate = ~(ca > 0) | ~(cc > 0) | ~(cut > -3.0e38)
keep = degenerate | inside | ~(qmin > thr)
print({"M": M, "visible": int((radii > 0).sum()), "kept_exact_tile": int(keep.sum()),
       "frac": round(float(keep.float().mean()), 4)})
