"""Minimal workload for PMC collection: a few cfg3 fwd+bwd steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
dev = torch.device("cuda:0")
cam = make_camera(cfg["W"], cfg["H"])
D = int(os.environ.get("LSR_D", cfg["lang_dim"]))
g0 = make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=D)
keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
g = {k: g0[k].to(dev).requires_grad_(True) for k in keys}
g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
r = GaussianRasterizer(bench.settings(cam, dev, 3, True))
dc = torch.randn(3, cfg["H"], cfg["W"], device=dev)
dl = torch.randn(D, cfg["H"], cfg["W"], device=dev)
for _ in range(int(os.environ.get("LSR_STEPS", "3"))):
    c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                language_feature_precomp=g["language_feature_precomp"], scales=g["scales"], rotations=g["rotations"])
    torch.autograd.backward([c, l], [dc, dl])
torch.cuda.synchronize()
print("ok")
