"""Minimal workload for PMC collection: a few cfg3 fwd+bwd steps (LSR_DET=1: with the
deterministic backward), or (LSR_QUICK=1)
quick-path forwards at 1280x800 with 1M Gaussians (K=12 sparse codes, Dq=192), each followed
by the 3 x 64 x 512 codebook decode + L2 norm."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
steps = int(os.environ.get("LSR_STEPS", "3"))
if os.environ.get("LSR_QUICK", "0") == "1":
    W, H = 1280, 800
    cam = make_camera(W, H)
    g0 = make_gaussians(1_000_000, cam, seed=0, sh_degree=3, quick_k=4)
    t = {k: v.to(dev) for k, v in g0.items() if isinstance(v, torch.Tensor)}
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"], bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev), projmatrix=cam["projmatrix"].to(dev), sh_degree=3,
        campos=cam["campos"].to(dev), prefiltered=False, debug=False, include_feature=False, quick_render=True,
        language_feature_layout=os.environ.get("LSR_QUICK_LAYOUT"))   # unset: the default (pixel-major)
    r = GaussianRasterizer(rs)
    z = torch.zeros_like(t["means3D"])
    from langsplatv2_amd import quick
    cb = torch.randn(3, 64, 512, generator=torch.Generator().manual_seed(3)).to(dev)
    with torch.no_grad():
        for _ in range(steps):
            lm = r(means3D=t["means3D"], means2D=z, opacities=t["opacities"], shs=t["shs"],
                   language_feature_weights_quick=t["language_feature_weights_quick"],
                   language_feature_indices=t["language_feature_indices"], scales=t["scales"],
                   rotations=t["rotations"])[1]
            quick.decode_language_features(lm, cb)   # eval_lerf.py:214-218
    torch.cuda.synchronize()
    print("ok")
    sys.exit(0)

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
cam = make_camera(cfg["W"], cfg["H"])
D = int(os.environ.get("LSR_D", cfg["lang_dim"]))
g0 = make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=D)
keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
g = {k: g0[k].to(dev).requires_grad_(True) for k in keys}
g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
r = GaussianRasterizer(bench.settings(cam, dev, 3, True))
dc = torch.randn(3, cfg["H"], cfg["W"], device=dev)
dl = torch.randn(D, cfg["H"], cfg["W"], device=dev)
if os.environ.get("LSR_DET", "0") == "1":   # the deterministic backward (LSR_OPT_DETERMINISTIC)
    from langsplatv2_amd import _lib
    _lib.set_deterministic(True)
for _ in range(steps):
    with torch.set_grad_enabled(cfg["backward"]):   # cfg5 is forward-only
        c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                    language_feature_precomp=g["language_feature_precomp"], scales=g["scales"],
                    rotations=g["rotations"])
    if cfg["backward"]:
        torch.autograd.backward([c, l], [dc, dl])
torch.cuda.synchronize()
print("ok")
