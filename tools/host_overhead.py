"""Diagnose host-side overhead of one fwd+bwd step (bench cfg3 workload)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402
from langsplatv2_amd.scenes import make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
cam = make_camera(1920, 1080)
g0 = make_gaussians(1_000_000, cam, seed=0, sh_degree=3, lang_dim=16)
keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
g = {k: g0[k].to(dev).requires_grad_(True) for k in keys}
g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
rs = bench.settings(cam, dev, 3, True)
r = GaussianRasterizer(rs)
dc = torch.randn(3, 1080, 1920, device=dev)
dl = torch.randn(16, 1080, 1920, device=dev)
params = list(g.values())


def step(tim):
    t0 = time.perf_counter()
    for p in params:
        p.grad = None
    c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                language_feature_precomp=g["language_feature_precomp"], scales=g["scales"], rotations=g["rotations"])
    t1 = time.perf_counter()
    torch.autograd.backward([c, l], [dc, dl])
    t2 = time.perf_counter()
    tim.append((t1 - t0, t2 - t1))


for prof in (False, True):
    _lib.profile_enable(prof)
    tim = []
    for _ in range(5):
        step(tim)
    torch.cuda.synchronize()
    tim = []
    t0 = time.perf_counter()
    for _ in range(30):
        step(tim)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 30
    f = sorted(x[0] for x in tim)
    b = sorted(x[1] for x in tim)
    print(f"profile={prof}: {el*1e3:.3f} ms/step; host fwd call median {f[15]*1e3:.3f} ms (max {f[-1]*1e3:.3f}), "
          f"host bwd call median {b[15]*1e3:.3f} ms (max {b[-1]*1e3:.3f})")
    _lib.profile_reset()
# host-only cost of the python/ctypes path: tiny problem
g1 = make_gaussians(100, cam, seed=0, sh_degree=3, lang_dim=16)
h = {k: g1[k].to(dev).requires_grad_(True) for k in keys}
h["means2D"] = torch.zeros_like(h["means3D"], requires_grad=True)
cam_s = make_camera(64, 64)
r2 = GaussianRasterizer(bench.settings(cam_s, dev, 3, True))
dc2 = torch.randn(3, 64, 64, device=dev)
dl2 = torch.randn(16, 64, 64, device=dev)
for i in range(60):
    if i == 10:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    c, l, _ = r2(means3D=h["means3D"], means2D=h["means2D"], opacities=h["opacities"], shs=h["shs"],
                 language_feature_precomp=h["language_feature_precomp"], scales=h["scales"], rotations=h["rotations"])
    torch.autograd.backward([c, l], [dc2, dl2])
torch.cuda.synchronize()
print(f"tiny problem fwd+bwd: {(time.perf_counter() - t0) / 50 * 1e3:.3f} ms/step (host-bound floor)")
print("nproc", os.cpu_count(), "load", os.getloadavg())
