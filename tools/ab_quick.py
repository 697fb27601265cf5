"""A/B of the quick decode (lsr_quick_decode_run) and the quick render between
liblsr variants in ONE process, interleaved rounds, at bench.py's quick_1mpix
workload (1M Gaussians, 1280x800, 3 levels x top-4 -> 192 channels, 3 x 64 x 512
codebooks).  Usage: python tools/ab_quick.py name=path.so ...; a name ending in
":nopack" runs that library with rasterizer.QUICK_PACKED_CODES off (the
indices passed as they are instead of the cached packed rows)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib, quick, rasterizer  # noqa: E402
from langsplatv2_amd.scenes import make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

variants = [a.split("=", 1) for a in sys.argv[1:]]
libs = {name: _lib.load(path) for name, path in variants}
dev = torch.device("cuda:0")
W, H, N = 1280, 800, 1_000_000
cam = make_camera(W, H)
g = make_gaussians(N, cam, seed=0, sh_degree=3, quick_k=4)
t = {k: v.to(dev) for k, v in g.items() if isinstance(v, torch.Tensor)}
# LSR_AB_LAYOUT=hwc: the pixel-major quick map (language_feature_layout)
r = GaussianRasterizer(bench.settings(cam, dev, 3, False, quick=True, quick_layout=os.environ.get("LSR_AB_LAYOUT")))
z = torch.zeros_like(t["means3D"])
cb = torch.randn(3, 64, 512, device=dev)


def render():
    with torch.no_grad():
        return r(means3D=t["means3D"], means2D=z, opacities=t["opacities"], shs=t["shs"],
                 language_feature_weights_quick=t["language_feature_weights_quick"],
                 language_feature_indices=t["language_feature_indices"], scales=t["scales"],
                 rotations=t["rotations"])[1]


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


res = {name: {"render": [], "decode": [], "both": []} for name, _ in variants}
for rnd in range(6):
    for name, _ in variants:
        _lib._lib = libs[name]
        rasterizer.QUICK_PACKED_CODES = not name.endswith(":nopack")
        rasterizer._PACKED.clear()
        quick._PLANS.clear()
        wm = render()
        quick.decode_language_features(wm, cb)   # plan + warm
        torch.cuda.synchronize()
        if rnd == 0:
            continue
        res[name]["render"].append(timed(render, 10))
        res[name]["decode"].append(timed(lambda: quick.decode_language_features(wm, cb), 10))
        res[name]["both"].append(timed(lambda: quick.decode_language_features(render(), cb), 10))
for name, _ in variants:
    m = {k: statistics.median(v) for k, v in res[name].items()}
    print(name, " ".join(f"{k}_ms={v:.4f}" for k, v in m.items()), f"fps={1e3 / m['both']:.1f}")
