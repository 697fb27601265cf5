"""Quick (sparse-coefficient) language rendering + codebook decode on one MI355X.

The reference's headline "450+ FPS" (README.md:1) is for this evaluation path:
render with quick_render=True (per-Gaussian top-4 codes of 3 levels -> a
192-channel weight map), then decode against 3 codebooks of 64 x 512 and
L2-normalise (eval_lerf.py:210-220).  Synthetic: 1M Gaussians (SURVEY §8d
generator), random codebooks.  Prints one JSON line per resolution with the
render, decode and total times, and the same decode done the reference's way
(torch.einsum + norm on the GPU) for comparison.

  python tools/bench_quick.py [--iters 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib, quick  # noqa: E402
from langsplatv2_amd.scenes import make_camera, make_gaussians  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cb = torch.randn(3, 64, 512, device=dev)
    for (W, H) in ((1280, 800), (1920, 1080)):
        cam = make_camera(W, H)
        g = make_gaussians(args.gaussians, cam, seed=0, sh_degree=3, quick_k=4)
        t = {k: v.to(dev) for k, v in g.items() if isinstance(v, torch.Tensor)}
        rs = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
            bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
            projmatrix=cam["projmatrix"].to(dev), sh_degree=3, campos=cam["campos"].to(dev), prefiltered=False,
            debug=False, include_feature=False, quick_render=True)
        r = GaussianRasterizer(rs)
        z = torch.zeros_like(t["means3D"])

        def render():
            with torch.no_grad():
                return r(means3D=t["means3D"], means2D=z, opacities=t["opacities"], shs=t["shs"],
                         language_feature_weights_quick=t["language_feature_weights_quick"],
                         language_feature_indices=t["language_feature_indices"], scales=t["scales"],
                         rotations=t["rotations"])

        _, wmap, _ = render()
        _lib.profile_reset()
        _lib.profile_enable(True)
        ms_render = timeit(render, args.iters)
        _lib.profile_enable(False)
        stages = {k: round(ms / calls, 4) for k, (ms, calls) in _lib.profile_query().items() if calls}
        ms_decode = timeit(lambda: quick.decode_language_features(wmap, cb), args.iters)

        def ref_decode():
            w = wmap.view(3, 64, H * W)
            f = torch.einsum("ldk,lkn->ldn", cb.permute(0, 2, 1), w).view(3, 512, H, W)
            return f / (f.norm(dim=1, keepdim=True) + 1e-10)

        ms_ref = timeit(ref_decode, max(3, args.iters // 4))
        out_bytes = 3 * 512 * H * W * 4
        flops = 2 * 3 * 512 * 64 * H * W * 1.125   # decode + Gram-norm products
        print(json.dumps({
            "workload": f"quick render + 3x64x512 codebook decode, {args.gaussians} Gaussians, {W}x{H}",
            "render_ms": round(ms_render, 4), "decode_ms": round(ms_decode, 4),
            "total_ms": round(ms_render + ms_decode, 4), "fps": round(1e3 / (ms_render + ms_decode), 1),
            "render_only_fps": round(1e3 / ms_render, 1),
            "decode_TFLOPs": round(flops / (ms_decode * 1e-3) / 1e12, 1), "decode_write_GBps":
            round(out_bytes / (ms_decode * 1e-3) / 1e9, 1),
            "torch_einsum_norm_decode_ms": round(ms_ref, 4), "render_stages_ms": stages}), flush=True)
        del wmap


if __name__ == "__main__":
    main()
