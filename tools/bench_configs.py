"""Timings for every BASELINE.json configuration that fits one GPU (cfg 1, 2,
3, 5; cfg 4 needs the LERF dataset).  Synthetic seeded inputs.
One JSON line per config: forward ms (and fwd+bwd ms where the config trains),
FPS, per-stage kernel times.

  python tools/bench_configs.py [--iters 10] [--configs 1,2,3,5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    _lib.profile_enable(False)
    st = {k: round(v / c, 4) for k, (v, c) in _lib.profile_query().items() if c}
    return ms, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--configs", default="1,2,3,5")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for cid in [int(x) for x in args.configs.split(",")]:
        cfg = CONFIGS[cid]
        N, W, H, D, deg = cfg["N"], cfg["W"], cfg["H"], cfg["lang_dim"], cfg["sh_degree"]
        cam = make_camera(W, H)
        g0 = make_gaussians(N, cam, seed=0, sh_degree=deg, lang_dim=D)
        keys = [k for k in ("means3D", "shs", "colors_precomp", "opacities", "scales", "rotations",
                            "language_feature_precomp") if k in g0]
        g = {k: g0[k].to(dev).requires_grad_(cfg["backward"]) for k in keys}
        g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=cfg["backward"])
        rs = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
            bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
            projmatrix=cam["projmatrix"].to(dev), sh_degree=g0.get("sh_degree", 0), campos=cam["campos"].to(dev),
            prefiltered=False, debug=False, include_feature=D > 0, quick_render=False)
        r = GaussianRasterizer(rs)
        kw = {k: g[k] for k in keys if k not in ("means3D", "opacities")}
        if "shs" in kw:
            pass
        out = {"config": cid, "workload": f"{N} Gaussians, {W}x{H}, " + (f"SH{deg}" if deg is not None else "RGB")
               + f" + {D} language channels", "data": "synthetic (seeded; SURVEY.md §8d generator)"}

        def fwd():
            with torch.no_grad():
                return r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], **kw)

        ms, st = timed(fwd, args.iters)
        out.update(fwd_ms=round(ms, 4), fwd_fps=round(1e3 / ms, 1), fwd_stages_ms=st)
        if cfg["backward"]:
            gc = torch.randn(3, H, W, device=dev)
            gl = torch.randn(D, H, W, device=dev) if D else None

            def step():
                for v in g.values():
                    v.grad = None
                c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], **kw)
                torch.autograd.backward([c, l] if D else [c], [gc, gl] if D else [gc])

            ms2, st2 = timed(step, args.iters)
            out.update(fwd_bwd_ms=round(ms2, 4), fwd_bwd_fps=round(1e3 / ms2, 1), fwd_bwd_stages_ms=st2)
        print(json.dumps(out), flush=True)
        del g, g0, r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
