"""Measured max |err| of the quick decode (quick.decode_language_features) against a
float64 restatement of eval_lerf.py:214-218, on (a) the unit tests' random sparse maps
and (b) a quick-rendered 1 Mpix map (1M Gaussians, 1280x800, 3 levels x top-4), the
verdict's requested figure.  Usage: python tools/dec_err.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import quick  # noqa: E402


def ref_decode(wmap, cb, eps=1e-10):
    L, K, Df = cb.shape
    D, H, W = wmap.shape
    F = np.einsum("ldk,lkn->ldn", np.transpose(cb, (0, 2, 1)).astype(np.float64),
                  wmap.reshape(L, K, H * W).astype(np.float64))
    return F / (np.linalg.norm(F, axis=1, keepdims=True) + eps)


def err_chunked(wm_gpu, cb_np, rows=40):
    cb = torch.from_numpy(cb_np).to("cuda")
    got = quick.decode_language_features(wm_gpu, cb)
    L, Df = cb_np.shape[0], cb_np.shape[2]
    H = wm_gpu.shape[1]
    worst, worst_px = 0.0, None
    for y0 in range(0, H, rows):
        w = wm_gpu[:, y0:y0 + rows].cpu().numpy()
        ref = ref_decode(w, cb_np).reshape(L, Df, w.shape[1], w.shape[2])
        e = np.abs(got[:, :, y0:y0 + rows].cpu().numpy() - ref)
        m = float(e.max())
        if m > worst:
            worst = m
            idx = np.unravel_index(int(e.argmax()), e.shape)
            worst_px = dict(level=int(idx[0]), y=int(idx[2] + y0), x=int(idx[3]),
                            wsum=float(w[idx[0] * 64:(idx[0] + 1) * 64, idx[2], idx[3]].sum()),
                            wmax=float(w[idx[0] * 64:(idx[0] + 1) * 64, idx[2], idx[3]].max()))
    return worst, worst_px


def main():
    out = {}
    g = np.random.default_rng(45)
    wmap = (g.random((192, 64, 128)) * (g.random((192, 64, 128)) < 0.15)).astype(np.float32)
    cb = g.standard_normal((3, 64, 512)).astype(np.float32)
    out["random_sparse_64x128"] = err_chunked(torch.from_numpy(wmap).cuda(), cb)
    # small-weight pixels: the same maps scaled by 1e-3 .. 1e-6 (a nearly transparent pixel)
    for s in (1e-3, 1e-6):
        out[f"random_sparse_scaled_{s:g}"] = err_chunked(torch.from_numpy(wmap * s).cuda(), cb)
    from diff_gaussian_rasterization import GaussianRasterizer
    import bench
    from langsplatv2_amd.scenes import make_camera, make_gaussians
    cam = make_camera(1280, 800)
    gg = make_gaussians(1_000_000, cam, seed=0, sh_degree=3, quick_k=4)
    t = {k: v.cuda() for k, v in gg.items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(bench.settings(cam, torch.device("cuda"), 3, False, quick=True))
    with torch.no_grad():
        lm = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"], shs=t["shs"],
               language_feature_weights_quick=t["language_feature_weights_quick"],
               language_feature_indices=t["language_feature_indices"], scales=t["scales"],
               rotations=t["rotations"])[1]
    cb2 = np.random.default_rng(3).standard_normal((3, 64, 512)).astype(np.float32)
    out["rendered_1mpix_1280x800"] = err_chunked(lm, cb2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
