"""Feature-mode language loss at one training view: the fused HIP head
(langsplatv2_amd.lang_loss.language_cos_loss) vs the reference's PyTorch
formulation on the same GPU (compute_layer_feature_map + gathered ground
truth + cos_loss, train.py:151-164), forward + backward, synthetic seeded
inputs: K = 64 codes, Df = 512, S segments in coherent regions.

  python tools/bench_lang_loss.py [--H 1080 --W 1920 --S 200 --iters 10]
Prints one JSON line per variant (ms per loss fwd+bwd, algorithmic bytes).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd.lang_loss import language_cos_loss  # noqa: E402


def reference(wm, cb, seg, feat):
    K, H, W = wm.shape
    f = (cb[0].T @ wm.reshape(K, -1)).reshape(-1, H, W)
    s = seg.reshape(-1).long()
    mask = (s != -1).reshape(1, H, W)
    gt = feat[s].reshape(H, W, -1).permute(2, 0, 1)
    return 1 - F.cosine_similarity(f * mask, gt * mask, dim=0).mean()


def timed(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--S", type=int, default=200)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    K, Df, H, W, S = 64, 512, a.H, a.W, a.S
    wm = torch.softmax(2 * torch.randn(K, H, W, device=dev, generator=g), 0).requires_grad_(True)
    cb = torch.randn(1, K, Df, device=dev, generator=g).requires_grad_(True)
    feat = torch.randn(S, Df, device=dev, generator=g)
    yy, xx = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing="ij")
    seg = (((yy // 60) * 37 + (xx // 80)) % (S + 1) - 1).to(torch.int32)

    def fused():
        wm.grad = cb.grad = None
        language_cos_loss(wm, cb, seg, feat).backward()

    def ref():
        wm.grad = cb.grad = None
        reference(wm, cb, seg, feat).backward()

    P = H * W
    # fused: weight map read twice (fwd, bwd), gradient map written once, seg read twice
    alg = 3 * K * P * 4 + 2 * P * 4
    ms = timed(fused, a.iters)
    print(json.dumps({"variant": "fused_hip", "H": H, "W": W, "S": S, "ms_fwd_bwd": round(ms, 4),
                      "algorithmic_bytes": alg, "GBps": round(alg / ms / 1e6, 1)}), flush=True)
    if not a.no_reference:
        torch.cuda.empty_cache()
        ms_r = timed(ref, max(2, a.iters // 2))
        with torch.no_grad():
            l_ref = reference(wm, cb, seg, feat).item()
            l_fused = language_cos_loss(wm, cb, seg, feat).item()
        print(json.dumps({"variant": "torch_reference_ops", "ms_fwd_bwd": round(ms_r, 4),
                          "speedup_fused": round(ms_r / ms, 2), "loss_ref": l_ref, "loss_fused": l_fused}),
              flush=True)


if __name__ == "__main__":
    main()
