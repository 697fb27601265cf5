"""Generate tests/golden/ref_lang_loss.npz: the feature-mode training loss and
its autograd gradients computed with the REFERENCE's own cos_loss
(utils/loss_utils.py:24-25, imported from /root/reference on CPU), in float64,
on seeded inputs shaped like one training view (K = 64 codes, Df = 512).

The steps around cos_loss follow the reference's semantics (written here,
since scene.* does not import without plyfile/cv2):
  f = codebooks[0].T @ weight_map.view(K, -1)        scene/gaussian_model.py:533-543 (layer 0)
  gt = feature_map[seg].permute, mask = seg != -1    scene/cameras.py:77-94
  loss = cos_loss(f * mask, gt * mask)               train.py:162-164
Edge cases: masked pixels (-1), an all-zero weight column (|f| < eps) inside a
segment, a segment whose feature row is zero (|gt| < eps), and pixels with
non-zero weights everywhere else.
Run:  python tests/golden/make_lang_loss_golden.py
"""
import os
import sys

import numpy as np
import torch

REF = os.environ.get("LSR_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
from utils.loss_utils import cos_loss  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_lang_loss.npz")


def case(g, K, Df, H, W, S):
    logits = torch.randn(K, H * W, generator=g, dtype=torch.float64)
    wm = torch.softmax(logits * 2.0, dim=0)                 # soft codes blended per pixel
    wm = wm * torch.rand(1, H * W, generator=g, dtype=torch.float64)   # partial coverage
    wm = wm.reshape(K, H, W)
    wm[:, 0, 1] = 0.0                                       # |f| = 0 inside a segment
    cb = torch.randn(1, K, Df, generator=g, dtype=torch.float64)
    feat = torch.randn(S, Df, generator=g, dtype=torch.float64)
    feat[S - 1] = 0.0                                       # |gt| = 0 segment
    seg = torch.randint(-1, S, (H, W), generator=g)
    seg[0, 1] = 0
    seg[1, :3] = S - 1
    return wm, cb, seg, feat


def reference_loss(wm, cb, seg, feat):
    K, H, W = wm.shape
    f = (cb[0].T @ wm.reshape(K, -1)).reshape(-1, H, W)
    s = seg.reshape(-1)
    mask = (s != -1).reshape(1, H, W)
    gt = feat[s].reshape(H, W, -1).permute(2, 0, 1)
    return cos_loss(f * mask, gt * mask)


def main():
    g = torch.Generator().manual_seed(2024)
    out = {}
    for name, (H, W, S) in {"a": (12, 20, 7), "b": (9, 33, 3)}.items():
        wm, cb, seg, feat = case(g, 64, 512, H, W, S)
        wm.requires_grad_(True)
        cb.requires_grad_(True)
        loss = reference_loss(wm, cb, seg, feat)
        loss.backward()
        out[f"{name}_weight_map"] = wm.detach().float().numpy()
        out[f"{name}_codebooks"] = cb.detach().float().numpy()
        out[f"{name}_seg"] = seg.numpy().astype(np.int32)
        out[f"{name}_features"] = feat.float().numpy()
        # the expected values from the float32-rounded inputs, in float64
        wm32 = torch.from_numpy(out[f"{name}_weight_map"]).double().requires_grad_(True)
        cb32 = torch.from_numpy(out[f"{name}_codebooks"]).double().requires_grad_(True)
        l32 = reference_loss(wm32, cb32, seg, torch.from_numpy(out[f"{name}_features"]).double())
        l32.backward()
        out[f"{name}_loss"] = np.float64(l32.item())
        out[f"{name}_grad_weight_map"] = wm32.grad.numpy()
        out[f"{name}_grad_codebooks"] = cb32.grad.numpy()
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
