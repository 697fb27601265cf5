"""Measured error of the fused language loss's gradients (csrc/lang_loss.hip) against the
float64 oracle, next to the error of the reference's own fp32 formulation
(train.py:157-163: f = codebooks[0].T @ W; cos_loss(f * mask, gt * mask),
utils/loss_utils.py:24-25, run in fp32 torch on the same GPU) against the same float64
truth.  Metrics as tests/test_lang_loss.py: dL/dW per pixel relative to that pixel's
largest |gradient| (worst pixel), dL/dcodebooks relative to the largest |entry|.
Usage: python tools/loss_err.py"""
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import oracle as O  # noqa: E402
from test_lang_loss import _gpu_loss, _random_case  # noqa: E402


def rel_w(got, ref):
    K = ref.shape[0]
    g = got.reshape(K, -1).astype(np.float64)
    r = ref.reshape(K, -1)
    scale = np.maximum(np.abs(r).max(0), 1e-12)
    e = np.abs(g - r).max(0) / scale
    return float(e.max()), float(np.percentile(e, 99.9))


def rel_cb(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1e-30))


def ref_fp32(wm, cb, seg, feat):
    dev = torch.device("cuda:0")
    W = torch.from_numpy(wm).to(dev).requires_grad_(True)
    C = torch.from_numpy(cb).to(dev).requires_grad_(True)
    K, H, Wd = wm.shape
    f = (C.T @ W.view(K, -1)).view(-1, H, Wd)
    s = torch.from_numpy(seg).to(dev).long()
    mask = (s >= 0).float()[None]
    gt = torch.from_numpy(feat).to(dev)[s.clamp(min=0)].permute(2, 0, 1)
    loss = 1 - F.cosine_similarity(f * mask, gt * mask, dim=0).mean()
    loss.backward()
    return loss.item(), W.grad.cpu().numpy(), C.grad.cpu().numpy()


out = {}
gold = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                            "ref_lang_loss.npz"))
for name in ("a", "b"):
    z = {k[2:]: gold[k] for k in gold.files if k.startswith(name + "_")}
    l, gw, gcb = _gpu_loss(z["weight_map"].astype(np.float32), z["codebooks"].astype(np.float32), z["seg"],
                           z["features"].astype(np.float32))
    # the oracle on the same fp32-rounded inputs (float64 arithmetic), and the golden (float64 inputs)
    ol, ow, ocb = O.lang_cos_loss(z["weight_map"].astype(np.float32), z["codebooks"][0].astype(np.float32),
                                  z["seg"], z["features"].astype(np.float32))
    out[f"golden_{name}"] = dict(
        fused_vs_golden=dict(loss_abs=abs(l - float(z["loss"])), dW_worst_pixel=rel_w(gw, z["grad_weight_map"])[0],
                             dCB=rel_cb(gcb[0], z["grad_codebooks"][0])),
        fused_vs_oracle_fp32_inputs=dict(loss_abs=abs(l - ol), dW_worst_pixel=rel_w(gw, ow)[0],
                                         dCB=rel_cb(gcb[0], ocb)))
for (H, W, S, seed) in [(67, 93, 40, 0), (128, 128, 5, 1), (4, 16, 1, 2), (33, 250, 300, 3), (270, 480, 200, 5)]:
    wm, cb, seg, feat = _random_case(64, 512, H, W, S, seed)
    rl, rw, rcb = O.lang_cos_loss(wm, cb, seg, feat)
    l, gw, gcb = _gpu_loss(wm, cb, seg, feat)
    fl, fw, fcb = ref_fp32(wm, cb, seg, feat)
    out[f"{H}x{W}_S{S}"] = dict(
        fused=dict(loss_abs=abs(l - rl), dW_worst_pixel=rel_w(gw, rw)[0], dW_p99_9=rel_w(gw, rw)[1],
                   dCB=rel_cb(gcb, rcb)),
        reference_fp32=dict(loss_abs=abs(fl - rl), dW_worst_pixel=rel_w(fw, rw)[0], dW_p99_9=rel_w(fw, rw)[1],
                            dCB=rel_cb(fcb, rcb)))
print(json.dumps(out, indent=1))
