"""Generate tests/golden/ref_utils.npz by running the REFERENCE's own Python
utilities (from /root/reference, importable here on CPU) on seeded inputs.

These vectors pin the oracle's / package's restatements of the path's edges:
  utils/sh_utils.py:57-112        eval_sh (degrees 0..3)
  utils/general_utils.py:78-110   build_rotation / build_scaling_rotation
                                  (hard-coded device="cuda" is redirected to
                                  CPU for generation only) + strip_symmetric
  utils/graphics_utils.py:38-71   getWorld2View2, getProjectionMatrix
  scene/cameras.py:55-58          world_view / full_proj / camera_center recipe
  utils/vq_utils.py:9-40          softmax_to_topk_soft_code, get_weights_and_indices
Run:  python tests/golden/make_ref_golden.py   (needs /root/reference; the
resulting .npz is committed and is all that travels to the GPU box).
"""
import math
import os
import sys

import numpy as np
import torch

REF = os.environ.get("LSR_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

_zeros = torch.zeros


def _cpu_zeros(*a, **k):
    k.pop("device", None)
    return _zeros(*a, **k)


torch.zeros = _cpu_zeros          # the reference hard-codes device="cuda"
from utils import general_utils, graphics_utils, sh_utils, vq_utils  # noqa: E402
torch.zeros = _zeros

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_utils.npz")


def main():
    g = torch.Generator().manual_seed(1234)
    out = {}
    # --- SH: per degree, (N, 3, 16) coefficients and unit directions
    N = 512
    sh = torch.randn(N, 3, 16, generator=g) * 0.3
    dirs = torch.randn(N, 3, generator=g)
    dirs = dirs / dirs.norm(dim=1, keepdim=True)
    out["sh_coeffs"] = sh.numpy()
    out["sh_dirs"] = dirs.numpy()
    for deg in range(4):
        out[f"sh_eval_deg{deg}"] = sh_utils.eval_sh(deg, sh, dirs).numpy()
    # --- covariance from scale + rotation (the reference normalises q)
    s = torch.exp(torch.randn(N, 3, generator=g) - 4.0)
    q = torch.randn(N, 4, generator=g)
    torch.zeros = _cpu_zeros
    try:
        L = general_utils.build_scaling_rotation(s, q)
        cov = general_utils.strip_symmetric(L @ L.transpose(1, 2))
        R = general_utils.build_rotation(q)
    finally:
        torch.zeros = _zeros
    out["cov_scales"] = s.numpy()
    out["cov_quats"] = q.numpy()
    out["cov3D"] = cov.numpy()
    out["rotmat"] = R.numpy()
    # --- cameras
    for i, (W, H, fovx_deg, yaw) in enumerate([(1920, 1080, 60.0, 0.0), (800, 800, 50.0, 12.0), (128, 96, 70.0, -20.0)]):
        tanfovx = math.tan(math.radians(fovx_deg) / 2)
        fovx = 2 * math.atan(tanfovx)
        fovy = 2 * math.atan(tanfovx * H / W)
        a = math.radians(yaw)
        Rm = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        T = np.array([0.1 * i, -0.2 * i, 0.3 * i])
        wv = torch.tensor(graphics_utils.getWorld2View2(Rm, T)).transpose(0, 1)
        proj = graphics_utils.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
        out[f"cam{i}_params"] = np.array([W, H, fovx_deg, yaw], np.float64)
        out[f"cam{i}_R"] = Rm
        out[f"cam{i}_T"] = T
        out[f"cam{i}_world_view"] = wv.numpy()
        out[f"cam{i}_full_proj"] = full.numpy()
        out[f"cam{i}_center"] = wv.inverse()[3, :3].numpy()
    # --- language codes (K = 64 codebook, k = 4; and a 3-level quick set)
    logits = torch.randn(300, 64, generator=g)
    out["lang_logits"] = logits.numpy()
    out["lang_topk4"] = vq_utils.softmax_to_topk_soft_code(logits, 4).numpy()
    w, idx = vq_utils.get_weights_and_indices(logits, 4)
    out["lang_quick_w"] = w.numpy()
    out["lang_quick_idx"] = idx.numpy()
    # k = 1 and 8 codes; torch-autograd gradient of the reference function
    for kk in (1, 8):
        out[f"lang_topk{kk}"] = vq_utils.softmax_to_topk_soft_code(logits, kk).numpy()
    gup = torch.randn(300, 64, generator=g)
    x = logits.clone().requires_grad_(True)
    vq_utils.softmax_to_topk_soft_code(x, 4).backward(gup)
    out["lang_grad_up"] = gup.numpy()
    out["lang_topk4_dlogits"] = x.grad.numpy()
    # 3 levels x 64: get_render_weights' per-level loop (scene/gaussian_model.py:510-518,
    # restated here because scene/ does not import offline) and the quick-path
    # level-offset concatenation (eval_lerf.py:340-348)
    logits3 = torch.randn(200, 192, generator=g) * 1.5
    out["lang3_logits"] = logits3.numpy()
    out["lang3_render_weights"] = torch.cat(
        [vq_utils.softmax_to_topk_soft_code(logits3[:, i * 64:(i + 1) * 64], 4) for i in range(3)], dim=-1).numpy()
    ws, ids = [], []
    for i in range(3):
        w3, i3 = vq_utils.get_weights_and_indices(logits3[:, i * 64:(i + 1) * 64], 4)
        ws.append(w3)
        ids.append(i3 + int(i * 64))
    out["lang3_quick_w"] = torch.cat(ws, dim=1).numpy()
    out["lang3_quick_idx"] = torch.cat(ids, dim=1).numpy()
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
