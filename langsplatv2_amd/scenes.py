"""Seeded synthetic cameras and Gaussian clouds for the BASELINE.json configs
(SURVEY.md §8d).  There is no dataset access here, so every benchmark and
parity case is built from these generators (data = "synthetic").

Camera conventions restate the reference:
  getWorld2View2        utils/graphics_utils.py:38-49
  getProjectionMatrix   utils/graphics_utils.py:51-71
  world_view_transform / full_proj_transform / camera_center
                        scene/cameras.py:55-58 (znear 0.01, zfar 100 :49-50)
Language inputs restate utils/vq_utils.py:9-40 on the CPU (input synthesis
only; the product producer is the fused HIP kernel behind lang_codes.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch



def softmax_to_topk_soft_code(logits: torch.Tensor, k: int) -> torch.Tensor:
    """CPU torch restatement of utils/vq_utils.py:9-24 (input synthesis)."""
    y = logits.softmax(dim=1)
    _, idx = torch.topk(y, k, dim=1)
    mask = torch.zeros_like(y, dtype=torch.bool).scatter_(1, idx, True)
    y = torch.where(mask, y, torch.zeros_like(y))
    return y / (y.sum(dim=1, keepdim=True) + 1e-10)


def get_weights_and_indices(logits: torch.Tensor, k: int):
    """CPU torch restatement of utils/vq_utils.py:26-40 (input synthesis)."""
    code = softmax_to_topk_soft_code(logits, k)
    nz = code != 0
    w = code[nz].view(code.shape[0], k)
    i = torch.arange(code.shape[1], device=code.device).expand_as(code)[nz].view(code.shape[0], k)
    return w.float(), i.float()


def get_world2view2(R: np.ndarray, t: np.ndarray, translate=np.zeros(3), scale=1.0) -> np.ndarray:
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    C2W[:3, 3] = (C2W[:3, 3] + translate) * scale
    return np.float32(np.linalg.inv(C2W))


def get_projection_matrix(znear: float, zfar: float, fovX: float, fovY: float) -> torch.Tensor:
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def make_camera(W: int, H: int, fovx_deg: float = 60.0, yaw_deg: float = 0.0, device="cpu") -> dict:
    """Camera at the origin, rotated by `yaw_deg` about +y; tanfovy = tanfovx*H/W."""
    tanfovx = math.tan(math.radians(fovx_deg) / 2)
    tanfovy = tanfovx * H / W
    fovx, fovy = 2 * math.atan(tanfovx), 2 * math.atan(tanfovy)
    a = math.radians(yaw_deg)
    R = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    wv = torch.tensor(get_world2view2(R, np.zeros(3))).transpose(0, 1)
    proj = get_projection_matrix(0.01, 100.0, fovx, fovy).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
    campos = wv.inverse()[3, :3]
    return dict(W=W, H=H, tanfovx=tanfovx, tanfovy=tanfovy, viewmatrix=wv.contiguous().to(device),
                projmatrix=full.contiguous().to(device), campos=campos.contiguous().to(device))


def make_gaussians(N: int, cam: dict, seed: int = 0, sh_degree: int | None = 3, lang_dim: int = 0,
                   quick_k: int = 0, quick_levels: int = 3, quick_codes: int = 64, device="cpu") -> dict:
    """Gaussians per SURVEY.md §8d: z ~ U[2,12] inside 1.1x the frustum, 1 % near-culled,
    log-uniform scales [0.003, 0.03], random unit quaternions, sigmoid(N(0,1.5))
    opacities; SH (deg 3: DC ~ N(0,0.5), rest ~ N(0,0.1)) or colors U[0,1];
    dense language = top-4 soft codes of N(0,1) logits (D < 4: U[0,1]);
    quick = per-level top-k (weights, fp32 indices + 64*level)."""
    g = torch.Generator().manual_seed(seed)
    tx, ty = cam["tanfovx"], cam["tanfovy"]
    z = 2.0 + 10.0 * torch.rand(N, generator=g)
    u = torch.rand(N, generator=g) * 2 - 1
    v = torch.rand(N, generator=g) * 2 - 1
    x = u * z * tx * 1.1
    y = v * z * ty * 1.1
    near = torch.rand(N, generator=g) < 0.01
    z = torch.where(near, -1.0 + 1.2 * torch.rand(N, generator=g), z)
    means = torch.stack([x, y, z], 1).float()
    # rotate the cloud with the camera's world frame: the view matrix is a
    # rotation here, so world = R_view^T * camera-space
    wv = cam["viewmatrix"].cpu().t()[:3, :3]
    means = (means @ wv).contiguous()
    logs = math.log(0.003) + (math.log(0.03) - math.log(0.003)) * torch.rand(N, 3, generator=g)
    scales = torch.exp(logs).float()
    rot = torch.randn(N, 4, generator=g)
    rot = (rot / rot.norm(dim=1, keepdim=True)).float()
    opac = torch.sigmoid(1.5 * torch.randn(N, 1, generator=g)).float()
    out = dict(means3D=means, scales=scales, rotations=rot, opacities=opac)
    if sh_degree is not None:
        M = (sh_degree + 1) ** 2
        sh = torch.empty(N, 16 if sh_degree <= 3 else M, 3)
        sh[:, 0] = 0.5 * torch.randn(N, 3, generator=g)
        sh[:, 1:] = 0.1 * torch.randn(N, sh.shape[1] - 1, 3, generator=g)
        out["shs"] = sh.float().contiguous()
        out["sh_degree"] = sh_degree
    else:
        out["colors_precomp"] = torch.rand(N, 3, generator=g).float()
        out["sh_degree"] = 0
    if lang_dim > 0:
        if lang_dim < 4:
            out["language_feature_precomp"] = torch.rand(N, lang_dim, generator=g).float()
        else:
            logits = torch.randn(N, lang_dim, generator=g)
            out["language_feature_precomp"] = softmax_to_topk_soft_code(logits, 4).float().contiguous()
    if quick_k > 0:
        ws, ids = [], []
        for lvl in range(quick_levels):
            logits = torch.randn(N, quick_codes, generator=g)
            w, i = get_weights_and_indices(logits, quick_k)
            ws.append(w)
            ids.append(i + float(lvl * quick_codes))
        out["language_feature_weights_quick"] = torch.cat(ws, 1).contiguous()
        out["language_feature_indices"] = torch.cat(ids, 1).contiguous()
        out["quick_dim"] = quick_levels * quick_codes
    return {k: (t.to(device) if isinstance(t, torch.Tensor) else t) for k, t in out.items()}


# BASELINE.json configs (index = position in "configs")
CONFIGS = {
    1: dict(N=1_000, W=128, H=128, sh_degree=None, lang_dim=0, backward=True),
    2: dict(N=100_000, W=800, H=800, sh_degree=None, lang_dim=3, backward=False),
    3: dict(N=1_000_000, W=1920, H=1080, sh_degree=3, lang_dim=16, backward=True),
    5: dict(N=5_000_000, W=3840, H=2160, sh_degree=3, lang_dim=32, backward=False),
}
