"""Work census of the render backward at cfg3 (analysis only, torch on the GPU).

For every tile-list instance at a position below its 8x8 block's largest
n_contrib, evaluates the pair (instance, pixel) over the block's 64 pixels and
counts:
  staged      (instance, block) pairs whose cut ellipse reaches the block
              (approximated: some pixel of the block has power >= cut)
  contrib_blk (instance, block) pairs with at least one contributing pixel
              (alpha >= 1/255 and position < that pixel's n_contrib)
  contrib_tile distinct (instance, tile) pairs with a contributing pixel
  contrib_px  contributing (instance, pixel) pairs
These bound the backward's group slots, its line atomics per 8x8 block and
per 16x16 tile.  Usage: python tools/bwd_work.py  (LSR_CFG=3 default)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import layout, rasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
dev = torch.device("cuda:0")
W, H, N, D = cfg["W"], cfg["H"], cfg["N"], cfg["lang_dim"]
cam = make_camera(W, H)
g0 = make_gaussians(N, cam, seed=0, sh_degree=3, lang_dim=D)
g = {k: v.to(dev) for k, v in g0.items() if isinstance(v, torch.Tensor)}
rs = bench.settings(cam, dev, 3, True)
e = torch.empty(0, device=dev)
with torch.no_grad():
    _, _, radii, M, bufs, _, _, _ = rasterizer._run_forward(
        g["means3D"], g["shs"], e, g["language_feature_precomp"], e, e, g["opacities"], g["scales"],
        g["rotations"], e, rs)
dec = layout.decode(bufs, N, W, H, M)
gx, gy = (W + 15) // 16, (H + 15) // 16
T = gx * gy
nc = torch.zeros((gy * 16, gx * 16), dtype=torch.int64, device=dev)
nc[:H, :W] = dec["n_contrib"].long()
# per tile, per block (4), per pixel (64): n_contrib
ncb = nc.view(gy, 2, 8, gx, 2, 8).permute(0, 3, 1, 4, 2, 5).reshape(T, 4, 64)
wmax_b = ncb.amax(dim=2)                     # (T, 4)
ranges = dec["ranges"].long()
pl = dec["point_list"].long()
xy = dec["xy"]
co = dec["conic_opacity"]
cut = dec["cut"]
# pixel coords of each (block, pixel)
by = torch.arange(4, device=dev) // 2
bx = torch.arange(4, device=dev) % 2
q = torch.arange(64, device=dev)
px_off = (bx[:, None] * 8 + q[None, :] % 8).float()   # (4, 64)
py_off = (by[:, None] * 8 + q[None, :] // 8).float()
stats = dict(staged=0, contrib_blk=0, contrib_tile=0, contrib_px=0, inst_visited=0)
chunk_tiles = 64
for t0 in range(0, T, chunk_tiles):
    t1 = min(T, t0 + chunk_tiles)
    for t in range(t0, t1):
        s, e_ = ranges[t, 0].item(), ranges[t, 1].item()
        wm = int(wmax_b[t].max().item())
        n = min(e_ - s, wm)
        if n <= 0:
            continue
        ids = pl[s:s + n]
        ty, tx = t // gx, t % gx
        px = tx * 16 + px_off            # (4, 64)
        py = ty * 16 + py_off
        dx = xy[ids, 0][:, None, None] - px[None]   # (n, 4, 64)
        dy = xy[ids, 1][:, None, None] - py[None]
        A, B, C, o = co[ids, 0], co[ids, 1], co[ids, 2], co[ids, 3]
        power = -0.5 * (A[:, None, None] * dx * dx + C[:, None, None] * dy * dy) - B[:, None, None] * dx * dy
        pos = torch.arange(n, device=dev)
        inblk = pos[:, None] < wmax_b[t][None, :]                        # (n, 4)
        stg = ((power >= cut[ids][:, None, None]) & (power <= 0)).any(dim=2) & inblk
        alpha = torch.clamp(o[:, None, None] * torch.exp(power), max=0.99)
        contrib = (power <= 0) & (alpha >= 1 / 255) & (pos[:, None, None] < ncb[t][None])
        cb = contrib.any(dim=2)
        stats["staged"] += int(stg.sum())
        stats["contrib_blk"] += int(cb.sum())
        stats["contrib_tile"] += int(cb.any(dim=1).sum())
        stats["contrib_px"] += int(contrib.sum())
        stats["inst_visited"] += int(inblk.sum())
print({"M": M, "visible": int((radii > 0).sum()), **stats})
