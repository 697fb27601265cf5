"""Measured work units of the list-driven render backward at cfg3 (or LSR_CFG):
the number of staged (candidate, 8x8-block) pairs k_render_bwd_mf<., LST> walks,
i.e. the sum of the per-block list counts the forward wrote (lsr_fwd_out.lists:
listA, listB, then lcount[4T] at 2 x align256(4 M x 16), csrc/lsr_api.hip
set_block_lists).  Prints the integer (tools/pass.py pmc feeds it to
tools/pmc_issue.py --units)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import _lib, rasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
dev = torch.device("cuda:0")
W, H, N, D = cfg["W"], cfg["H"], cfg["N"], cfg["lang_dim"]
cam = make_camera(W, H)
g0 = make_gaussians(N, cam, seed=0, sh_degree=3, lang_dim=D)
g = {k: v.to(dev) for k, v in g0.items() if isinstance(v, torch.Tensor)}
rs = bench.settings(cam, dev, 3, D > 0)
e = torch.empty(0, device=dev)
with torch.no_grad():
    _, _, _, M, bufs, _, _, _ = rasterizer._run_forward(
        g["means3D"], g["shs"], e, g["language_feature_precomp"], e, e, g["opacities"], g["scales"],
        g["rotations"], e, rs, grad_request=_lib.LSR_GWS_GEOM | (_lib.LSR_GWS_LANG if D else 0))
torch.cuda.synchronize()
lists = bufs.get(_lib.LSR_BUF_LISTS)
if lists is None:
    raise SystemExit("no block lists written (LSR_OPT_LISTS_MAX_MB budget?)")
align = lambda x: (x + 255) // 256 * 256  # noqa: E731
off = 2 * align(4 * M * 16)
T = ((W + 15) // 16) * ((H + 15) // 16)
lcount = lists[off:off + 4 * T * 4].view(torch.int32)
print(int(lcount.long().sum()))
