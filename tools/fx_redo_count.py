"""Census of the fast-exp forward's exact re-renders (render.hip FX): with the
variant built by
  python tools/variant.py fxmark 'if (FX && !exact && redo != 0u) continue;' 'const bool mark = ...'
(lane 0 of a block whose termination test fell in the error band stores
final_T = -1 instead of re-rendering), count the marked 8x8 blocks per config.
Usage: python tools/fx_redo_count.py path/to/liblsr.so [cfg ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import _lib, layout, rasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

lib = _lib.load(sys.argv[1])
_lib._lib = lib
dev = torch.device("cuda:0")
for cid in [int(c) for c in (sys.argv[2:] or ["3", "5"])]:
    cfg = CONFIGS[cid]
    W, H, N, D = cfg["W"], cfg["H"], cfg["N"], cfg["lang_dim"]
    cam = make_camera(W, H)
    g = {k: v.to(dev) for k, v in make_gaussians(N, cam, seed=0, sh_degree=3, lang_dim=D).items()
         if isinstance(v, torch.Tensor)}
    rs = bench.settings(cam, dev, 3, True)
    e = torch.empty(0, device=dev)
    _, _, _, M, bufs, _, _, _ = rasterizer._run_forward(g["means3D"], g["shs"], e, g["language_feature_precomp"], e, e,
                                                         g["opacities"], g["scales"], g["rotations"], e, rs)
    fT = layout.decode(bufs, N, W, H, M)["final_T"]
    marked = int((fT == -1.0).sum().item())
    blocks = ((W + 7) // 8) * ((H + 7) // 8)
    print(f"cfg{cid}: {marked} of {blocks} 8x8 blocks re-rendered exactly ({100.0 * marked / blocks:.3f} %)", flush=True)
