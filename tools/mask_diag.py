"""Check the forward's block lists (listA/B/lcount/listM) of one small case:
every entry's contribution mask against a float32 re-evaluation of the pair at
the block's 64 pixels (power <= 0, alpha >= 1/255 with the fast exp, position
< n_contrib); prints the disagreements (outside the exp's error band they are
bugs)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from harness import gpu_inputs, make_case, settings_for  # noqa: E402
from test_gpu_parity import CASES  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import layout  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cov_precomp_lang8"
dev = torch.device("cuda:0")
case = make_case(**CASES[name])
t = gpu_inputs(case, dev, requires_grad=True)
kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations", "cov3D_precomp", "language_feature_precomp")
      if k in t}
color, lang, radii = GaussianRasterizer(settings_for(case, dev))(means3D=t["means3D"], means2D=t["means2D"],
                                                                  opacities=t["opacities"], **kw)
torch.cuda.synchronize()
node = color.grad_fn
M = int(node.num_rendered)
W, H = case["cam"]["W"], case["cam"]["H"]
gx, gy = (W + 15) // 16, (H + 15) // 16
T = gx * gy
a256 = lambda x: (x + 255) // 256 * 256  # noqa: E731
lb = node.lists.detach().view(torch.uint8).cpu().numpy()
offB = a256(4 * M * 16)
offC = 2 * offB
offM = offC + a256(4 * T * 4)
LA = lb[:4 * M * 16].view(np.float32).reshape(-1, 4)
LB = lb[offB:offB + 4 * M * 16].view(np.float32).reshape(-1, 4)
LC = lb[offC:offC + 4 * T * 4].view(np.uint32)
LM = lb[offM + 16 * 8:offM + 16 * 8 + 4 * M * 8].view(np.uint64)
saved = node.saved_tensors
image = saved[-1]
N = t["means3D"].shape[0]
dec = {k: v.cpu().numpy() for k, v in layout.decode({2: image, 1: saved[-2], 0: saved[-3]}, N, W, H, M).items()}
ts = dec["ranges"][:, 0].astype(np.int64)
ncon = dec["n_contrib"]
f = np.float32
bad = 0
tot = 0
for tile in range(T):
    tx, ty = tile % gx, tile // gx
    rs = ts[tile]
    n_tile = dec["ranges"][tile, 1] - rs
    for sub in range(4):
        cnt = int(LC[4 * tile + sub])
        if cnt == 0:
            continue
        base = 4 * rs + sub * n_tile
        bx = tx * 16 + (sub & 1) * 8
        by = ty * 16 + (sub >> 1) * 8
        ls = np.arange(64)
        px, py = bx + (ls & 7), by + (ls >> 3)
        inside = (px < W) & (py < H)
        nc = np.where(inside, ncon[np.minimum(py, H - 1), np.minimum(px, W - 1)], 0)
        for e in range(cnt):
            A, B = LA[base + e], LB[base + e]
            pos = int(B[3:4].view(np.int32)[0])
            dx, dy = f(A[0]) - px.astype(f), f(A[1]) - py.astype(f)
            p = f(-0.5) * (f(A[2]) * dx * dx + f(B[0]) * dy * dy) - f(A[3]) * dx * dy
            al = np.minimum(f(0.99), f(B[1]) * np.exp(p.astype(np.float64)).astype(f))
            want = inside & (p <= 0) & (al >= 1 / 255) & (pos < nc)
            got = (np.uint64(LM[base + e]) >> ls.astype(np.uint64)) & np.uint64(1)
            diff = np.nonzero(want != got.astype(bool))[0]
            tot += 1
            if len(diff):
                bad += 1
                if bad <= 12:
                    print(f"tile {tile} sub {sub} entry {e}/{cnt} pos {pos} gid {int(B[2:3].view(np.uint32)[0])}: "
                          f"lanes {diff[:8].tolist()} want {want[diff[:8]].astype(int).tolist()} "
                          f"alpha {al[diff[:4]].tolist()} nc {nc[diff[:4]].tolist()} mask {int(LM[base + e]):016x}")
print(f"{name}: {bad} of {tot} entries disagree")
