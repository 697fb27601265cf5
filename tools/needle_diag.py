"""Diagnose tests/test_cull_vs_full.py::test_needles_culled_gpu_equals_full_reference_lists:
on the sampled needle tiles, compare the GPU image with the oracle rendering
the CULLED lists and the UNCULLED lists, and for mismatching pixels list the
instances the cull dropped that contribute there (alpha >= 1/255 in fp32)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from harness import add_needles, make_case, needle_contributing_tiles, oracle_problem, run_gpu_forward  # noqa: E402
from oracle import oracle as O  # noqa: E402

W = H = 3072
gx = (W + 15) // 16
case = add_needles(make_case(N=60, W=W, H=H, seed=31, sh_degree=None, lang_dim=3), frac=1.0, seed=1,
                   sigma_px=(400.0, 1500.0))
pb = oracle_problem(case)
nt = 16
culled0 = O.forward(pb, nthreads=nt, tiles=np.zeros(0, np.int32), cull=True)
contrib = needle_contributing_tiles(culled0, W, H)
alltiles = sorted(set().union(*contrib.values()))
tiles = np.sort(np.random.default_rng(4).choice(alltiles, size=min(96, len(alltiles)), replace=False)).astype(np.int32)
ref_u = O.forward(pb, nthreads=nt, tiles=tiles, cull=False)
ref_c = O.forward(pb, nthreads=nt, tiles=tiles, cull=True)
got = run_gpu_forward(case, torch.device("cuda:0"))
print("lists equal:", np.array_equal(got["point_list"], culled0["point_list"].astype(np.int32)))
for t in tiles:
    tx, ty = t % gx, t // gx
    sl = (slice(None), slice(ty * 16, ty * 16 + 16), slice(tx * 16, tx * 16 + 16))
    g, u, c = got["color"][sl], ref_u["color"][sl], ref_c["color"][sl]
    ngu, ngc, ncu = int((g != u).sum()), int((g != c).sum()), int((c != u).sum())
    if ngu or ngc or ncu:
        print(f"tile {t} ({tx},{ty}): gpu!=uncull {ngu}  gpu!=cull {ngc}  cull!=uncull {ncu}")
        # which Gaussians the unculled list has for this tile and the culled one not
        ru, rc = ref_u["ranges"][t], ref_c["ranges"][t]
        lu = set(ref_u["point_list"][ru[0]:ru[1]].tolist())
        lc = set(ref_c["point_list"][rc[0]:rc[1]].tolist())
        print("   dropped by cull:", sorted(lu - lc)[:20], " n_contrib gpu/cull/uncull max:",
              int(got["n_contrib"][sl[1:]].max()), int(ref_c["n_contrib"][sl[1:]].max()),
              int(ref_u["n_contrib"][sl[1:]].max()))
        ys, xs = np.nonzero((g != u).any(0))
        for y, x in list(zip(ys, xs))[:3]:
            py, px = ty * 16 + y, tx * 16 + x
            print(f"   px ({px},{py}) gpu {g[:, y, x]} uncull {u[:, y, x]} cull {c[:, y, x]}"
                  f" T gpu {got['final_T'][py, px]} uncull {ref_u['final_T'][py, px]}")

# records: GPU vs oracle for the visible Gaussians
vis = culled0["radii"] > 0
for k in ("xy", "conic_opacity", "depth"):
    a, b = got[k][vis], culled0[k][vis]
    bad = np.nonzero((a != b).reshape(a.shape[0], -1).any(1))[0]
    print(k, "mismatching Gaussians:", len(bad), "of", int(vis.sum()))
    for i in bad[:3]:
        print("   gpu", a[i], "oracle", b[i])
# the pair behind the first mismatching pixels: the Gaussian the GPU blended (colour / 0.99) and the
# forward's operations on it, in float32 with fmaf emulated through float64 (exact product)
col = case["g"]["colors_precomp"].numpy()
f32 = np.float32


def fmaf(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


shown = 0
for tt in tiles:
    tx, ty = tt % gx, tt // gx
    sl = (slice(None), slice(ty * 16, ty * 16 + 16), slice(tx * 16, tx * 16 + 16))
    ys, xs = np.nonzero((got["color"][sl] != ref_c["color"][sl]).any(0))
    if not len(ys):
        continue
    py, px = ty * 16 + ys[0], tx * 16 + xs[0]
    c = got["color"][:, py, px]
    r = culled0["ranges"][tt]
    ids = culled0["point_list"][r[0]:r[1]]
    best = min(ids, key=lambda i: float(np.abs(col[i] * 0.99 - c).sum()))
    x, y = got["xy"][best]
    ca, cb, cc, o = got["conic_opacity"][best]
    dx, dy = f32(f32(x) - f32(px)), f32(f32(y) - f32(py))
    inner = fmaf(f32(ca * dx), dx, f32(f32(cc * dy) * dy))
    p = fmaf(f32(-0.5), inner, -f32(f32(cb * dx) * dy))
    print(f"px ({px},{py}) gpu colour {c} -> id {best} colour*0.99 {col[best] * 0.99} in-list pos "
          f"{int(np.nonzero(ids == best)[0][0])}/{len(ids)} xy ({x},{y}) conic ({ca!r},{cb!r},{cc!r}) o {o!r}"
          f" dx {dx!r} dy {dy!r} inner {inner!r} power {p!r}")
    shown += 1
    if shown >= 4:
        break
