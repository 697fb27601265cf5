"""The product's tile cull against the reference's FULL instance lists.

The binning here drops (Gaussian, tile) instances whose cut ellipse misses the
tile (DESIGN §3 "Tile cull"); the reference emits one instance per tile of the
3-sigma rect (consumed by
/root/reference/gaussian_renderer/__init__.py:108-119 through the
rasterizer).  These tests run the GPU's culled path against the oracle
rendering the reference's UNCULLED lists (oracle.forward(cull=False)) at
BASELINE sizes:

  * cfg2 (100k, 800x800, RGB + 3 language channels): the whole frame —
    colour, language, final_T, radii bit-exact; n_contrib, which is a position
    in a tile's list, compared as the Gaussian id of each pixel's last
    contributor (the same Gaussian in both lists);
  * cfg3 (1M, 1920x1080, SH3 + 16): 48 seeded tiles' images bit-exact, and the
    full backward with dL/dout restricted to 32 tiles against the oracle's
    backward over the full lists (GRAD_RTOL).
"""
import os

import numpy as np
import pytest

from harness import assert_grad_close, assert_img, fwd_atol, make_case, oracle_problem, run_gpu_fwd_bwd, run_gpu_forward
from langsplatv2_amd.scenes import CONFIGS

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _case(cfg_id):
    c = CONFIGS[cfg_id]
    return make_case(N=c["N"], W=c["W"], H=c["H"], sh_degree=c["sh_degree"], lang_dim=c["lang_dim"], seed=0)


def _threads():
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else min(16, os.cpu_count() or 1)


def _tile_pixels(tiles, gx, W, H):
    ys, xs = [], []
    for t in tiles:
        tx, ty = t % gx, t // gx
        yy, xx = np.mgrid[ty * 16:min(ty * 16 + 16, H), tx * 16:min(tx * 16 + 16, W)]
        ys.append(yy.ravel())
        xs.append(xx.ravel())
    return np.concatenate(ys), np.concatenate(xs)


def _last_contributor_ids(out, W, H):
    """Per pixel: the Gaussian id at list position n_contrib - 1 of its tile (-1: none)."""
    gx = (W + 15) // 16
    ys, xs = np.mgrid[0:H, 0:W]
    tile = (ys // 16) * gx + xs // 16
    start = out["ranges"][:, 0].astype(np.int64)[tile]
    nc = out["n_contrib"].astype(np.int64)
    pl = out["point_list"].astype(np.int64)
    idx = np.clip(start + nc - 1, 0, max(pl.size - 1, 0))
    return np.where(nc > 0, pl[idx] if pl.size else -1, -1)


def test_cfg2_culled_gpu_equals_full_reference_lists(gpu, oracle_lib):
    case = _case(2)
    W, H = case["cam"]["W"], case["cam"]["H"]
    pb = oracle_problem(case)
    ref = oracle_lib.forward(pb, nthreads=_threads(), cull=False)
    got = run_gpu_forward(case, gpu)
    assert got["num_rendered"] < ref["num_rendered"]          # the cull removed instances
    np.testing.assert_array_equal(got["radii"], ref["radii"])
    fa = fwd_atol(case)
    assert_img(got["color"], ref["color"], fa, "color")
    assert_img(got["lang"], ref["lang"], fa, "lang")
    assert_img(got["final_T"], ref["final_T"], fa, "final_T")
    np.testing.assert_array_equal(_last_contributor_ids(got, W, H), _last_contributor_ids(ref, W, H))
    assert float(np.abs(ref["lang"]).max()) > 0.1


def test_cfg3_culled_gpu_equals_full_reference_lists(gpu, oracle_lib):
    case = _case(3)
    W, H = case["cam"]["W"], case["cam"]["H"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    pb = oracle_problem(case)
    tiles = np.sort(np.random.default_rng(3).choice(gx * gy, size=48, replace=False)).astype(np.int32)
    ref = oracle_lib.forward(pb, nthreads=_threads(), tiles=tiles, cull=False)
    ys, xs = _tile_pixels(tiles, gx, W, H)
    # backward restricted to 32 of the tiles (upstream gradient zero elsewhere)
    btiles = tiles[:32]
    bys, bxs = _tile_pixels(btiles, gx, W, H)
    rng = np.random.default_rng(1)
    dcol = np.zeros((3, H, W), np.float32)
    dlang = np.zeros((pb.D, H, W), np.float32)
    dcol[:, bys, bxs] = rng.standard_normal((3, bys.size)).astype(np.float32)
    dlang[:, bys, bxs] = rng.standard_normal((pb.D, bys.size)).astype(np.float32)
    gf = run_gpu_forward(case, gpu)
    assert gf["num_rendered"] < ref["num_rendered"]
    np.testing.assert_array_equal(gf["radii"], ref["radii"])
    fa = fwd_atol(case)
    assert_img(gf["color"][:, ys, xs], ref["color"][:, ys, xs], fa, "color")
    assert_img(gf["lang"][:, ys, xs], ref["lang"][:, ys, xs], fa, "lang")
    assert_img(gf["final_T"][ys, xs], ref["final_T"][ys, xs], fa, "final_T")
    lc_got, lc_ref = _last_contributor_ids(gf, W, H), _last_contributor_ids(ref, W, H)
    np.testing.assert_array_equal(lc_got[ys, xs], lc_ref[ys, xs])
    del gf
    got = run_gpu_fwd_bwd(case, gpu, dcol, dlang)
    assert_img(got["color"][:, ys, xs], ref["color"][:, ys, xs], fa, "color")
    rb = oracle_lib.backward(pb, ref, dcol, dlang, tiles=btiles, nthreads=_threads())
    assert_grad_close("means2D", got["grad_means2D"], rb["dmean2D"])
    assert_grad_close("opacities", got["grad_opacities"], rb["dopacity"][:, None])
    assert_grad_close("means3D", got["grad_means3D"], rb["dmeans3D"])
    assert_grad_close("shs", got["grad_shs"], rb["dsh"])
    assert_grad_close("scales", got["grad_scales"], rb["dscales"])
    assert_grad_close("rotations", got["grad_rotations"], rb["drot"])
    assert_grad_close("language_feature_precomp", got["grad_language_feature_precomp"], rb["dlang"])


def test_needles_culled_gpu_equals_full_reference_lists(gpu, oracle_lib):
    """Needle splats (2D condition numbers 1e5-1e7, 30-60 degrees):
    the GPU's culled lists equal the oracle's culled lists bit for bit, those
    keep every (Gaussian, tile) with a contributing pixel, and the GPU's image
    equals the oracle rendering the reference's UNCULLED lists on every tile a
    needle contributes to (sampled)."""
    from harness import add_needles, needle_contributing_tiles
    W = H = 3072
    case = add_needles(make_case(N=60, W=W, H=H, seed=31, sh_degree=None, lang_dim=3), frac=1.0, seed=1,
                       sigma_px=(400.0, 1500.0))
    gx = (W + 15) // 16
    pb = oracle_problem(case)
    culled = oracle_lib.forward(pb, nthreads=_threads(), tiles=np.zeros(0, np.int32), cull=True)
    contrib = needle_contributing_tiles(culled, W, H)
    alltiles = sorted(set().union(*contrib.values()))
    tiles = np.sort(np.random.default_rng(4).choice(alltiles, size=min(96, len(alltiles)), replace=False)).astype(np.int32)
    ref = oracle_lib.forward(pb, nthreads=_threads(), tiles=tiles, cull=False)
    got = run_gpu_forward(case, gpu)
    np.testing.assert_array_equal(got["point_list"], culled["point_list"].astype(np.int32))
    np.testing.assert_array_equal(got["ranges"], culled["ranges"].astype(np.int32))
    ys, xs = _tile_pixels(tiles, gx, W, H)
    fa = fwd_atol(case)
    assert_img(got["color"][:, ys, xs], ref["color"][:, ys, xs], fa, "color")
    assert_img(got["lang"][:, ys, xs], ref["lang"][:, ys, xs], fa, "lang")
    assert_img(got["final_T"][ys, xs], ref["final_T"][ys, xs], fa, "final_T")
    assert float(ref["color"][:, ys, xs].max()) > 0.05
