"""Parity at BASELINE.json's full sizes: the oracle is too slow to
render a whole 1080p / 4K frame in a test, so these compare what is exact at
any size.

cfg3 (1M Gaussians, 1920x1080, SH3 + 16 language channels):
  * forward: the WHOLE binning (ranges of all 8160 tiles, the full 8.2M-entry
    depth-ordered point list) and the per-Gaussian records bit-exactly, and
    the images / final_T / n_contrib bit-exactly on 48 seeded tiles the oracle
    renders;
  * backward: with dL/dout zero outside those tiles, the GPU's full backward
    equals the oracle's tile-restricted backward (GRAD_RTOL).
cfg2 (100k Gaussians, 800x800, RGB colours + 3 language channels,
  forward-only): the WHOLE frame bit-exactly against the oracle (every tile
  rendered on the host's cores): radii, the full binning, colour, language,
  final_T, n_contrib.
cfg5 (5M Gaussians, 3840x2160, SH3 + 32 language channels, 120M instances):
  the WHOLE binning (ranges + point list) and per-Gaussian records
  bit-exactly, images / final_T / n_contrib bit-exactly on 32 seeded tiles;
  plus size-independent properties of the binning (every instance once, lists
  in strict (depth, id) order per tile, ranges partition the list) and of the
  images (finite, final_T in [0, 1], colour >= 0 with a black background).
"""
import os

import numpy as np
import pytest
import torch

from harness import assert_grad_close, make_case, oracle_problem, run_gpu_fwd_bwd, run_gpu_forward
from langsplatv2_amd.scenes import CONFIGS

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _case(cfg_id):
    c = CONFIGS[cfg_id]
    return make_case(N=c["N"], W=c["W"], H=c["H"], sh_degree=c["sh_degree"], lang_dim=c["lang_dim"], seed=0)


def _tile_pixels(tiles, gx, W, H):
    ys, xs = [], []
    for t in tiles:
        tx, ty = t % gx, t // gx
        y0, x0 = ty * 16, tx * 16
        yy, xx = np.mgrid[y0:min(y0 + 16, H), x0:min(x0 + 16, W)]
        ys.append(yy.ravel())
        xs.append(xx.ravel())
    return np.concatenate(ys), np.concatenate(xs)


def _sample_tiles(gx, gy, n=48, seed=3):
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(gx * gy, size=n, replace=False)).astype(np.int32)


def test_cfg3_forward_full_binning_and_sampled_tiles(gpu, oracle_lib):
    case = _case(3)
    W, H = case["cam"]["W"], case["cam"]["H"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = _sample_tiles(gx, gy)
    pb = oracle_problem(case)
    ref = oracle_lib.forward(pb, nthreads=8, tiles=tiles)
    got = run_gpu_forward(case, gpu)
    assert got["num_rendered"] == ref["num_rendered"]
    np.testing.assert_array_equal(got["radii"], ref["radii"])
    np.testing.assert_array_equal(got["tiles_touched"], ref["tiles_touched"].astype(np.int32))
    vis = ref["radii"] > 0
    np.testing.assert_array_equal(got["xy"][vis], ref["xy"][vis])
    np.testing.assert_array_equal(got["conic_opacity"][vis], ref["conic_opacity"][vis])
    np.testing.assert_array_equal(got["rgb"][vis], ref["rgb"][vis])
    np.testing.assert_array_equal(got["ranges"], ref["ranges"].astype(np.int32))
    np.testing.assert_array_equal(got["point_list"], ref["point_list"].astype(np.int32))
    ys, xs = _tile_pixels(tiles, gx, W, H)
    np.testing.assert_array_equal(got["n_contrib"][ys, xs], ref["n_contrib"][ys, xs].astype(np.int32))
    np.testing.assert_array_equal(got["final_T"][ys, xs], ref["final_T"][ys, xs])
    np.testing.assert_array_equal(got["color"][:, ys, xs], ref["color"][:, ys, xs])
    np.testing.assert_array_equal(got["lang"][:, ys, xs], ref["lang"][:, ys, xs])


def _threads():
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else min(16, os.cpu_count() or 1)


def _compare_forward(got, ref, sh, tiles=None, gx=None, W=None, H=None):
    assert got["num_rendered"] == ref["num_rendered"]
    np.testing.assert_array_equal(got["radii"], ref["radii"])
    np.testing.assert_array_equal(got["tiles_touched"], ref["tiles_touched"].astype(np.int32))
    vis = ref["radii"] > 0
    np.testing.assert_array_equal(got["xy"][vis], ref["xy"][vis])
    np.testing.assert_array_equal(got["conic_opacity"][vis], ref["conic_opacity"][vis])
    if sh:   # with colors_precomp the renderer reads the caller's colours, no rgb record is written
        np.testing.assert_array_equal(got["rgb"][vis], ref["rgb"][vis])
    np.testing.assert_array_equal(got["ranges"], ref["ranges"].astype(np.int32))
    np.testing.assert_array_equal(got["point_list"], ref["point_list"].astype(np.int32))
    if tiles is None:
        np.testing.assert_array_equal(got["n_contrib"], ref["n_contrib"].astype(np.int32))
        np.testing.assert_array_equal(got["final_T"], ref["final_T"])
        np.testing.assert_array_equal(got["color"], ref["color"])
        np.testing.assert_array_equal(got["lang"], ref["lang"])
    else:
        ys, xs = _tile_pixels(tiles, gx, W, H)
        np.testing.assert_array_equal(got["n_contrib"][ys, xs], ref["n_contrib"][ys, xs].astype(np.int32))
        np.testing.assert_array_equal(got["final_T"][ys, xs], ref["final_T"][ys, xs])
        np.testing.assert_array_equal(got["color"][:, ys, xs], ref["color"][:, ys, xs])
        np.testing.assert_array_equal(got["lang"][:, ys, xs], ref["lang"][:, ys, xs])


def test_cfg2_whole_frame_bit_exact(gpu, oracle_lib):
    case = _case(2)
    assert case["g"]["means3D"].shape[0] == 100_000 and case["cam"]["W"] == 800 and case["cam"]["H"] == 800
    assert "colors_precomp" in case["g"] and case["g"]["language_feature_precomp"].shape[1] == 3
    ref = oracle_lib.forward(oracle_problem(case), nthreads=_threads())
    got = run_gpu_forward(case, gpu)
    assert got["lang"].shape == (3, 800, 800)
    _compare_forward(got, ref, sh=False)
    # the frame is not trivially empty
    assert ref["num_rendered"] > 100_000 and float(np.abs(ref["lang"]).max()) > 0.1


def test_cfg5_full_binning_and_sampled_tiles(gpu, oracle_lib):
    case = _case(5)
    W, H = case["cam"]["W"], case["cam"]["H"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = _sample_tiles(gx, gy, n=32, seed=7)
    ref = oracle_lib.forward(oracle_problem(case), nthreads=_threads(), tiles=tiles)
    got = run_gpu_forward(case, gpu)
    assert got["lang"].shape[0] == 32
    _compare_forward(got, ref, True, tiles, gx, W, H)


def test_cfg3_backward_sampled_tiles(gpu, oracle_lib):
    case = _case(3)
    W, H = case["cam"]["W"], case["cam"]["H"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = _sample_tiles(gx, gy, n=32, seed=5)
    pb = oracle_problem(case)
    ref = oracle_lib.forward(pb, nthreads=8, tiles=tiles)
    rng = np.random.default_rng(1)
    ys, xs = _tile_pixels(tiles, gx, W, H)
    dcol = np.zeros((3, H, W), np.float32)
    dlang = np.zeros((pb.D, H, W), np.float32)
    dcol[:, ys, xs] = rng.standard_normal((3, ys.size)).astype(np.float32)
    dlang[:, ys, xs] = rng.standard_normal((pb.D, ys.size)).astype(np.float32)
    rb = oracle_lib.backward(pb, ref, dcol, dlang, tiles=tiles)
    got = run_gpu_fwd_bwd(case, gpu, dcol, dlang)
    assert_grad_close("means2D", got["grad_means2D"], rb["dmean2D"])
    assert_grad_close("opacities", got["grad_opacities"], rb["dopacity"][:, None])
    assert_grad_close("means3D", got["grad_means3D"], rb["dmeans3D"])
    assert_grad_close("shs", got["grad_shs"], rb["dsh"])
    assert_grad_close("scales", got["grad_scales"], rb["dscales"])
    assert_grad_close("rotations", got["grad_rotations"], rb["drot"])
    assert_grad_close("language_feature_precomp", got["grad_language_feature_precomp"], rb["dlang"])


def test_cfg5_binning_and_image_properties(gpu):
    from langsplatv2_amd import layout, rasterizer
    from harness import gpu_inputs, settings_for
    case = _case(5)
    rs = settings_for(case, gpu)
    t = gpu_inputs(case, gpu, requires_grad=False)
    e = torch.empty(0, device=gpu)
    color, lang, radii, M, bufs, _, _, _ = rasterizer._run_forward(
        t["means3D"], t["shs"], e, t["language_feature_precomp"], e, e, t["opacities"], t["scales"],
        t["rotations"], e, rs)
    N, W, H = t["means3D"].shape[0], rs.image_width, rs.image_height
    dec = layout.decode(bufs, N, W, H, M)
    tt = dec["tiles_touched"].to(torch.int64)
    assert 0 < M <= int(tt[radii > 0].sum())
    ts = dec["tile_start"].to(torch.int64)
    assert int(ts[0]) == 0 and int(ts[-1]) == M and bool((ts[1:] >= ts[:-1]).all())
    pl = dec["point_list"].to(torch.int64)
    # every visible Gaussian appears at most tiles_touched times (the tile
    # cull keeps the rect tiles its cut ellipse meets), invisible ones never
    counts = torch.bincount(pl, minlength=N)
    assert bool((counts <= torch.where(radii > 0, tt, torch.zeros_like(tt))).all())
    # strict (depth bits, id) order inside each tile
    key = (dec["depth"].contiguous().view(torch.int32).to(torch.int64)[pl] << 32) | pl
    tile_of = torch.repeat_interleave(torch.arange(ts.numel() - 1, device=gpu), ts[1:] - ts[:-1])
    same = tile_of[1:] == tile_of[:-1]
    assert bool((key[1:][same] > key[:-1][same]).all())
    # images
    assert bool(torch.isfinite(color).all()) and bool(torch.isfinite(lang).all())
    fT = dec["final_T"]
    assert bool(((fT >= 0) & (fT <= 1)).all()) and bool((color >= 0).all())


# --- the paths the bench and tools time at full size ---

def test_quick_1mpix_full_binning_and_sampled_tiles(gpu, oracle_lib):
    """bench.py quick_1mpix's render: 1M Gaussians, 1280x800, 3 levels x top-4
    codes -> 192 channels (k_render_fwd_quick_v<6>, the VGPR-index-mode kernel,
    reference eval_lerf.py:210-220).  The whole binning and 32 seeded tiles'
    colour, 192-channel weight map, final_T and n_contrib bit-exact."""
    case = make_case(N=1_000_000, W=1280, H=800, sh_degree=3, quick_k=4, seed=0)
    W, H = 1280, 800
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = _sample_tiles(gx, gy, n=32, seed=9)
    ref = oracle_lib.forward(oracle_problem(case), nthreads=_threads(), tiles=tiles)
    got = run_gpu_forward(case, gpu)
    assert got["lang"].shape == (192, H, W)
    _compare_forward(got, ref, True, tiles, gx, W, H)
    ys, xs = _tile_pixels(tiles, gx, W, H)
    assert float(np.abs(ref["lang"][:, ys, xs]).max()) > 0.1     # the sampled tiles carry weights


def _lang_only_grad(case, gpu, dcol, dlang):
    """Feature-mode autograd (scene/gaussian_model.py:238-243): geometry frozen,
    means2D without grad, only the language input requires grad -> the
    library's language-only backward k_render_bwd_mf<NL, true>."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from harness import settings_for
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    lang = t["language_feature_precomp"].clone().requires_grad_(True)
    r = GaussianRasterizer(settings_for(case, gpu))
    color, lo, _ = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                     shs=t["shs"], scales=t["scales"], rotations=t["rotations"], language_feature_precomp=lang)
    torch.autograd.backward([color, lo], [torch.from_numpy(dcol).to(gpu), torch.from_numpy(dlang).to(gpu)])
    return lo.detach().cpu().numpy(), lang.grad.cpu().numpy()


def test_d64_feature_step_shape_sampled_tiles(gpu, oracle_lib):
    """tools/bench_train_step.py's rasterizer shape (BASELINE cfg4's step):
    1M Gaussians, 1920x1080, SH3 + 64 language channels.  The ML-form forward
    k_render_fwd<64, ., true> bit-exact on 48 seeded tiles (and the whole
    binning), and the language-only backward k_render_bwd_mf<64, true> with
    dL/dout zero outside 32 of them equal to the oracle's tile-restricted
    backward (GRAD_RTOL)."""
    case = make_case(N=1_000_000, W=1920, H=1080, sh_degree=3, lang_dim=64, seed=0)
    W, H = 1920, 1080
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = _sample_tiles(gx, gy, n=48, seed=11)
    pb = oracle_problem(case)
    ref = oracle_lib.forward(pb, nthreads=_threads(), tiles=tiles)
    got = run_gpu_forward(case, gpu)
    assert got["lang"].shape == (64, H, W)
    _compare_forward(got, ref, True, tiles, gx, W, H)
    del got
    btiles = tiles[:32]
    ys, xs = _tile_pixels(btiles, gx, W, H)
    rng = np.random.default_rng(2)
    dcol = np.zeros((3, H, W), np.float32)
    dlang = np.zeros((64, H, W), np.float32)
    dcol[:, ys, xs] = rng.standard_normal((3, ys.size)).astype(np.float32)
    dlang[:, ys, xs] = rng.standard_normal((64, ys.size)).astype(np.float32)
    rb = oracle_lib.backward(pb, ref, dcol, dlang, tiles=btiles, nthreads=_threads())
    lo, g = _lang_only_grad(case, gpu, dcol, dlang)
    np.testing.assert_array_equal(lo[:, ys, xs], ref["lang"][:, ys, xs])
    assert float(np.abs(rb["dlang"]).max()) > 0.0
    assert_grad_close("language_feature_precomp", g, rb["dlang"])
