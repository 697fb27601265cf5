"""The ordered binning mode (csrc/order.hip: Gaussians radix-sorted by depth,
tile lists placed in that order, no per-tile sort) against the oracle — the
whole binning and the images bit-exact — and against the sorted-tiles mode at
cfg3's full size (identical point lists).  The oracle's lists are the
reference's order: (tile, depth bits, Gaussian id) ascending
(oracle/lsr_oracle.c lso_forward, cuda_rasterizer/rasterizer_impl.cu
duplicateWithKeys + SortPairs)."""
import numpy as np
import pytest
import torch

from harness import make_case, run_gpu_forward
from test_gpu_parity import CASES, _fwd_compare

pytestmark = pytest.mark.gpu


@pytest.fixture
def bin_mode():
    from langsplatv2_amd import _lib
    prev = []

    def set_mode(m):
        p = _lib.set_bin_mode(m)
        if not prev:
            prev.append(p)
    yield set_mode
    if prev:
        _lib.set_bin_mode(prev[0])


@pytest.mark.parametrize("name", list(CASES))
def test_ordered_forward_bit_exact(name, gpu, oracle_lib, bin_mode):
    bin_mode("ordered")
    _fwd_compare(make_case(**CASES[name]), gpu, oracle_lib)


def test_ordered_depth_ties_keep_id_order(gpu, oracle_lib, bin_mode):
    """Many Gaussians at the same depth (one plane facing the camera): equal
    depth bits are ordered by Gaussian id, as the reference's stable sort."""
    bin_mode("ordered")
    case = make_case(N=6000, W=160, H=120, sh_degree=None, seed=21)
    m = case["g"]["means3D"]
    m[::2, 2] = 4.0            # every other Gaussian on the plane z = 4
    m[1::6, 2] = 7.5           # and a second plane
    ref, got = _fwd_compare(case, gpu, oracle_lib)
    d = ref["depth"][ref["radii"] > 0]
    assert len(d) - len(np.unique(d)) > 1000   # the case really has ties


def test_ordered_big_tiles_and_empty(gpu, oracle_lib, bin_mode):
    """> 4096 instances per tile (many steps per tile run), and the empty /
    all-culled frames."""
    bin_mode("ordered")
    _fwd_compare(make_case(N=26000, W=48, H=32, sh_degree=None, seed=12), gpu, oracle_lib)
    case = make_case(N=300, W=64, H=48, sh_degree=None, seed=11)
    case["g"]["means3D"][:, 2] = -1.0
    ref, got = _fwd_compare(case, gpu, oracle_lib)
    assert got["num_rendered"] == 0


def test_ordered_backward_vs_sorted_tiles(gpu, bin_mode):
    """Same lists => the same forward (bit-identical) and the same backward
    computation (equal up to the order of the gradient atomics: GRAD_RTOL)."""
    from harness import assert_grad_close, run_gpu_fwd_bwd
    case = make_case(**CASES["sh3_lang16_ragged"])
    rng = np.random.default_rng(2)
    H, W = case["cam"]["H"], case["cam"]["W"]
    dcol = rng.standard_normal((3, H, W)).astype(np.float32)
    dlang = rng.standard_normal((16, H, W)).astype(np.float32)
    bin_mode("sorted_tiles")
    a = run_gpu_fwd_bwd(case, gpu, dcol, dlang)
    bin_mode("ordered")
    b = run_gpu_fwd_bwd(case, gpu, dcol, dlang)
    for k in a:
        if k in ("color", "lang", "radii"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        elif k.startswith("grad_"):
            assert_grad_close(k, b[k], a[k])


@pytest.mark.slow
def test_ordered_equals_sorted_tiles_cfg3(gpu, bin_mode):
    """cfg3's full size (1M Gaussians, 1080p, 4.7M instances): the two modes'
    ranges and point lists are identical, and the lists are in strict
    (depth, id) order per tile."""
    from langsplatv2_amd.scenes import CONFIGS
    c = CONFIGS[3]
    case = make_case(N=c["N"], W=c["W"], H=c["H"], sh_degree=c["sh_degree"], lang_dim=c["lang_dim"], seed=0)
    bin_mode("sorted_tiles")
    a = run_gpu_forward(case, gpu)
    bin_mode("ordered")
    b = run_gpu_forward(case, gpu)
    assert a["num_rendered"] == b["num_rendered"] > 1_000_000
    np.testing.assert_array_equal(a["ranges"], b["ranges"])
    np.testing.assert_array_equal(a["point_list"], b["point_list"])
    np.testing.assert_array_equal(a["color"], b["color"])
    pl = b["point_list"].astype(np.int64)
    depth = b["depth"]
    key = (depth.view(np.uint32).astype(np.int64)[pl] << 32) | pl
    tile_of = np.repeat(np.arange(len(b["ranges"])), b["ranges"][:, 1] - b["ranges"][:, 0])
    same = tile_of[1:] == tile_of[:-1]
    assert np.all(key[1:][same] > key[:-1][same])


def test_bin_mode_option_validation(gpu):
    from langsplatv2_amd import _lib
    with pytest.raises(ValueError):
        _lib.set_bin_mode("bogus")
    lib = _lib.load()
    assert lib.lsr_set_option(1, 7) != 0
    assert lib.lsr_set_option(99, 0) != 0
