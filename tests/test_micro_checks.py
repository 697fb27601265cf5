"""Hardware facts the product's bit-exactness rests on, checked on the GPU
(fold tools/micro/mfma_order.hip and dpp_xor.hip into -m gpu).
tests/micro/micro_checks.hip, built by __graft_entry__.build().

* The wave sort's register-path lane exchange (lsr_device.h xor_lane_u32,
  used by k_tile_sort_wave) equals __shfl_xor at every distance.
* v_mfma_f32_16x16x4_f32 is bitwise a fmaf chain over k = 0..3 in order --
  on wide-exponent normals AND with zeros, signed zeros, subnormals,
  infinities, near-overflow values and NaN mixed in -- which is what makes the
  ML-form forward (language channels accumulated on MFMA) bit-identical to the
  oracle's sequential per-pixel blend."""
import ctypes
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "micro", "libmicro_checks.so")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def micro(gpu):
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB)
    lib.micro_dpp_xor.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    lib.micro_mfma_order.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
    return lib


@pytest.mark.parametrize("seed", [0, 1])
def test_lane_exchange_matches_shfl_xor(micro, seed):
    mm = (ctypes.c_int * 6)()
    assert micro.micro_dpp_xor(seed, mm) == 0
    assert list(mm) == [0] * 6, dict(zip((1, 2, 4, 8, 16, 32), mm))


@pytest.mark.parametrize("specials", [0, 1])
def test_mfma_f32_is_an_in_order_fmaf_chain(micro, specials):
    c = (ctypes.c_longlong * 4)()
    assert micro.micro_mfma_order(2048, 7 + specials, specials, c) == 0
    tot, fwd, rev, spec = list(c)
    assert tot == 2048 * 256
    if specials:
        assert spec > tot // 4          # the special operands are really exercised
    assert fwd == tot, f"MFMA != fmaf chain k=0..3 on {tot - fwd} of {tot} (reverse order matches {rev})"


def test_fast_exp_inside_the_backward_alpha_band(micro):
    """The render backward evaluates G with the hardware v_exp_f32 (power * log2 e)
    and re-takes the alpha >= 1/255 decision with expf_det (the forward's, the
    oracle's) for every lane whose alpha is within 2e-8 of 1/255 (render.hip,
    k_render_bwd_mf phase 1).  That is exact only if the two exponentials differ
    by less than 2e-8 * 255 = 5.1e-6 relative wherever alpha can reach 1/255:
    powers >= ln(1/255) - ln(opacity), i.e. >= -5.55 for opacities <= 1
    (sigmoid-activated); -8 leaves room for opacities up to e^2.5.  Checked over
    EVERY float power in [-8, 0] (1.09e9 values) against a bound of half the
    band.  (Over [-87, 0] the product power * log2 e rounds to 2^-24 of 125 and
    the difference reaches 3.9e-6: still inside, with less margin.)"""
    micro.micro_exp_band.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_double)]
    out = (ctypes.c_double * 2)()
    assert micro.micro_exp_band(-8.0, out) == 0
    band_rel = 2e-8 * 255.0
    print(f"max relative |exp_hw - expf_det| / expf_det = {out[0]:.3e} over {int(out[1])} powers; "
          f"backward band {band_rel:.2e} relative")
    assert out[1] > 1.0e9   # every float in [-8, 0]
    assert 0.0 < out[0] < 0.5 * band_rel
    out87 = (ctypes.c_double * 2)()
    assert micro.micro_exp_band(-87.0, out87) == 0
    assert out87[0] < band_rel
