"""LSR_OPT_SPLIT_PREPROCESS: the forward's SH colour pass on a second stream,
concurrent with the binning (preprocess.hip k_preprocess<., ., 1> +
k_preprocess_colour).  The same expressions in both layouts: every forward
output and workspace value must equal the fused pass's bit for bit, and the
gradients (summed by float atomics) to rounding."""
import numpy as np
import pytest

from harness import make_case, run_gpu_forward, run_gpu_fwd_bwd


def test_option_roundtrip_on_cpu():
    from langsplatv2_amd import _lib
    lib = _lib.load()
    assert _lib.set_split_preprocess(False) is True      # default on
    assert _lib.set_split_preprocess(True) is False
    assert lib.lsr_set_option(_lib.LSR_OPT_SPLIT_PREPROCESS, 2) == _lib.LSR_EINVAL


def _both(fn):
    from langsplatv2_amd import _lib
    try:
        _lib.set_split_preprocess(False)
        a = fn()
        _lib.set_split_preprocess(True)
        b = fn()
    finally:
        _lib.set_split_preprocess(True)
    return a, b


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(sh_degree=3, lang_dim=16), dict(sh_degree=1), dict(sh_degree=3, quick_k=4)])
def test_split_equals_fused_forward(gpu, kw):
    case = make_case(N=(1 << 19) + 5000, W=512, H=384, seed=5, **kw)   # P >= 2^19: the split applies
    a, b = _both(lambda: run_gpu_forward(case, gpu))
    for k in ("color", "lang", "radii", "rgb", "clamped", "depth", "xy", "conic_opacity", "n_contrib", "final_T",
              "point_list"):
        np.testing.assert_array_equal(np.asarray(b[k]), np.asarray(a[k]), err_msg=k)


@pytest.mark.gpu
def test_split_equals_fused_backward(gpu):
    case = make_case(N=(1 << 19) + 5000, W=512, H=384, seed=6, sh_degree=3, lang_dim=16)
    rng = np.random.default_rng(2)
    dc = rng.standard_normal((3, 384, 512)).astype(np.float32)
    dl = rng.standard_normal((16, 384, 512)).astype(np.float32)
    a, b = _both(lambda: run_gpu_fwd_bwd(case, gpu, dc, dl))
    np.testing.assert_array_equal(b["color"], a["color"])
    for k in a:
        if k.startswith("grad_"):
            # two backwards of one forward differ only in float-atomic summation order
            np.testing.assert_allclose(b[k], a[k], rtol=1e-4, atol=1e-5 * max(1.0, float(np.abs(a[k]).max())),
                                       err_msg=k)
