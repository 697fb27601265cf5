"""Failure detection: C-ABI status codes surface as RuntimeError with
lsr_strerror's text, and settings.debug turns on the NaN/Inf guard (every input
and output array scanned; LSR_ENONFINITE names the array on stderr).  Reference
hooks: pipe.debug (gaussian_renderer/__init__.py:49), --detect_anomaly
(train.py:362)."""
import os

import pytest
import torch

from harness import gpu_inputs, make_case, settings_for
from langsplatv2_amd import _lib


def test_status_codes_have_text():
    lib = _lib.load()
    assert b"non-finite" in lib.lsr_strerror(_lib.LSR_ENONFINITE).lower()
    assert b"binning lists" in lib.lsr_strerror(_lib.LSR_ELISTS).lower()
    assert lib.lsr_abi_version() == 12


def test_options_roundtrip():
    """lsr_set_option / lsr_get_option (host-only: no GPU needed).  One binning
    mode is built (sorted tiles; the round-4 ordered mode is rejected)."""
    import ctypes
    lib = _lib.load()
    prev = _lib.set_bin_mode("sorted_tiles")
    v = ctypes.c_int64(-1)
    assert lib.lsr_get_option(_lib.LSR_OPT_BIN_MODE, ctypes.byref(v)) == 0 and v.value == 1
    assert _lib.set_bin_mode(prev) == "sorted_tiles"
    assert lib.lsr_set_option(_lib.LSR_OPT_BIN_MODE, 2) == _lib.LSR_EINVAL      # LSR_BIN_ORDERED: removed
    assert lib.lsr_set_option(_lib.LSR_OPT_BIN_MODE, 3) == _lib.LSR_EINVAL
    assert lib.lsr_set_option(12345, 0) == _lib.LSR_EINVAL
    with pytest.raises(ValueError):
        _lib.set_bin_mode("ordered")
    old = _lib.set_lists_max_mb(100)
    assert old == 2048 and _lib.set_lists_max_mb(old) == 100
    assert lib.lsr_set_option(_lib.LSR_OPT_LISTS_MAX_MB, -1) == _lib.LSR_EINVAL


def _render(case, dev, debug, poison=None):
    from diff_gaussian_rasterization import GaussianRasterizer
    rs = settings_for(case, dev)._replace(debug=debug)
    t = gpu_inputs(case, dev, requires_grad=True)
    if poison:
        with torch.no_grad():
            t[poison].view(-1)[7] = float("nan")
    r = GaussianRasterizer(rs)
    return t, r(means3D=t["means3D"], means2D=t["means2D"], opacities=t["opacities"], shs=t["shs"],
                 language_feature_precomp=t["language_feature_precomp"], scales=t["scales"], rotations=t["rotations"])


@pytest.mark.gpu
def test_debug_guard_catches_nan_inputs_and_grads(gpu, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)   # snapshot_fw.dump / snapshot_bw.dump land here
    case = make_case(N=2000, W=96, H=80, sh_degree=3, lang_dim=16, seed=0)
    # clean inputs: debug mode runs the guard and passes
    t, (color, lang, radii) = _render(case, gpu, True)
    torch.autograd.backward([color, lang], [torch.ones_like(color), torch.ones_like(lang)])
    assert bool(torch.isfinite(t["means3D"].grad).all())
    # a NaN in an input: the forward refuses, naming the failure, and dumps the snapshot
    for k in ("means3D", "shs", "language_feature_precomp"):
        with pytest.raises(RuntimeError, match="non-finite"):
            _render(case, gpu, True, poison=k)
    assert os.path.exists(tmp_path / "snapshot_fw.dump")
    # a NaN in the upstream gradient: the backward refuses
    t, (color, lang, radii) = _render(case, gpu, True)
    bad = torch.ones_like(color)
    bad[0, 3, 5] = float("inf")
    with pytest.raises(RuntimeError, match="non-finite"):
        torch.autograd.backward([color, lang], [bad, torch.ones_like(lang)])
    # without debug nothing is scanned (the product path pays nothing)
    _render(case, gpu, False, poison="means3D")


@pytest.mark.gpu
def test_debug_list_check_catches_bad_ids(gpu, tmp_path, monkeypatch):
    """with settings.debug the binning lists are checked
    before a render gathers through them, so a corrupt list (an id >= P, as a
    faulty sort would produce) returns LSR_ELISTS instead of faulting the GPU.
    Here the forward's saved point_list is corrupted before the backward."""
    from langsplatv2_amd import layout
    monkeypatch.chdir(tmp_path)
    case = make_case(N=2000, W=96, H=80, sh_degree=3, lang_dim=16, seed=0)
    t, (color, lang, radii) = _render(case, gpu, True)
    node = color.grad_fn                       # the autograd ctx of the rasterizer call
    binning = node.saved_tensors[-3]           # (..., radii, geom, binning, image, lists)
    pl_off = layout.bin_layout(int(node.num_rendered))["point_list"]
    # through .data: the saved tensor's version counter stays, as a kernel's stray write would leave it
    binning.data[pl_off:pl_off + 4].view(torch.int32)[0] = 10 ** 8      # id far past P
    with pytest.raises(RuntimeError, match="binning lists"):
        torch.autograd.backward([color, lang], [torch.ones_like(color), torch.ones_like(lang)])
