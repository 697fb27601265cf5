"""Host rule for the forward-prepared backward accumulators (rasterizer._grad_request):
which LSR_GWS_* bits a forward asks for, from autograd's needs_input_grad and the
grad mode at the call (no GPU needed)."""
from types import SimpleNamespace

import torch

from langsplatv2_amd import _lib, rasterizer

E = torch.empty(0)
X = torch.zeros(4, 3)


def _rs(quick=False, feature=True):
    return SimpleNamespace(quick_render=quick, include_feature=feature)


def _req(need, grad_on=True, lang=X, quick=False, feature=True, sh=X, scales=X, rotations=X):
    rasterizer._CALL.grad_enabled = grad_on
    try:
        return rasterizer._grad_request(need, sh, E, lang, scales, rotations, E, _rs(quick, feature))
    finally:
        rasterizer._CALL.grad_enabled = False


def _need(*idx):
    n = [False] * 12
    for i in idx:
        n[i] = True
    return tuple(n)


def test_geometry_and_language():
    assert _req(_need(0, 1, 2, 4, 7, 8, 9)) == _lib.LSR_GWS_GEOM | _lib.LSR_GWS_LANG
    assert _req(_need(0)) == _lib.LSR_GWS_GEOM
    assert _req(_need(1)) == _lib.LSR_GWS_GEOM          # means2D alone is a geometry output
    assert _req(_need(4)) == _lib.LSR_GWS_LANG          # feature-mode training


def test_nothing_prepared():
    assert _req(_need()) == 0
    assert _req(_need(0, 4), grad_on=False) == 0         # torch.no_grad() at the call
    assert _req(_need(0, 4), quick=True) == 0            # quick path: its backward clears its own
    assert _req(_need(4), feature=False) == 0            # no dense language channels rendered
    assert _req(_need(4), lang=E) == 0
    assert _req(_need(3)) == 0                           # colors_precomp absent (empty)
    assert rasterizer._CALL.grad_enabled is False
