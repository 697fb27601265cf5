"""The backward's accumulators prepared by the forward (lsr_fwd_out.grad_ws).

With a gradient pending, the forward allocates the gradient rows (and the
(N, D) dL/dlang accumulator) and zeroes them inside the render kernel; the
backward adds into them instead of clearing its own with two memsets
(lsr_api.hip grad_ws_layout, render.hip zero_backward_accumulators).  A
second backward over the same graph (retain_graph) finds the workspace taken
and clears its own, so the two must agree: they sum the same per-pair terms,
in an arrival order the atomics do not fix (harness.GRAD_RTOL).
"""
import numpy as np
import pytest
import torch

from harness import assert_grad_close, gpu_inputs, make_case, settings_for

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _twice(case, lang_only=False):
    """Forward once, backward twice (first with the forward's workspace, then without)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    rs = settings_for(case, DEV)
    t = gpu_inputs(case, DEV, requires_grad=True)
    if lang_only:   # feature-mode training: only the language input needs a gradient
        for k in list(t):
            if k != "language_feature_precomp" and isinstance(t[k], torch.Tensor):
                t[k] = t[k].detach()
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations", "language_feature_precomp") if k in t}
    color, lang, _ = GaussianRasterizer(raster_settings=rs)(means3D=t["means3D"], means2D=t["means2D"],
                                                            opacities=t["opacities"], **kw)
    gen = torch.Generator(device=DEV).manual_seed(7)
    dc = torch.randn(color.shape, device=DEV, generator=gen)
    outs, grads = [color], [dc]
    if lang.numel():
        outs.append(lang)
        grads.append(torch.randn(lang.shape, device=DEV, generator=gen))
    leaves = {k: v for k, v in t.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    node = color.grad_fn   # the autograd context of the rasterizer call
    assert node.grad_ws is not None, "the forward prepared no accumulators"
    runs = []
    for i in range(2):
        assert (node.grad_ws is None) == (i == 1)
        for v in leaves.values():
            v.grad = None
        torch.autograd.backward(outs, grads, retain_graph=True)
        torch.cuda.synchronize()
        runs.append({k: v.grad.detach().cpu().numpy().copy() for k, v in leaves.items() if v.grad is not None})
    return runs


@pytest.mark.parametrize("lang_dim", [16, 32, 3, 0])
def test_workspace_backward_matches_own_clear(lang_dim):
    case = make_case(N=4000, W=160, H=128, sh_degree=3, lang_dim=lang_dim, seed=3)
    a, b = _twice(case)
    assert set(a) == set(b) and "means3D" in a
    for k in a:
        assert_grad_close(k, a[k], b[k])
        assert np.any(a[k] != 0.0), k


@pytest.mark.parametrize("lang_dim", [16, 8])
def test_workspace_language_only_backward(lang_dim):
    case = make_case(N=4000, W=160, H=128, sh_degree=3, lang_dim=lang_dim, seed=4)
    a, b = _twice(case, lang_only=True)
    assert set(a) == {"language_feature_precomp"}
    assert_grad_close("language_feature_precomp", a["language_feature_precomp"], b["language_feature_precomp"])


def test_forward_prepares_zeroed_workspace():
    from langsplatv2_amd import _lib, rasterizer
    case = make_case(N=3000, W=128, H=96, sh_degree=3, lang_dim=16, seed=5)
    rs = settings_for(case, DEV)
    t = gpu_inputs(case, DEV, requires_grad=False)
    e = torch.empty(0, device=DEV)
    args = (t["means3D"], t["shs"], e, t["language_feature_precomp"], e, e, t["opacities"], t["scales"],
            t["rotations"], e, rs)
    N, D = t["means3D"].shape[0], 16
    for req, has_lang, vp in ((_lib.LSR_GWS_GEOM | _lib.LSR_GWS_LANG, True, 16), (_lib.LSR_GWS_GEOM, False, 32),
                              (_lib.LSR_GWS_LANG, True, 0)):
        # poison the allocator's free blocks so a missing clear shows
        junk = torch.full((1 << 22,), float("nan"), device=DEV)
        del junk
        *_, ws = rasterizer._run_forward(*args, grad_request=req)
        torch.cuda.synchronize()
        assert ws is not None, req
        rows, nbytes, kind, lang = ws
        assert (kind >> 8) == vp, (req, kind)
        assert (lang is not None) == has_lang
        assert (rows is not None) == (vp > 0)
        assert nbytes == N * vp * 4, (req, nbytes)
        if rows is not None:
            assert int(torch.count_nonzero(rows[:nbytes])) == 0, req
        if lang is not None:
            # its own allocation: the gradient returned from it keeps no rows alive
            assert rows is None or lang.untyped_storage().data_ptr() != rows.untyped_storage().data_ptr()
            assert int(torch.count_nonzero(lang[:N * D * 4])) == 0, req
    *_, ws = rasterizer._run_forward(*args, grad_request=0)
    assert ws is None


def _grads_once(case, seed=7):
    from diff_gaussian_rasterization import GaussianRasterizer
    rs = settings_for(case, DEV)
    t = gpu_inputs(case, DEV, requires_grad=True)
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations", "language_feature_precomp") if k in t}
    color, lang, _ = GaussianRasterizer(raster_settings=rs)(means3D=t["means3D"], means2D=t["means2D"],
                                                            opacities=t["opacities"], **kw)
    gen = torch.Generator(device=DEV).manual_seed(seed)
    outs, grads = [color], [torch.randn(color.shape, device=DEV, generator=gen)]
    if lang.numel():
        outs.append(lang)
        grads.append(torch.randn(lang.shape, device=DEV, generator=gen))
    torch.autograd.backward(outs, grads)
    torch.cuda.synchronize()
    return {k: v.grad.detach().cpu().numpy() for k, v in t.items() if isinstance(v, torch.Tensor) and v.grad is not None}


@pytest.mark.parametrize("lang_dim", [16, 0])
def test_lists_budget_zero_falls_back_to_restaging(lang_dim):
    """LSR_OPT_LISTS_MAX_MB: with no budget the forward writes no
    per-block lists and the backward re-stages from the tile lists; the
    gradients are the same sums (GRAD_RTOL: atomics arrival order)."""
    from langsplatv2_amd import _lib
    case = make_case(N=4000, W=160, H=128, sh_degree=3, lang_dim=lang_dim, seed=6)
    a = _grads_once(case)
    prev = _lib.set_lists_max_mb(0)
    try:
        b = _grads_once(case)
    finally:
        assert _lib.set_lists_max_mb(prev) == 0
    assert set(a) == set(b) and "means3D" in a
    for k in a:
        assert_grad_close(k, a[k], b[k])
