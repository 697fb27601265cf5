"""The deterministic backward (LSR_OPT_DETERMINISTIC, include/lsr.h; render.hip
det_shift / k_det_finish): bit-reproducible gradients, compared with the oracle
at tolerances DERIVED from an error analysis, not fitted to measurements.

Two levels, both against the C restatement (oracle/lsr_oracle.c):
  render rows   the per-Gaussian render gradients (dL/dmeans2D, dL/dconic,
                dL/dopacity, dL/dcolour, dL/dlanguage) -- where every sum over
                pixels and blocks happens -- within
                  bound = lso_render_bwd_bound (running forward-error analysis of
                          both evaluations, oracle/lsr_oracle.c)
                        + the fixed-point rounding, nb 2^-(s+1) per element
                        + u (|gpu| + |oracle|)   (the two final fp32 roundings);
  chain rule    the product's preprocess backward applied to its own rows, against
                the oracle's applied to the same rows, within
                  u (64 + 16 kappa) sum_k |J e_k| |row_k| + u |oracle|
                (J: the per-Gaussian chain-rule Jacobian, linear in the rows;
                 64 bounds the fp32 operations on its longest path; kappa =
                 (|a c| + b^2) / |a c - b^2| of the 2D conic covers the one
                 cancellation in it, the determinant and 1/det^2).
Together they bound every gradient the rasterizer returns.  u = 2^-24.
The default backward (fp32 atomics) is held to the same analysis with the
any-order summation bound nblocks u sum|term| in place of the fixed-point term
(check_rows(deterministic=False))."""
import json
import os

import numpy as np
import pytest
import torch

from harness import gpu_inputs, make_case, oracle_problem, run_gpu_bwd_rows, settings_for

pytestmark = pytest.mark.gpu
U = 2.0 ** -24
LOG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "det_bounds.json")


def record(test, res):
    """Append one case's max |err| and max |err| / bound per quantity to
    gpurun_out/det_bounds.json (the numbers DESIGN.md §4 quotes)."""
    os.makedirs(os.path.dirname(LOG), exist_ok=True)
    doc = {}
    if os.path.exists(LOG):
        try:
            with open(LOG) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            doc = {}
    doc[test] = res
    with open(LOG, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)


def _upstream(H, W, D, seed=1):
    gen = torch.Generator().manual_seed(seed)
    return torch.randn((3, H, W), generator=gen).numpy(), (torch.randn((D, H, W), generator=gen).numpy() if D else None)


def _frexp_e(x):
    return np.frexp(np.asarray(x, np.float32))[1].astype(np.int64)


def _quant(radii, cls, Dm, Am, WH):
    """nb 2^-(s+1): the fixed-point rounding of one element's block partials
    (render.hip det_shift restated; x2 margin for the fp32 evaluation of the
    exponent's inputs)."""
    rr = np.maximum(radii, 1).astype(np.float32)
    q = np.float32(0.25) * rr + np.float32(2.0)
    nb = q * q
    B = {0: np.float32(64.0) * Dm, 1: np.float32(64.0) * Am, 2: np.float32(40.0) * WH * Am,
         3: np.float32(3.0) * rr * rr * Am}[cls]
    B = np.broadcast_to(np.maximum(np.float32(B), np.float32(1e-30)), rr.shape)
    s = np.clip(61 - _frexp_e(nb) - _frexp_e(B), -100, 100)
    return 2.0 * nb.astype(np.float64) * np.ldexp(1.0, -(s + 1))


def _scales(pb, ref, dcol, dlang):
    vis = ref["radii"] > 0
    Dm = np.float32(max(float(np.abs(dcol).max()), float(np.abs(dlang).max()) if dlang is not None else 0.0))
    feats = [np.abs(pb.colors if pb.colors is not None else ref["rgb"])[vis]]
    if pb.D:
        feats.append(np.abs(pb.lang)[vis])
    Fm = np.float32(max(float(f.max(initial=0.0)) for f in feats))
    bg1 = np.float32(np.abs(pb.bg).sum())
    Am = (np.float32(2.0) * np.float32(3 + pb.D) * Fm + bg1) * Dm
    return Dm, Am, np.float32(max(pb.W, pb.H))


def _check(name, got, ref, tol):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    tol = np.asarray(tol, np.float64) + U * (np.abs(got) + np.abs(ref)) + 1e-30
    err = np.abs(got - ref)
    ratio = err / tol
    k = int(np.argmax(ratio)) if ratio.size else 0
    assert bool((err <= tol).all()), (f"{name}: |err| {err.flat[k]:.3e} > analytic bound {tol.flat[k]:.3e} at {k} "
                                      f"(got {got.flat[k]:.6e}, oracle {ref.flat[k]:.6e})")
    return dict(max_abs=float(err.max(initial=0.0)), max_err_over_bound=float(ratio.max(initial=0.0)),
                median_bound=float(np.median(tol)) if tol.size else 0.0)


def check_rows(case, got, oracle_lib, dcol, dlang, nthreads=1, deterministic=True):
    """The render rows of `got` (run_gpu_bwd_rows) against the oracle within the
    derived bound; returns the per-quantity max |err| and max |err| / bound.
    deterministic=False: rows from the default backward, whose cross-block sums
    are fp32 atomics in arbitrary order -- in place of the fixed-point rounding,
    the recursive-summation bound of nb partials in any order, nb u sum_b |partial_b|
    <= nblocks u mag (mag = the element's sum of |term|, nblocks = the 8x8 blocks
    the Gaussian contributes in; both from the oracle's bound pass)."""
    pb = oracle_problem(case)
    ref = oracle_lib.forward(pb, nthreads=nthreads)
    rb = oracle_lib.backward(pb, ref, dcol, dlang, nthreads=max(nthreads, 2))
    bd = oracle_lib.backward_bound(pb, ref, dcol, dlang, nthreads=nthreads, with_mag=not deterministic)
    Dm, Am, WH = _scales(pb, ref, dcol, dlang)
    rows, radii = got["rows"], got["radii"]
    np.testing.assert_array_equal(radii, ref["radii"])
    if deterministic:
        qm, qc, qo, q0 = (_quant(radii, c, Dm, Am, WH) for c in (2, 3, 1, 0))
        ql = q0
    else:
        nbu = U * bd["nblocks"].astype(np.float64)
        mg = bd["mag"]
        qm = nbu[:, None] * mg["dmean2D"][:, :2]
        qc = nbu[:, None] * mg["dconic"]
        qo = nbu * mg["dopacity"]
        q0 = nbu[:, None] * mg["dcolor"]
        ql = nbu[:, None] * mg["dlang"] if pb.D else None
    col = (lambda q: q[:, None]) if deterministic else (lambda q: q)   # per Gaussian / per element
    res = {"mean2D": _check("mean2D", rows[:, 0:2], rb["dmean2D"][:, :2], bd["dmean2D"][:, :2] + col(qm)),
           "conic": _check("conic", rows[:, 2:5], rb["dconic"], bd["dconic"] + col(qc)),
           "opacity": _check("opacity", rows[:, 5], rb["dopacity"], bd["dopacity"] + qo),
           "colour": _check("colour", rows[:, 6:9], rb["dcolor"], bd["dcolor"] + col(q0))}
    if pb.D:
        gl = got["grad_language_feature_precomp"]
        res["language"] = _check("language", gl, rb["dlang"], bd["dlang"] + col(ql))
    return pb, ref, res


def check_chain(pb, ref, got, oracle_lib):
    """The product's preprocess backward (its returned 3D gradients) against the
    oracle's chain rule applied to the product's own rows, within the derived bound."""
    rows = got["rows"]
    rg = dict(dmean2D=np.concatenate([rows[:, 0:2], np.zeros((pb.N, 1), np.float32)], 1),
              dconic=rows[:, 2:5], dopacity=rows[:, 5], dcolor=rows[:, 6:9])
    want = oracle_lib.preprocess_backward(pb, ref, rg)
    mag = oracle_lib.preprocess_backward_abs(pb, ref, rg)
    co = ref["conic_opacity"].astype(np.float64)
    acc = np.abs(co[:, 0] * co[:, 2])
    kappa = (acc + co[:, 1] ** 2) / np.maximum(np.abs(co[:, 0] * co[:, 2] - co[:, 1] ** 2), 1e-300)
    kappa = np.where(ref["radii"] > 0, kappa, 1.0)
    res = {}
    for name, key in (("means3D", "dmeans3D"), ("shs", "dsh"), ("scales", "dscales"), ("rotations", "drot"),
                      ("cov3D_precomp", "dcov3D")):
        if "grad_" + name not in got or key not in want:
            continue
        k = kappa.reshape((-1,) + (1,) * (want[key].ndim - 1))
        res[name] = _check(name, got["grad_" + name], want[key], U * (64.0 + 16.0 * k) * mag[key])
    return res


CASES = {
    "sh3_lang16_direct": dict(N=20000, W=256, H=192, sh_degree=3, lang_dim=16, seed=3),
    "rgb_lang4_rows_bg": dict(N=15000, W=200, H=150, sh_degree=None, lang_dim=4, seed=4, bg=(1.0, 0.5, 0.25)),
    "sh1_nolang_cov": dict(N=12000, W=160, H=120, sh_degree=1, lang_dim=0, seed=5, cov_precomp=True),
    "sh3_lang32_direct_bg": dict(N=8000, W=128, H=96, sh_degree=3, lang_dim=32, seed=6, bg=(0.2, 0.2, 0.9)),
    "sh2_lang64_rows": dict(N=6000, W=112, H=80, sh_degree=2, lang_dim=64, seed=10),
    "rgb_lang24_rows_scale": dict(N=7000, W=97, H=61, sh_degree=None, lang_dim=24, seed=11, scale_modifier=1.3),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_deterministic_backward_is_bit_reproducible(gpu, name):
    case = make_case(**CASES[name])
    D = CASES[name]["lang_dim"]
    dcol, dlang = _upstream(case["cam"]["H"], case["cam"]["W"], D)
    a = run_gpu_bwd_rows(case, gpu, dcol, dlang)
    b = run_gpu_bwd_rows(case, gpu, dcol, dlang)
    assert a.keys() == b.keys()
    for k in a:
        if isinstance(a[k], np.ndarray):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert float(np.abs(a["rows"]).max()) > 1e-3


@pytest.mark.parametrize("name", sorted(CASES))
def test_deterministic_backward_within_analytic_bound(gpu, oracle_lib, name):
    case = make_case(**CASES[name])
    D = CASES[name]["lang_dim"]
    dcol, dlang = _upstream(case["cam"]["H"], case["cam"]["W"], D)
    got = run_gpu_bwd_rows(case, gpu, dcol, dlang)
    pb, ref, r1 = check_rows(case, got, oracle_lib, dcol, dlang)
    r2 = check_chain(pb, ref, got, oracle_lib)
    record(name, {"rows": r1, "chain": r2})


@pytest.mark.parametrize("name", sorted(CASES))
def test_default_backward_within_analytic_bound(gpu, oracle_lib, name):
    """The DEFAULT backward (fp32 atomic cross-block sums) against the same
    derived bound with the any-order summation term in place of the fixed-point
    rounding: its tolerance, too, comes from the analysis, not from a fit."""
    case = make_case(**CASES[name])
    D = CASES[name]["lang_dim"]
    dcol, dlang = _upstream(case["cam"]["H"], case["cam"]["W"], D)
    got = run_gpu_bwd_rows(case, gpu, dcol, dlang, deterministic=False)
    pb, ref, r1 = check_rows(case, got, oracle_lib, dcol, dlang, deterministic=False)
    r2 = check_chain(pb, ref, got, oracle_lib)
    record("default_" + name, {"rows": r1, "chain": r2})


@pytest.mark.parametrize("D", [16, 3])
def test_deterministic_language_only_backward(gpu, oracle_lib, D):
    """Feature-mode shape (geometry frozen, only the language input requires
    grad): the language-only kernel in fixed point, bit-reproducible and within
    the bound (D = 3: a width that is not a multiple of the conversion's column
    quads); the default language-only kernel within its derived bound."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from langsplatv2_amd import _lib
    case = make_case(N=20000, W=256, H=192, sh_degree=3, lang_dim=D, seed=7)
    dcol, dlang = _upstream(192, 256, D, seed=2)
    t = gpu_inputs(case, gpu, requires_grad=False)
    lang = t["language_feature_precomp"].clone().requires_grad_(True)
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu))

    def run(det):
        with _lib.deterministic(det):
            _, L, _ = r(means3D=t["means3D"], means2D=t["means2D"], opacities=t["opacities"], shs=t["shs"],
                        scales=t["scales"], rotations=t["rotations"], language_feature_precomp=lang)
            (g,) = torch.autograd.grad(L, lang, torch.from_numpy(dlang).to(gpu))
        return g.cpu().numpy()
    g1, g2, gf = run(True), run(True), run(False)
    np.testing.assert_array_equal(g1, g2)
    pb = oracle_problem(case)
    ref = oracle_lib.forward(pb)
    rb = oracle_lib.backward(pb, ref, dcol, dlang, nthreads=2)
    bd = oracle_lib.backward_bound(pb, ref, dcol, dlang, with_mag=True)
    Dm, Am, WH = _scales(pb, ref, dcol, dlang)
    tol = bd["dlang"] + _quant(ref["radii"], 0, Dm, Am, WH)[:, None]
    _check("language (deterministic)", g1, rb["dlang"], tol)
    # the default (float-atomic) language-only kernel: the any-order summation term
    tol_f = bd["dlang"] + U * bd["nblocks"].astype(np.float64)[:, None] * bd["mag"]["dlang"]
    _check("language (default)", gf, rb["dlang"], tol_f)


def test_deterministic_quick_weights_only(gpu):
    """Quick (sparse) input, weights alone requiring grad: the deterministic mode
    routes through the dense expansion (fixed-point language-only backward), so
    two runs are bit-identical and equal the default path within fp32 noise."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from langsplatv2_amd import _lib
    case = make_case(N=5000, W=128, H=96, sh_degree=None, quick_k=4, seed=9)
    case["g"]["quick_dim"] = 64
    case["g"]["language_feature_indices"] = torch.remainder(case["g"]["language_feature_indices"], 64.0)
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu))
    dl = torch.randn(64, 96, 128, generator=torch.Generator().manual_seed(2)).to(gpu)

    def run(det):
        w = t["language_feature_weights_quick"].clone().requires_grad_(True)
        with _lib.deterministic(det):
            _, lang, _ = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                           colors_precomp=t["colors_precomp"], scales=t["scales"], rotations=t["rotations"],
                           language_feature_weights_quick=w, language_feature_indices=t["language_feature_indices"])
            (g,) = torch.autograd.grad(lang, w, dl)
        return g
    a, b, f = run(True), run(True), run(False)
    assert torch.equal(a, b)
    torch.testing.assert_close(a, f, rtol=1e-5, atol=1e-5 * float(f.abs().max()))


def test_deterministic_nonfinite_upstream_poisons_the_call(gpu):
    """A NaN in dL/dout makes every gradient of that call NaN (the bounds pass
    flags it), never a silently wrong finite value."""
    case = make_case(N=3000, W=96, H=64, sh_degree=3, lang_dim=16, seed=8)
    dcol, dlang = _upstream(64, 96, 16)
    dcol[1, 10, 20] = np.nan
    got = run_gpu_bwd_rows(case, gpu, dcol, dlang)
    assert np.isnan(got["rows"]).all() and np.isnan(got["grad_language_feature_precomp"]).all()


def test_deterministic_backward_independent_of_list_mode(gpu):
    """The forward's per-block candidate lists (LSR_OPT_LISTS_MAX_MB) change how
    the backward finds its candidates, not which ones or in what order: with
    fixed-point cross-block sums, the list-driven and the re-staging backward
    give the same bits."""
    from langsplatv2_amd import _lib
    case = make_case(**CASES["sh3_lang16_direct"])
    dcol, dlang = _upstream(192, 256, 16)
    a = run_gpu_bwd_rows(case, gpu, dcol, dlang)
    prev = _lib.set_lists_max_mb(0)
    try:
        b = run_gpu_bwd_rows(case, gpu, dcol, dlang)
    finally:
        _lib.set_lists_max_mb(prev)
    for k in a:
        if isinstance(a[k], np.ndarray):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
