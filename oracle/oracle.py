"""numpy/ctypes wrapper of the CPU restatement (oracle/lsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product path.  See lsr_oracle.h
for the parity status (pinned by the reference's importable Python on the
path's edges; against the absent CUDA kernels: parity unpinned).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LSO_ORACLE_LIB: another build of the same restatement (tests/test_asan.py: the ASan build)
_SO = os.environ.get("LSO_ORACLE_LIB", os.path.join(_HERE, "_build", "liblsr_oracle.so"))
_vp = ctypes.c_void_p


class _Settings(ctypes.Structure):
    _fields_ = [("W", ctypes.c_int), ("H", ctypes.c_int), ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
                ("bg", _vp), ("scale_modifier", ctypes.c_float), ("viewmatrix", _vp), ("projmatrix", _vp),
                ("sh_degree", ctypes.c_int), ("campos", _vp), ("include_feature", ctypes.c_int),
                ("quick_render", ctypes.c_int), ("quick_dim", ctypes.c_int)]


class _Inputs(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("M", ctypes.c_int), ("D", ctypes.c_int), ("K", ctypes.c_int),
                ("means3D", _vp), ("shs", _vp), ("colors_precomp", _vp), ("opacities", _vp), ("scales", _vp),
                ("rotations", _vp), ("cov3D_precomp", _vp), ("lang", _vp), ("qweights", _vp), ("qindices", _vp)]


class _Geom(ctypes.Structure):
    _fields_ = [("depth", _vp), ("radii", _vp), ("xy", _vp), ("conic_opacity", _vp), ("rgb", _vp),
                ("clamped", _vp), ("cov3D", _vp), ("tiles_touched", _vp)]


class _RGrads(ctypes.Structure):
    _fields_ = [("dmean2D", _vp), ("dconic", _vp), ("dopacity", _vp), ("dcolor", _vp), ("dlang", _vp)]


class _PGrads(ctypes.Structure):
    _fields_ = [("dmeans3D", _vp), ("dsh", _vp), ("dcolors", _vp), ("dscales", _vp), ("drot", _vp),
                ("dcov3D", _vp)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        lib.lso_num_rendered.restype = ctypes.c_int64
        lib.lso_num_rendered.argtypes = [ctypes.c_int, _vp]
        lib.lso_num_rendered_ex.restype = ctypes.c_int64
        lib.lso_num_rendered_ex.argtypes = [_vp, ctypes.c_int, _vp, ctypes.c_int]
        lib.lso_binning_ex.restype = None
        lib.lso_binning_ex.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int]
        lib.lso_power_cut.restype = ctypes.c_float
        lib.lso_power_cut.argtypes = [ctypes.c_float]
        lib.lso_expf.restype = ctypes.c_float
        lib.lso_expf.argtypes = [ctypes.c_float]
        lib.lso_render_bwd_bound_tiles_mt.restype = None
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_vp)


def _np(t, dtype=np.float32):
    if t is None:
        return None
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    return np.ascontiguousarray(t, dtype=dtype)


class Problem:
    """Host copies of one rasterizer call (settings + inputs), fp32/C-contiguous."""

    def __init__(self, cam: dict, g: dict, bg=(0.0, 0.0, 0.0), scale_modifier=1.0, include_feature=None,
                 quick=False, sh_degree=None):
        self.W, self.H = int(cam["W"]), int(cam["H"])
        self.tanfovx, self.tanfovy = float(cam["tanfovx"]), float(cam["tanfovy"])
        self.view = _np(cam["viewmatrix"])
        self.proj = _np(cam["projmatrix"])
        self.campos = _np(cam["campos"])
        self.bg = np.asarray(bg, dtype=np.float32)
        self.scale_modifier = float(scale_modifier)
        self.means3D = _np(g["means3D"])
        self.N = self.means3D.shape[0]
        self.shs = _np(g.get("shs"))
        self.colors = _np(g.get("colors_precomp"))
        self.opac = _np(g["opacities"])
        self.scales = _np(g.get("scales"))
        self.rot = _np(g.get("rotations"))
        self.cov3D = _np(g.get("cov3D_precomp"))
        if self.cov3D is not None:
            self.scales = self.rot = None
        self.lang = _np(g.get("language_feature_precomp"))
        self.include_feature = (self.lang is not None) if include_feature is None else include_feature
        self.quick = quick
        self.qw = _np(g.get("language_feature_weights_quick")) if quick else None
        self.qi = _np(g.get("language_feature_indices")) if quick else None
        self.quick_dim = int(g.get("quick_dim", 192)) if quick else 0
        self.sh_degree = int(g.get("sh_degree", 0) if sh_degree is None else sh_degree)
        self.M = self.shs.shape[1] if self.shs is not None else 0
        self.D = self.lang.shape[1] if (self.lang is not None and self.include_feature and not quick) else 0
        self.K = self.qw.shape[1] if self.qw is not None else 0
        self.gx, self.gy = (self.W + 15) // 16, (self.H + 15) // 16

    def _structs(self):
        s = _Settings(self.W, self.H, self.tanfovx, self.tanfovy, _p(self.bg), self.scale_modifier, _p(self.view),
                      _p(self.proj), self.sh_degree, _p(self.campos), int(self.D > 0), int(self.quick),
                      self.quick_dim)
        i = _Inputs(self.N, self.M, self.D, self.K, _p(self.means3D), _p(self.shs), _p(self.colors), _p(self.opac),
                    _p(self.scales), _p(self.rot), _p(self.cov3D), _p(self.lang) if self.D else None, _p(self.qw),
                    _p(self.qi))
        return s, i


def forward(pb: Problem, nthreads: int = 1, tiles=None, cull: bool = True, timings: dict | None = None) -> dict:
    """Full oracle forward; returns geometry, binning and image outputs.
    `tiles`: optional subset of tile ids to render (others left zero).
    `cull`: the product's tile cull in the binning (lso_binning_ex); False
    gives the reference's instance lists (A.2) — the rendered outputs are the
    same either way (tests/test_oracle.py::test_tile_cull_changes_no_output).
    `timings`: filled with the wall seconds of preprocess + binning and of the
    render (bench.py's CPU baseline)."""
    import time
    lib = load()
    t0 = time.perf_counter()
    N = pb.N
    g = dict(depth=np.zeros(N, np.float32), radii=np.zeros(N, np.int32), xy=np.zeros((N, 2), np.float32),
             conic_opacity=np.zeros((N, 4), np.float32), rgb=np.zeros((N, 3), np.float32),
             clamped=np.zeros((N, 3), np.uint8), cov3D=np.zeros((N, 6), np.float32),
             tiles_touched=np.zeros(N, np.uint32))
    geom = _Geom(*[_p(g[k]) for k in ("depth", "radii", "xy", "conic_opacity", "rgb", "clamped", "cov3D",
                                     "tiles_touched")])
    s, i = pb._structs()
    lib.lso_preprocess(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom))
    M = int(lib.lso_num_rendered_ex(ctypes.byref(s), N, ctypes.byref(geom), int(bool(cull))))
    T = pb.gx * pb.gy
    point_list = np.zeros(max(M, 1), np.uint32)
    ranges = np.zeros((T, 2), np.uint32)
    lib.lso_binning_ex(ctypes.byref(s), N, ctypes.byref(geom), _p(point_list), _p(ranges), int(bool(cull)))
    Dout = pb.quick_dim if pb.quick else pb.D
    H, W = pb.H, pb.W
    t1 = time.perf_counter()
    color = np.zeros((3, H, W), np.float32)
    lang = np.zeros((Dout, H, W), np.float32)
    final_T = np.zeros((H, W), np.float32)
    n_contrib = np.zeros((H, W), np.uint32)
    if tiles is None:
        lib.lso_render_fwd(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), _p(point_list), _p(ranges),
                           _p(color), _p(lang) if Dout else None, _p(final_T), _p(n_contrib), int(nthreads))
    else:
        tl = np.ascontiguousarray(tiles, dtype=np.int32)
        lib.lso_render_fwd_tiles(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), _p(point_list), _p(ranges),
                                 _p(tl), len(tl), _p(color), _p(lang) if Dout else None, _p(final_T), _p(n_contrib),
                                 int(nthreads))
    if timings is not None:
        timings.update(preprocess_binning=t1 - t0, render=time.perf_counter() - t1)
    out = dict(g)
    out.update(num_rendered=M, point_list=point_list[:M], ranges=ranges, color=color, lang=lang, final_T=final_T,
               n_contrib=n_contrib)
    out["_keep"] = (g, geom)
    return out


def backward(pb: Problem, fwd: dict, dout_color: np.ndarray, dout_lang: np.ndarray | None = None, tiles=None,
             nthreads: int = 1) -> dict:
    lib = load()
    N, D = pb.N, pb.D
    g, geom = fwd["_keep"]
    s, i = pb._structs()
    qdense = qcodes = None
    if pb.quick:
        # quick (sparse) language input: with an upstream language gradient the
        # rows are expanded to dense (N, Dq) coefficients (duplicates summed) and
        # the dense backward runs; dL/dweights[j][m] = dL/dlang[j][code[j][m]]
        # (lsr_bwd_out.dL_dlang_weights).  Without one, RGB only.
        s.quick_render = 0
        if dout_lang is None:
            s.include_feature = 0
            i.D = 0
            i.lang = None
            D = 0
        else:
            qcodes = quick_codes(pb.qi)
            qdense = expand_quick(pb.qw, qcodes, pb.quick_dim)
            D = pb.quick_dim
            s.include_feature = 1
            i.D = D
            i.lang = _p(qdense)
    dcol = _np(dout_color)
    dlang = _np(dout_lang) if (D and dout_lang is not None) else None
    rg = dict(dmean2D=np.zeros((N, 3), np.float32), dconic=np.zeros((N, 3), np.float32),
              dopacity=np.zeros(N, np.float32), dcolor=np.zeros((N, 3), np.float32),
              dlang=np.zeros((N, max(D, 1)), np.float32))
    rgs = _RGrads(_p(rg["dmean2D"]), _p(rg["dconic"]), _p(rg["dopacity"]), _p(rg["dcolor"]),
                  _p(rg["dlang"]) if D else None)
    pl = fwd["point_list"] if fwd["num_rendered"] > 0 else np.zeros(1, np.uint32)
    pl = np.ascontiguousarray(pl)
    if tiles is None and nthreads <= 1:
        lib.lso_render_bwd(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), _p(pl), _p(fwd["ranges"]),
                           _p(fwd["final_T"]), _p(fwd["n_contrib"]), _p(dcol), _p(dlang), ctypes.byref(rgs))
    else:
        tl = np.ascontiguousarray(np.arange(pb.gx * pb.gy) if tiles is None else tiles, dtype=np.int32)
        lib.lso_render_bwd_tiles_mt(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), _p(pl),
                                    _p(fwd["ranges"]), _p(tl), len(tl), _p(fwd["final_T"]), _p(fwd["n_contrib"]),
                                    _p(dcol), _p(dlang), ctypes.byref(rgs), int(nthreads))
    pgd = dict(dmeans3D=np.zeros((N, 3), np.float32), dcolors=np.zeros((N, 3), np.float32))
    if pb.shs is not None:
        pgd["dsh"] = np.zeros_like(pb.shs)
    if pb.scales is not None:
        pgd["dscales"] = np.zeros((N, 3), np.float32)
        pgd["drot"] = np.zeros((N, 4), np.float32)
    if pb.cov3D is not None:
        pgd["dcov3D"] = np.zeros((N, 6), np.float32)
    pgs = _PGrads(_p(pgd["dmeans3D"]), _p(pgd.get("dsh")), _p(pgd["dcolors"]), _p(pgd.get("dscales")),
                  _p(pgd.get("drot")), _p(pgd.get("dcov3D")))
    lib.lso_preprocess_bwd(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), ctypes.byref(rgs), ctypes.byref(pgs))
    out = dict(rg)
    out["dlang"] = rg["dlang"][:, :D] if D else None
    out.update(pgd)
    if qdense is not None:
        ok = (qcodes >= 0) & (qcodes < D)
        rows = np.repeat(np.arange(N)[:, None], qcodes.shape[1], 1)
        out["dlang_weights"] = np.where(ok, out["dlang"][rows, np.clip(qcodes, 0, D - 1)], 0.0).astype(np.float32)
        out["dlang"] = None
    return out


def backward_bound(pb: Problem, fwd: dict, dout_color: np.ndarray, dout_lang: np.ndarray | None = None,
                   nthreads: int = 1, with_mag: bool = False) -> dict:
    """A-priori bound of |product deterministic backward - oracle| per render-gradient
    element (lso_render_bwd_bound_tiles_mt; dense language input): dmean2D (N,3),
    dconic (N,3), dopacity (N,), dcolor (N,3), dlang (N,D).  Excludes the fixed-point
    rounding of the block partials and the two final fp32 roundings.  with_mag: also
    "mag" (the same keys: each element's sum of |term|) and "nblocks" (N,): the 8x8
    blocks each Gaussian contributes in, for the default float-atomic cross-block sum
    (at most nblocks u mag more)."""
    lib = load()
    N, D = pb.N, pb.D
    g, geom = fwd["_keep"]
    s, i = pb._structs()
    dcol = _np(dout_color)
    dlang = _np(dout_lang) if (D and dout_lang is not None) else None

    def grads():
        b = dict(dmean2D=np.zeros((N, 3), np.float32), dconic=np.zeros((N, 3), np.float32),
                 dopacity=np.zeros(N, np.float32), dcolor=np.zeros((N, 3), np.float32),
                 dlang=np.zeros((N, max(D, 1)), np.float32))
        st = _RGrads(_p(b["dmean2D"]), _p(b["dconic"]), _p(b["dopacity"]), _p(b["dcolor"]), _p(b["dlang"]) if D else None)
        return b, st

    b, bs = grads()
    m, ms = grads() if with_mag else (None, None)
    nbk = np.zeros(N, np.float32) if with_mag else None
    pl = np.ascontiguousarray(fwd["point_list"] if fwd["num_rendered"] > 0 else np.zeros(1, np.uint32))
    tl = np.arange(pb.gx * pb.gy, dtype=np.int32)
    lib.lso_render_bwd_bound_tiles_mt(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), _p(pl), _p(fwd["ranges"]),
                                      _p(tl), len(tl), _p(fwd["final_T"]), _p(fwd["n_contrib"]), _p(dcol), _p(dlang),
                                      ctypes.byref(bs), ctypes.byref(ms) if with_mag else None,
                                      _p(nbk) if with_mag else None, int(nthreads))
    b["dlang"] = b["dlang"][:, :D] if D else None
    if with_mag:
        m["dlang"] = m["dlang"][:, :D] if D else None
        b["mag"] = m
        b["nblocks"] = nbk
    return b


def preprocess_backward(pb: Problem, fwd: dict, rg: dict) -> dict:
    """The oracle's preprocess backward (lso_preprocess_bwd) from GIVEN render
    gradients rg = {dmean2D (N,3), dconic (N,3), dopacity (N,), dcolor (N,3)}:
    the chain rule alone, e.g. applied to the product's own gradient rows."""
    lib = load()
    N = pb.N
    g, geom = fwd["_keep"]
    s, i = pb._structs()
    r = {k: np.ascontiguousarray(rg[k], dtype=np.float32) for k in ("dmean2D", "dconic", "dopacity", "dcolor")}
    rgs = _RGrads(_p(r["dmean2D"]), _p(r["dconic"]), _p(r["dopacity"]), _p(r["dcolor"]), None)
    pgd = dict(dmeans3D=np.zeros((N, 3), np.float32), dcolors=np.zeros((N, 3), np.float32))
    if pb.shs is not None:
        pgd["dsh"] = np.zeros_like(pb.shs)
    if pb.scales is not None:
        pgd["dscales"] = np.zeros((N, 3), np.float32)
        pgd["drot"] = np.zeros((N, 4), np.float32)
    if pb.cov3D is not None:
        pgd["dcov3D"] = np.zeros((N, 6), np.float32)
    pgs = _PGrads(_p(pgd["dmeans3D"]), _p(pgd.get("dsh")), _p(pgd["dcolors"]), _p(pgd.get("dscales")),
                  _p(pgd.get("drot")), _p(pgd.get("dcov3D")))
    lib.lso_preprocess_bwd(ctypes.byref(s), ctypes.byref(i), ctypes.byref(geom), ctypes.byref(rgs), ctypes.byref(pgs))
    return pgd


def preprocess_backward_abs(pb: Problem, fwd: dict, rg: dict) -> dict:
    """sum_k |J e_k| |rg_k| per output element: the chain rule's Jacobian J (per
    Gaussian, linear in the render gradients) applied to each render-gradient slot
    k alone (mean2D x/y, conic a/b/c, colour r/g/b), in absolute value, weighted
    by |rg_k|: the magnitude against which the chain's fp32 rounding is bounded."""
    N = pb.N
    slots = [("dmean2D", 0), ("dmean2D", 1), ("dconic", 0), ("dconic", 1), ("dconic", 2),
             ("dcolor", 0), ("dcolor", 1), ("dcolor", 2)]
    out = None
    for key, c in slots:
        unit = {k: np.zeros((N, 3), np.float32) for k in ("dmean2D", "dconic", "dcolor")}
        unit["dopacity"] = np.zeros(N, np.float32)
        unit[key][:, c] = np.abs(np.asarray(rg[key], np.float32)[:, c])
        pg = preprocess_backward(pb, fwd, unit)
        if out is None:
            out = {k: np.abs(v).astype(np.float64) for k, v in pg.items()}
        else:
            for k, v in pg.items():
                out[k] += np.abs(v)
    return out


def quick_codes(qi: np.ndarray) -> np.ndarray:
    """Integer codes of quick indices: fp32-encoded integers round half up (u5)."""
    qi = np.asarray(qi)
    if qi.dtype.kind == "f":
        r = np.floor(qi.astype(np.float32) + np.float32(0.5))
        ok = (r >= 0) & (r < 2.0 ** 31)   # NaN and out-of-range values -> -1 (dropped)
        return np.where(ok, np.where(ok, r, 0).astype(np.int64), -1)
    return qi.astype(np.int64)


def expand_quick(qw: np.ndarray, codes: np.ndarray, Dq: int) -> np.ndarray:
    """Dense (N, Dq) rows of the quick input: row[j][code] += w in code order; out-of-range codes dropped."""
    N, K = qw.shape
    dense = np.zeros((N, Dq), np.float32)
    for m in range(K):
        c = codes[:, m]
        ok = (c >= 0) & (c < Dq)
        r = np.nonzero(ok)[0]
        dense[r, c[ok]] += qw[r, m].astype(np.float32)
    return dense


def expf(x: float) -> float:
    return float(load().lso_expf(ctypes.c_float(x)))


def sh_eval(deg: int, sh_nm3: np.ndarray, dirs: np.ndarray) -> np.ndarray:
    sh = np.ascontiguousarray(sh_nm3, np.float32)
    d = np.ascontiguousarray(dirs, np.float32)
    out = np.zeros((sh.shape[0], 3), np.float32)
    load().lso_sh_eval(int(deg), sh.shape[0], sh.shape[1], _p(sh), _p(d), _p(out))
    return out


def quat_to_R(q: np.ndarray) -> np.ndarray:
    q = np.ascontiguousarray(q, np.float32)
    R = np.zeros((q.shape[0], 3, 3), np.float32)
    load().lso_quat_to_R(q.shape[0], _p(q), _p(R))
    return R


def cov3D(s: np.ndarray, q: np.ndarray, mod: float = 1.0) -> np.ndarray:
    s = np.ascontiguousarray(s, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    out = np.zeros((s.shape[0], 6), np.float32)
    load().lso_cov3D(s.shape[0], _p(s), ctypes.c_float(mod), _p(q), _p(out))
    return out


def knn_dist2(pts: np.ndarray) -> np.ndarray:
    """simple_knn distCUDA2 by brute force (lso_knn_dist2); O(N^2), N <= ~30k."""
    p = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
    out = np.zeros(p.shape[0], np.float32)
    load().lso_knn_dist2(p.shape[0], _p(p), _p(out))
    return out


# --------------------------------------------------------------- language codes
# numpy float64 restatement of the top-k soft codes (utils/vq_utils.py:9-40)
# and of their autograd chain; checks the fused HIP producer
# (csrc/lang_codes.hip).  Pinned by tests/golden/ref_utils.npz (the
# reference's own functions, forward and torch-autograd gradients).

def _topk_mask(y: np.ndarray, k: int) -> np.ndarray:
    """utils/vq_utils.py:16-18: top-k of each row; ties -> lower channel
    (stable sort of -y)."""
    order = np.argsort(-y, axis=1, kind="stable")[:, :k]
    mask = np.zeros(y.shape, dtype=bool)
    np.put_along_axis(mask, order, True, axis=1)
    return mask


def _softmax(x: np.ndarray) -> np.ndarray:
    """utils/vq_utils.py:14 (row softmax, max-shifted)."""
    e = np.exp(x - x.max(axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def topk_soft_code(logits: np.ndarray, k: int, levels: int = 1) -> np.ndarray:
    """softmax_to_topk_soft_code (utils/vq_utils.py:9-24); with levels > 1 the
    per-level concatenation of GaussianModel.get_render_weights
    (scene/gaussian_model.py:510-518).  float64."""
    x = np.asarray(logits, np.float64)
    N, LK = x.shape
    K = LK // levels
    out = np.zeros_like(x)
    for l in range(levels):
        y = _softmax(x[:, l * K:(l + 1) * K])
        z = np.where(_topk_mask(y, k), y, 0.0)
        out[:, l * K:(l + 1) * K] = z / (z.sum(axis=1, keepdims=True) + 1e-10)
    return out


def weights_and_indices(logits: np.ndarray, k: int, levels: int = 1, level_offset: bool = True):
    """get_weights_and_indices (utils/vq_utils.py:26-40) per level, indices
    offset by l*K and concatenated as the quick-path callers do
    (eval_lerf.py:340-348).  Returns (w (N, L*k) float64, idx (N, L*k) int64)."""
    x = np.asarray(logits, np.float64)
    N, LK = x.shape
    K = LK // levels
    ws, ids = [], []
    for l in range(levels):
        y = _softmax(x[:, l * K:(l + 1) * K])
        m = _topk_mask(y, k)
        z = np.where(m, y, 0.0)
        z = z / (z.sum(axis=1, keepdims=True) + 1e-10)
        idx = np.nonzero(m)[1].reshape(N, k)          # ascending channel order per row
        ws.append(np.take_along_axis(z, idx, axis=1))
        ids.append(idx + (l * K if level_offset else 0))
    return np.concatenate(ws, axis=1), np.concatenate(ids, axis=1)


def topk_soft_code_backward(logits: np.ndarray, grad: np.ndarray, k: int, levels: int = 1) -> np.ndarray:
    """dL/dlogits of topk_soft_code for upstream dL/dcode: the chain torch's
    autograd applies to utils/vq_utils.py:14-21 (division by sum + 1e-10, the
    where-mask, softmax).  float64."""
    x = np.asarray(logits, np.float64)
    g = np.asarray(grad, np.float64)
    N, LK = x.shape
    K = LK // levels
    out = np.zeros_like(x)
    for l in range(levels):
        sl = slice(l * K, (l + 1) * K)
        y = _softmax(x[:, sl])
        m = _topk_mask(y, k)
        z = np.where(m, y, 0.0)
        d = z.sum(axis=1, keepdims=True) + 1e-10
        gz = g[:, sl] / d - (g[:, sl] * z).sum(axis=1, keepdims=True) / (d * d)
        dy = np.where(m, gz, 0.0)
        out[:, sl] = y * (dy - (dy * y).sum(axis=1, keepdims=True))
    return out


def lang_cos_loss(weight_map: np.ndarray, codebook: np.ndarray, seg: np.ndarray, features: np.ndarray,
                  eps: float = 1e-8):
    """The feature-mode training loss, materialised as the reference does it
    (float64): f = codebook.T @ W (compute_layer_feature_map, layer 0,
    scene/gaussian_model.py:533-543), gt[:, p] = features[seg[p]] with mask
    seg != -1 (get_language_feature, scene/cameras.py:77-94), loss =
    cos_loss(f*mask, gt*mask) = 1 - mean_p x.y / (max|x|,eps max|y|,eps)
    (utils/loss_utils.py:24-25; torch cosine_similarity semantics).  Ids
    outside [0, S) are masked.  Returns (loss, dL/dW (K, H, W), dL/dcodebook
    (K, Df)) with the gradients differentiated directly in the Df-dim space
    (the GPU kernel factorises through the code space instead)."""
    Wm = np.asarray(weight_map, np.float64)
    cb = np.asarray(codebook, np.float64)
    F = np.asarray(features, np.float64)
    K, H, W = Wm.shape
    P = H * W
    w = Wm.reshape(K, P)
    s = np.asarray(seg).reshape(P).astype(np.int64)
    m = (s >= 0) & (s < F.shape[0])
    f = cb.T @ w                                          # (Df, P)
    gt = np.zeros_like(f)
    gt[:, m] = F[s[m]].T
    x = f * m
    y = gt * m
    nx = np.sqrt((x * x).sum(0))
    ny = np.sqrt((y * y).sum(0))
    Nx, Ny = np.maximum(nx, eps), np.maximum(ny, eps)
    dot = (x * y).sum(0)
    cos = dot / (Nx * Ny)
    loss = 1.0 - cos.mean()
    # d(-mean cos)/dx, then through the mask and f = cb^T w
    live = nx > eps
    dcos_dx = y / (Nx * Ny) - np.where(live, dot / (np.where(live, nx, 1.0) ** 3 * Ny), 0.0) * x
    gx = -dcos_dx / P * m
    dW = (cb @ gx).reshape(K, H, W)
    dcb = w @ gx.T
    return loss, dW, dcb


def adam_steps(param: np.ndarray, grads: list, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
               weight_decay: float = 0.0):
    """torch.optim.Adam's update (no amsgrad; the reference's optimizer,
    scene/gaussian_model.py:255) applied for each gradient in `grads`, in
    float64: m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
    p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).  Returns (p, m, v)."""
    p = np.asarray(param, np.float64).copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    b1, b2 = betas
    for t, g in enumerate(grads, start=1):
        g = np.asarray(g, np.float64)
        if weight_decay:
            g = g + weight_decay * p
        m = m + (1.0 - b1) * (g - m)
        v = b2 * v + (1.0 - b2) * g * g
        step_size = lr / (1.0 - b1 ** t)
        denom = np.sqrt(v) / np.sqrt(1.0 - b2 ** t) + eps
        p = p - step_size * m / denom
    return p, m, v
