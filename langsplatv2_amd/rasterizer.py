"""Host-side mirror of the reference operator `diff_gaussian_rasterization`.

Surface (what gaussian_renderer/__init__.py:15,37-54,108-119 uses):
  GaussianRasterizationSettings  NamedTuple, the 14 fields of
                                 gaussian_renderer/__init__.py:37-52, plus an
                                 optional trailing `language_feature_dim`
                                 (quick-path output channels, default 192) and
                                 `language_feature_layout` of the quick map:
                                 None (default) = "hwc" whenever the 12-code,
                                 192-channel kernel applies, else "chw";
                                 "hwc" = stored pixel-major and returned as a
                                 (Dq,H,W) view with strides (1, Dq*W, Dq)
                                 (values identical; the reference's consumers'
                                 .view(3, 64, H, W).view(3, 64, H*W) + einsum
                                 and .view(D, -1) run on it unchanged);
                                 "chw" = the reference's contiguous (Dq,H,W).
  GaussianRasterizer(raster_settings)  nn.Module;
      forward(means3D, means2D, opacities, shs=None, colors_precomp=None,
              language_feature_precomp=None,
              language_feature_weights_quick=None,
              language_feature_indices=None, scales=None, rotations=None,
              cov3D_precomp=None) -> (color (3,H,W), language map (D,H,W), radii (N,))
      markVisible(positions) -> bool (N,)
  rasterize_gaussians(...)       functional form (autograd).

Behaviour kept from the reference:
  - exactly one of shs / colors_precomp, exactly one of (scales, rotations) /
    cov3D_precomp, else `Exception` before any launch;
  - means2D receives dL/d(NDC xy) in [:, :2] (scene/gaussian_model.py:507);
  - `debug=True`: synchronous per-stage checks in the library, and on failure
    the inputs are dumped to snapshot_fw.dump / snapshot_bw.dump;
  - placeholder tensors with numel <= 1 (torch.zeros((1,)),
    gaussian_renderer/__init__.py:93,97-98,101-103) mean "absent".
Language modes (gaussian_renderer/__init__.py:87-103):
  include_feature=True  -> dense (N,D) coefficients, output (D,H,W);
  quick_render=True     -> sparse (N,K) weights + (N,K) indices (fp32-encoded
                           integers, or int32/int64), output (Dq,H,W); the
                           weights are differentiable (the
                           fused top-k producer feeds training sparse codes),
                           the indices are not;
  neither               -> output (0,H,W).
Data-parallel hook: `GradSink` (a context manager) hands the backward
preallocated gradient destinations (views of an all-reduce bucket, so no pack
copy) and an event the library records once the language gradient is final.
All compute runs in liblsr.so (hand-written HIP, gfx950); this module only
moves pointers.  There is no CPU path.
"""
from __future__ import annotations

import ctypes
import threading
import weakref
from typing import NamedTuple, Optional

import torch
import torch.nn as nn

from . import _lib


# The active sinks, process-wide: autograd runs a CUDA backward on its own
# device thread, not on the thread that entered the context (a thread-local
# stack is invisible there).
_SINKS: list = []
_SINKS_LOCK = threading.Lock()


class GradSink:
    """Destinations for the gradients of the rasterizer backward(s) run while
    the context is active (process-wide: the backward runs on autograd's
    device thread):

      buffers     {input name: tensor}: preallocated fp32 outputs, used when
                  shape / device match (the library writes every element), e.g.
                  views of a flat all-reduce bucket (langsplatv2_amd/dp.py);
      lang_ready  optional torch.cuda.Event, recorded on the backward's stream
                  as soon as dL/dlanguage is final (before the preprocess
                  backward), so a collective on another stream can start early;
      on_lang_ready  optional callable run right after the library call has
                  been enqueued (host side), e.g. to launch that collective;
      rgb_sh      optional (N,3) fp32 tensor: the view-factored SH gradient
                  (multi-GPU exchange, dp.py): the backward writes the SH
                  colour gradient dL/dRGB here instead of dL/dshs, and returns
                  buffers["shs"] as the SH gradient, which the caller fills
                  after the exchange (lsr_sh_grad_from_views).  Used only when
                  buffers has "shs" and the SH input needs a gradient.
      sh_return   optional tensor autograd receives as the SH gradient of a
                  factored backward instead of buffers["shs"] (dp.py passes an
                  expanded zero: a second gradient path into the SH leaf then
                  sums to exactly its own contribution, which the exchange adds).

      params      optional {input name: leaf tensor}: a buffer is used only when
                  the rasterizer's input of that name IS this tensor (the bucketed
                  leaf itself; with the reference glue, e.g. shs = cat(f_dc, f_rest),
                  the input is a non-leaf and its gradient goes to a fresh tensor).

    `used` collects the names whose buffer a backward wrote; a second backward
    in the same sink that would write the same buffer raises (autograd would
    otherwise sum two views of one tensor).  on_lang_ready is called with the
    sink, after `used` is updated.

    Input names: means3D, means2D, shs, colors_precomp, language_feature_precomp,
    language_feature_weights_quick, opacities, scales, rotations, cov3D_precomp."""

    def __init__(self, buffers=None, lang_ready=None, on_lang_ready=None, rgb_sh=None, params=None, sh_return=None):
        self.buffers = dict(buffers or {})
        self.lang_ready = lang_ready
        self.on_lang_ready = on_lang_ready
        self.rgb_sh = rgb_sh
        self.sh_return = sh_return
        self.params = dict(params) if params is not None else None
        self.used: set = set()

    def take(self, name, shape, dev, input_id) -> Optional[torch.Tensor]:
        """The buffer for input `name` of a backward (None: allocate a fresh one)."""
        t = self.buffers.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != torch.float32 or t.device != dev \
                or not t.is_contiguous():
            return None
        if self.params is not None:
            leaf = self.params.get(name)
            if leaf is None or id(leaf) != input_id:
                return None
        if name in self.used:
            raise RuntimeError(f"GradSink: the {name} buffer was already written by another backward in this sink")
        self.used.add(name)
        return t

    def __enter__(self):
        with _SINKS_LOCK:
            _SINKS.append(self)
        return self

    def __exit__(self, *exc):
        with _SINKS_LOCK:
            _SINKS.remove(self)
        return False


def _sink() -> Optional[GradSink]:
    with _SINKS_LOCK:
        return _SINKS[-1] if _SINKS else None


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    include_feature: bool = False
    quick_render: bool = False
    language_feature_dim: Optional[int] = None
    language_feature_layout: Optional[str] = None


def _quick_layout(rs, hwc_ok: bool = False) -> int:
    """LSR_LAYOUT_* of the quick map: "chw" the reference's contiguous (Dq,H,W); "hwc"
    pixel-major; None (the default) pixel-major when `hwc_ok` (the inputs fit the kernel
    that writes it: 12 codes, 192 channels, 16-B aligned rows), else "chw"."""
    lay = rs.language_feature_layout if len(rs) > 15 else None
    if lay is None:
        return _lib.LSR_LAYOUT_HWC if (hwc_ok and rs.quick_render) else _lib.LSR_LAYOUT_CHW
    if lay == "chw":
        return _lib.LSR_LAYOUT_CHW
    if lay == "hwc":
        if not rs.quick_render:
            raise ValueError('language_feature_layout="hwc" applies to the quick_render map only')
        return _lib.LSR_LAYOUT_HWC
    raise ValueError(f'language_feature_layout must be "chw" or "hwc", got {lay!r}')


def _present(t: Optional[torch.Tensor]) -> bool:
    """False for None, empty tensors and the reference's 1-element placeholders
    (torch.zeros((1,)), gaussian_renderer/__init__.py:93,97-98,101-103)."""
    return t is not None and t.numel() > 0 and not (t.dim() <= 1 and t.numel() <= 1)


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a ROCm device tensor (got {t.device}); "
                           "the rasterizer has no CPU path")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


class _Alloc:
    """Workspace allocator handed to the C ABI: torch's caching allocator."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}

        def cb(_ctx, nbytes, which):
            t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self.device)
            self.bufs[int(which)] = t
            return t.data_ptr()

        self.fn = _lib.ALLOC_FN(cb)


def _settings_struct(rs: GaussianRasterizationSettings, dev, layout: int = 0) -> tuple:
    bg = _f32(rs.bg, "bg")
    view = _f32(rs.viewmatrix, "viewmatrix")
    proj = _f32(rs.projmatrix, "projmatrix")
    campos = _f32(rs.campos, "campos")
    qdim = rs.language_feature_dim if (len(rs) > 14 and rs.language_feature_dim) else 0
    s = _lib.Settings(int(rs.image_height), int(rs.image_width), float(rs.tanfovx), float(rs.tanfovy),
                      bg.data_ptr(), float(rs.scale_modifier), view.data_ptr(), proj.data_ptr(),
                      int(rs.sh_degree), campos.data_ptr(), int(bool(rs.prefiltered)), int(bool(rs.debug)),
                      int(bool(rs.include_feature)), int(bool(rs.quick_render)), int(qdim), int(layout))
    return s, (bg, view, proj, campos)


def _index_dtype(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.LSR_INDEX_F32
    if t.dtype == torch.int32:
        return _lib.LSR_INDEX_I32
    if t.dtype == torch.int64:
        return _lib.LSR_INDEX_I64
    raise RuntimeError(f"language_feature_indices dtype {t.dtype} unsupported (float32/int32/int64)")


# The quick render stages each candidate's 12 code indices; converting the
# reference's fp32 indices (u5: round half up, range check) is per candidate and
# frame work, so the forward hands the library packed rows (LSR_INDEX_PACKED,
# lsr_quick_pack_codes) converted once per indices tensor and kept while that
# tensor is unchanged (same object, same version counter).  An entry holds only
# a weak reference to the indices tensor (a dropped tensor's rows are not pinned;
# a freed tensor's reused storage cannot match: the referent is gone), and the
# packed rows are marked as used on every stream that reads them (record_stream),
# so an eviction never returns their block to one stream's pool while a render on
# another stream still reads it.  False: the forward passes the indices as they
# are (A/B, tests).
QUICK_PACKED_CODES = True
_PACKED = {}
_PACKED_MAX = 2


def _packed_codes(qi: torch.Tensor, Dq: int) -> torch.Tensor:
    try:
        ver = qi._version
    except RuntimeError:   # an inference tensor tracks no version: convert every call
        ver = None
    stream = torch.cuda.current_stream(qi.device)
    key = (qi.data_ptr(), qi.device, tuple(qi.shape), qi.dtype, int(Dq))
    hit = _PACKED.get(key)
    if ver is not None and hit is not None and hit[0]() is qi and hit[1] == ver:
        packed = hit[2]
        if stream != hit[3]:
            packed.record_stream(stream)
        return packed
    packed = torch.empty((qi.shape[0], 4), dtype=torch.int32, device=qi.device)
    _lib.check(_lib.load().lsr_quick_pack_codes(qi.data_ptr(), _index_dtype(qi), int(qi.shape[0]), int(qi.shape[1]),
                                                int(Dq), packed.data_ptr(), stream.cuda_stream),
               "lsr_quick_pack_codes")
    if ver is not None:
        _PACKED.pop(key, None)
        while len(_PACKED) >= _PACKED_MAX:
            _PACKED.pop(next(iter(_PACKED)))
        _PACKED[key] = (weakref.ref(qi), ver, packed, stream)
    return packed


def _use_packed(qw: torch.Tensor, qi: torch.Tensor, Dq: int) -> bool:
    """The packed rows apply: 12 codes per Gaussian, Dq <= 192, 16-B aligned rows
    (the LDS-DMA quick kernel, csrc/render.hip k_render_fwd_quick_d)."""
    return (QUICK_PACKED_CODES and qi.dim() == 2 and qi.shape[0] > 0 and qi.shape[1] == 12 and qw.shape[1] == 12
            and Dq <= 192 and qi.dtype in (torch.float32, torch.int32, torch.int64)
            and qw.data_ptr() % 16 == 0 and qi.data_ptr() % 16 == 0)


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _dump(path, tensors):
    try:
        torch.save([t.detach().cpu() if isinstance(t, torch.Tensor) else t for t in tensors], path)
        print(f"\nAn error occured in the rasterizer. Please forward {path} for debugging.")
    except Exception:  # pragma: no cover - best effort
        pass


def _run_forward(means3D, sh, colors_precomp, language_feature_precomp, language_feature_weights_quick,
                 language_feature_indices, opacities, scales, rotations, cov3Ds_precomp, rs, grad_request=0):
    """One lsr_forward call.  Returns (color, lang, radii, num_rendered, bufs, saved, dims, grad_ws) where
    bufs = {LSR_BUF_*: uint8 workspace tensor}, saved = contiguous inputs and grad_ws = None or
    (uint8 tensor, bytes, kind, lang_off): the backward's accumulators, zeroed by the forward render
    when grad_request (LSR_GWS_*) asked for them (lsr_fwd_out.grad_ws)."""
    dev = means3D.device
    lib = _lib.load()
    N = means3D.shape[0]
    means3D_c = _f32(means3D, "means3D")
    opac_c = _f32(opacities, "opacities")
    sh_c = _f32(sh, "shs") if _present(sh) else None
    col_c = _f32(colors_precomp, "colors_precomp") if _present(colors_precomp) else None
    sc_c = _f32(scales, "scales") if _present(scales) else None
    rot_c = _f32(rotations, "rotations") if _present(rotations) else None
    cov_c = _f32(cov3Ds_precomp, "cov3D_precomp") if _present(cov3Ds_precomp) else None
    quick = bool(rs.quick_render)
    dense = bool(rs.include_feature) and not quick
    lang_c = _f32(language_feature_precomp, "language_feature_precomp") \
        if (dense and _present(language_feature_precomp)) else None
    qw_c = qi_c = None
    if quick:
        qw_c = _f32(language_feature_weights_quick, "language_feature_weights_quick")
        qi_c = language_feature_indices.contiguous()
        if not qi_c.is_cuda:
            raise RuntimeError("language_feature_indices must be a ROCm device tensor")
    M = sh_c.shape[1] if sh_c is not None and sh_c.dim() == 3 else (
        sh_c.shape[1] // 3 if sh_c is not None else 0)
    D = lang_c.shape[1] if lang_c is not None else 0
    K = qw_c.shape[1] if qw_c is not None else 0
    Dq = (rs.language_feature_dim if (len(rs) > 14 and rs.language_feature_dim) else 192) if quick else 0
    Dout = Dq if quick else D
    H, W = int(rs.image_height), int(rs.image_width)

    qi_fwd, qi_dt = qi_c, (_index_dtype(qi_c) if qi_c is not None else 0)
    if quick and _use_packed(qw_c, qi_c, Dq):
        qi_fwd, qi_dt = _packed_codes(qi_c, Dq), _lib.LSR_INDEX_PACKED
    # the quick map's layout: pixel-major by default where its kernel applies (lsr_api validate)
    layout = _quick_layout(rs, quick and K == 12 and Dq == 192 and qw_c.data_ptr() % 16 == 0
                           and qi_fwd.data_ptr() % 16 == 0)
    s, keep = _settings_struct(rs, dev, layout)
    ins = _lib.Inputs(N, M, D, K, qi_dt,
                      means3D_c.data_ptr(), _ptr(sh_c), _ptr(col_c), opac_c.data_ptr(), _ptr(sc_c), _ptr(rot_c),
                      _ptr(cov_c), _ptr(lang_c), _ptr(qw_c), _ptr(qi_fwd))
    color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
    if layout == _lib.LSR_LAYOUT_HWC:
        lang_out = torch.empty((H, W, Dout), dtype=torch.float32, device=dev).permute(2, 0, 1)
    else:
        lang_out = torch.empty((Dout, H, W), dtype=torch.float32, device=dev)
    radii = torch.empty((N,), dtype=torch.int32, device=dev)
    out = _lib.FwdOut(color.data_ptr(), lang_out.data_ptr() if Dout else None, radii.data_ptr())
    out.grad_ws_request = int(grad_request)
    alloc = _Alloc(dev)
    rc = lib.lsr_forward(ctypes.byref(s), ctypes.byref(ins), ctypes.byref(out), alloc.fn, None, _stream(dev))
    if rc != _lib.LSR_OK:
        if rs.debug:
            _dump("snapshot_fw.dump", [means3D, sh, colors_precomp, opacities, scales, rotations,
                                       cov3Ds_precomp, language_feature_precomp, rs.viewmatrix, rs.projmatrix])
        _lib.check(rc, "rasterize_gaussians (forward)")
    saved = (means3D_c, opac_c, sh_c, col_c, sc_c, rot_c, cov_c, lang_c, qw_c, qi_c)
    grad_ws = None
    if out.grad_ws_kind:
        # (rows or None, rows bytes, kind, (N, D) dL/dlang accumulator or None): the
        # accumulator is its own allocation (LSR_BUF_GRAD_LANG), so the gradient handed
        # to autograd from it keeps no gradient rows alive
        grad_ws = (alloc.bufs.get(_lib.LSR_BUF_GRAD) if out.grad_ws else None, int(out.grad_ws_bytes),
                   int(out.grad_ws_kind), alloc.bufs.get(_lib.LSR_BUF_GRAD_LANG) if out.grad_ws_lang else None)
    return color, lang_out, radii, int(out.num_rendered), alloc.bufs, saved, (N, M, D, K), grad_ws


_CALL = threading.local()   # grad mode at the rasterize_gaussians call (see _grad_request)


def _grad_request(need, sh, colors_precomp, language_feature_precomp, scales, rotations, cov3Ds_precomp, rs) -> int:
    """LSR_GWS_* bits for the gradients the backward will request (the same rule as backward's outputs)."""
    # (called inside Function.forward, where grad mode is always off: whether
    # the caller had it on is recorded by rasterize_gaussians before apply)
    if bool(rs.quick_render) or not getattr(_CALL, "grad_enabled", False):
        return 0
    geom = (need[0] or need[1] or (need[2] and _present(sh)) or (need[3] and _present(colors_precomp)) or need[7]
            or (need[8] and _present(scales)) or (need[9] and _present(rotations))
            or (need[10] and _present(cov3Ds_precomp)))
    lang = need[4] and bool(rs.include_feature) and _present(language_feature_precomp)
    return (_lib.LSR_GWS_GEOM if geom else 0) | (_lib.LSR_GWS_LANG if lang else 0)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, language_feature_precomp,
                language_feature_weights_quick, language_feature_indices, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings):
        req = _grad_request(ctx.needs_input_grad, sh, colors_precomp, language_feature_precomp, scales, rotations,
                            cov3Ds_precomp, raster_settings)
        color, lang_out, radii, num_rendered, bufs, saved, dims, grad_ws = _run_forward(
            means3D, sh, colors_precomp, language_feature_precomp, language_feature_weights_quick,
            language_feature_indices, opacities, scales, rotations, cov3Ds_precomp, raster_settings, req)
        # zeroed accumulators for ONE backward (taken there)
        ctx.grad_ws = grad_ws
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        # identities of the inputs (GradSink.params: a sink buffer is used only for its own leaf)
        ctx.input_ids = {"means3D": id(means3D), "means2D": id(means2D), "shs": id(sh),
                         "colors_precomp": id(colors_precomp), "language_feature_precomp": id(language_feature_precomp),
                         "language_feature_weights_quick": id(language_feature_weights_quick),
                         "opacities": id(opacities), "scales": id(scales), "rotations": id(rotations),
                         "cov3D_precomp": id(cov3Ds_precomp)}
        ctx.dims = dims
        # each 8x8 block's candidate list, written by the forward render for the
        # backward (lsr_fwd_out.lists; read only, kept for every backward of this
        # graph).  Saved like the binning buffers, so autograd frees it with the
        # graph after the backward (unless retain_graph) instead of holding it for
        # as long as an output's grad_fn lives
        ctx.save_for_backward(*saved, radii, bufs[_lib.LSR_BUF_GEOM], bufs[_lib.LSR_BUF_BINNING],
                              bufs[_lib.LSR_BUF_IMAGE], bufs.get(_lib.LSR_BUF_LISTS))
        ctx.mark_non_differentiable(radii)
        # backward handles None upstream gradients itself; without this autograd
        # zero-fills a gradient for the int radii output every step
        ctx.set_materialize_grads(False)
        return color, lang_out, radii

    @staticmethod
    def backward(ctx, grad_color, grad_lang, _grad_radii):
        rs = ctx.raster_settings
        (means3D, opac, sh, col, sc, rot, cov, lang, qw, qi, radii, geom, binning, image, lists) = ctx.saved_tensors
        N, M, D, K = ctx.dims
        dev = means3D.device
        lib = _lib.load()
        need = ctx.needs_input_grad
        quick = bool(rs.quick_render)
        # inputs: 0 means3D 1 means2D 2 sh 3 colors 4 lang 5 qw 6 qi 7 opac 8 scales 9 rot 10 cov 11 settings
        grad_color = grad_color.contiguous() if grad_color is not None else torch.zeros(
            (3, rs.image_height, rs.image_width), device=dev)
        gl = None
        if lang is not None:
            gl = grad_lang.contiguous() if grad_lang is not None else torch.zeros(
                (D, rs.image_height, rs.image_width), device=dev)
        elif quick and grad_lang is not None:
            # the quick channels take part in the backward only when a gradient reaches them
            gl = grad_lang.contiguous()
        # (the backward reads the contiguous upstream gradient: the map's layout plays no part)
        s, keep = _settings_struct(rs, dev, _lib.LSR_LAYOUT_CHW)
        ins = _lib.Inputs(N, M, D, K if quick else 0, _index_dtype(qi) if quick else 0, means3D.data_ptr(), _ptr(sh),
                          _ptr(col), opac.data_ptr(), _ptr(sc), _ptr(rot), _ptr(cov), _ptr(lang),
                          _ptr(qw) if quick else None, _ptr(qi) if quick else None)
        bin_ = _lib.BwdIn(geom.data_ptr(), binning.data_ptr(), image.data_ptr(), ctx.num_rendered, radii.data_ptr(),
                          grad_color.data_ptr(), _ptr(gl))
        if lists is not None:
            bin_.lists = lists.data_ptr()
        ws = ctx.grad_ws
        ctx.grad_ws = None   # a second backward (retain_graph) clears its own
        if ws is not None:
            bin_.grad_ws = ws[0].data_ptr() if ws[0] is not None else None
            bin_.grad_ws_bytes, bin_.grad_ws_kind = ws[1], ws[2]
            bin_.grad_ws_lang = ws[3].data_ptr() if ws[3] is not None else None
        sink = _sink()

        def mk(name, shape, flag):
            if not flag:
                return None
            if sink is not None:
                t = sink.take(name, shape, dev, ctx.input_ids[name])
                if t is not None:
                    return t
            return torch.empty(shape, dtype=torch.float32, device=dev)

        # only what autograd asks for: with the language input alone requiring
        # grad (feature mode, means2D without grad) the library runs its
        # language-only backward (dense rows, or the quick weights)
        g_means2D = mk("means2D", (N, 3), need[1])
        g_means3D = mk("means3D", (N, 3), need[0])
        g_sh = mk("shs", tuple(sh.shape), need[2]) if sh is not None else None
        g_col = mk("colors_precomp", (N, 3), need[3]) if col is not None else None
        g_lang = None
        if lang is not None and need[4]:
            if sink is not None:
                g_lang = sink.take("language_feature_precomp", (N, D), dev, ctx.input_ids["language_feature_precomp"])
            if g_lang is None and ws is not None and ws[3] is not None:
                # the forward's zeroed (N, D) accumulator: the library adds into it in place
                g_lang = ws[3][:N * D * 4].view(torch.float32).view(N, D)
            if g_lang is None:
                g_lang = torch.empty((N, D), dtype=torch.float32, device=dev)
        g_qw = mk("language_feature_weights_quick", (N, K), need[5]) if (quick and qw is not None) else None
        g_opac = mk("opacities", (N, 1), need[7])
        g_sc = mk("scales", (N, 3), need[8]) if sc is not None else None
        g_rot = mk("rotations", (N, 4), need[9]) if rot is not None else None
        g_cov = mk("cov3D_precomp", (N, 6), need[10]) if cov is not None else None
        ev = sink.lang_ready if sink is not None else None
        if ev is not None and not ev.cuda_event:
            ev.record(torch.cuda.current_stream(dev))   # materialise the event handle
        # view-factored SH gradient: the library writes dL/dRGB of the SH
        # evaluation; g_sh (the sink's buffer) is filled by the exchange
        rgb_sh = None
        if (sink is not None and sink.rgb_sh is not None and g_sh is not None and "shs" in sink.buffers
                and g_sh.data_ptr() == sink.buffers["shs"].data_ptr()):
            rgb_sh = sink.rgb_sh
            if tuple(rgb_sh.shape) != (N, 3) or rgb_sh.dtype != torch.float32 or not rgb_sh.is_contiguous():
                raise ValueError("GradSink.rgb_sh must be a contiguous (N, 3) fp32 tensor")
        bout = _lib.BwdOut(_ptr(g_means2D), _ptr(g_col), _ptr(g_lang), _ptr(g_opac), _ptr(g_means3D), _ptr(g_cov),
                           None if rgb_sh is not None else _ptr(g_sh), _ptr(g_sc), _ptr(g_rot), _ptr(g_qw),
                           ev.cuda_event if ev is not None else None, _ptr(rgb_sh))
        alloc = _Alloc(dev)
        rc = lib.lsr_backward(ctypes.byref(s), ctypes.byref(ins), ctypes.byref(bin_), ctypes.byref(bout), alloc.fn,
                              None, _stream(dev))
        if rc != _lib.LSR_OK:
            if rs.debug:
                _dump("snapshot_bw.dump", [grad_color, gl, means3D, sh, col, opac, sc, rot, cov, lang, qw, qi])
            _lib.check(rc, "rasterize_gaussians_backward")
        if sink is not None and sink.on_lang_ready is not None:
            sink.on_lang_ready(sink)
        if rgb_sh is not None and sink.sh_return is not None:
            g_sh = sink.sh_return
        return (g_means3D if need[0] else None, g_means2D if need[1] else None, g_sh, g_col, g_lang, g_qw, None,
                g_opac if need[7] else None, g_sc, g_rot, g_cov, None)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, language_feature_precomp,
                        language_feature_weights_quick, language_feature_indices, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings):
    _CALL.grad_enabled = torch.is_grad_enabled()
    try:
        return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, language_feature_precomp,
                                         language_feature_weights_quick, language_feature_indices, opacities, scales,
                                         rotations, cov3Ds_precomp, raster_settings)
    finally:
        _CALL.grad_enabled = False


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            rs = self.raster_settings
            pos = _f32(positions, "positions")
            view = _f32(rs.viewmatrix, "viewmatrix")
            proj = _f32(rs.projmatrix, "projmatrix")
            out = torch.empty((pos.shape[0],), dtype=torch.bool, device=pos.device)
            rc = _lib.load().lsr_mark_visible(int(pos.shape[0]), pos.data_ptr(), view.data_ptr(), proj.data_ptr(),
                                              out.data_ptr(), _stream(pos.device))
            _lib.check(rc, "mark_visible")
        return out

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, language_feature_precomp=None,
                language_feature_weights_quick=None, language_feature_indices=None, scales=None, rotations=None,
                cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = torch.empty(0, device=means3D.device)
        shs = empty if shs is None else shs
        colors_precomp = empty if colors_precomp is None else colors_precomp
        scales = empty if scales is None else scales
        rotations = empty if rotations is None else rotations
        cov3D_precomp = empty if cov3D_precomp is None else cov3D_precomp
        if language_feature_precomp is None:
            language_feature_precomp = empty
        if language_feature_weights_quick is None:
            language_feature_weights_quick = empty
        if language_feature_indices is None:
            language_feature_indices = empty
        if rs.quick_render and not (_present(language_feature_weights_quick) and
                                    _present(language_feature_indices)):
            raise Exception('quick_render requires language_feature_weights_quick and language_feature_indices!')
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, language_feature_precomp,
                                   language_feature_weights_quick, language_feature_indices, opacities, scales,
                                   rotations, cov3D_precomp, rs)
