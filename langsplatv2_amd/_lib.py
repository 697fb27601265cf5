"""ctypes binding of liblsr.so (the C ABI declared in include/lsr.h).

This is the Python side of the drop-in boundary: the same role the
reference's compiled `diff_gaussian_rasterization._C` plays
(gaussian_renderer/__init__.py:15).  No CPU fallback exists: if the HIP
library is missing, or tensors are not on a ROCm device, calls raise.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSR_LIB", os.path.join(_HERE, "liblsr.so"))

LSR_OK = 0
LSR_EINVAL = 1
LSR_ENONFINITE = 6
LSR_ELISTS = 7
LSR_BUF_GEOM, LSR_BUF_BINNING, LSR_BUF_IMAGE, LSR_BUF_GRAD, LSR_BUF_DECODE, LSR_BUF_KNN, LSR_BUF_LOSS = 0, 1, 2, 3, 4, 5, 6
LSR_BUF_GUARD, LSR_BUF_SPARSE, LSR_BUF_GRAD_LANG, LSR_BUF_LISTS, LSR_BUF_DET = 7, 8, 9, 10, 11
LSR_INDEX_F32, LSR_INDEX_I32, LSR_INDEX_I64, LSR_INDEX_PACKED = 0, 1, 2, 3
LSR_GWS_GEOM, LSR_GWS_LANG = 1, 2
LSR_LAYOUT_CHW, LSR_LAYOUT_HWC = 0, 1

_vp = ctypes.c_void_p


class Settings(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int),
        ("image_width", ctypes.c_int),
        ("tanfovx", ctypes.c_float),
        ("tanfovy", ctypes.c_float),
        ("bg", _vp),
        ("scale_modifier", ctypes.c_float),
        ("viewmatrix", _vp),
        ("projmatrix", _vp),
        ("sh_degree", ctypes.c_int),
        ("campos", _vp),
        ("prefiltered", ctypes.c_int),
        ("debug", ctypes.c_int),
        ("include_feature", ctypes.c_int),
        ("quick_render", ctypes.c_int),
        ("quick_dim", ctypes.c_int),
        ("quick_layout", ctypes.c_int),
    ]


class Inputs(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int),
        ("max_coeffs", ctypes.c_int),
        ("lang_dim", ctypes.c_int),
        ("quick_k", ctypes.c_int),
        ("quick_index_dtype", ctypes.c_int),
        ("means3D", _vp),
        ("shs", _vp),
        ("colors_precomp", _vp),
        ("opacities", _vp),
        ("scales", _vp),
        ("rotations", _vp),
        ("cov3D_precomp", _vp),
        ("language_feature_precomp", _vp),
        ("language_feature_weights_quick", _vp),
        ("language_feature_indices", _vp),
    ]


class FwdOut(ctypes.Structure):
    _fields_ = [
        ("out_color", _vp),
        ("out_lang", _vp),
        ("radii", _vp),
        ("geom", _vp),
        ("geom_bytes", ctypes.c_size_t),
        ("binning", _vp),
        ("binning_bytes", ctypes.c_size_t),
        ("image", _vp),
        ("image_bytes", ctypes.c_size_t),
        ("num_rendered", ctypes.c_int64),
        ("grad_ws_request", ctypes.c_int),
        ("grad_ws_kind", ctypes.c_int),
        ("grad_ws", _vp),
        ("grad_ws_bytes", ctypes.c_size_t),
        ("grad_ws_lang", _vp),
        ("lists", _vp),
        ("lists_bytes", ctypes.c_size_t),
    ]


class BwdIn(ctypes.Structure):
    _fields_ = [
        ("geom", _vp),
        ("binning", _vp),
        ("image", _vp),
        ("num_rendered", ctypes.c_int64),
        ("radii", _vp),
        ("dL_dout_color", _vp),
        ("dL_dout_lang", _vp),
        ("grad_ws", _vp),
        ("grad_ws_bytes", ctypes.c_size_t),
        ("grad_ws_kind", ctypes.c_int),
        ("grad_ws_lang", _vp),
        ("lists", _vp),
    ]


class BwdOut(ctypes.Structure):
    _fields_ = [
        ("dL_dmeans2D", _vp),
        ("dL_dcolors", _vp),
        ("dL_dlang", _vp),
        ("dL_dopacity", _vp),
        ("dL_dmeans3D", _vp),
        ("dL_dcov3D", _vp),
        ("dL_dsh", _vp),
        ("dL_dscales", _vp),
        ("dL_drotations", _vp),
        ("dL_dlang_weights", _vp),
        ("lang_ready_event", _vp),
        ("dL_drgb_sh", _vp),
    ]


ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)

EXPORTS = ("lsr_forward", "lsr_backward", "lsr_mark_visible", "lsr_quick_decode", "lsr_quick_decode_plan_bytes",
           "lsr_quick_decode_prepare", "lsr_quick_decode_run", "lsr_quick_pack_codes", "lsr_topk_code_forward",
           "lsr_topk_code_backward", "lsr_topk_code_backward_sparse", "lsr_knn_dist2", "lsr_lang_loss_forward", "lsr_lang_loss_backward", "lsr_adam_step", "lsr_sh_grad_from_views", "lsr_strerror",
           "lsr_abi_version", "lsr_max_lang_dim", "lsr_profile_enable", "lsr_profile_stages", "lsr_profile_reset",
           "lsr_profile_query", "lsr_set_option", "lsr_get_option", "lsr_stream_create", "lsr_stream_destroy")

_lib = None


def load(path: str | None = None):
    """Load liblsr.so (after torch, so the HIP runtime torch already mapped is
    the one the library binds to).  Raises if the library is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"liblsr.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C langsplatv2_amd/csrc`).  There is no CPU fallback.")
    lib = ctypes.CDLL(p)
    lib.lsr_forward.argtypes = [ctypes.POINTER(Settings), ctypes.POINTER(Inputs), ctypes.POINTER(FwdOut),
                                ALLOC_FN, _vp, _vp]
    lib.lsr_forward.restype = ctypes.c_int
    lib.lsr_backward.argtypes = [ctypes.POINTER(Settings), ctypes.POINTER(Inputs), ctypes.POINTER(BwdIn),
                                 ctypes.POINTER(BwdOut), ALLOC_FN, _vp, _vp]
    lib.lsr_backward.restype = ctypes.c_int
    lib.lsr_mark_visible.argtypes = [ctypes.c_int, _vp, _vp, _vp, _vp, _vp]
    lib.lsr_mark_visible.restype = ctypes.c_int
    lib.lsr_quick_decode.argtypes = [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_float, _vp, ALLOC_FN, _vp, _vp]
    lib.lsr_quick_decode.restype = ctypes.c_int
    lib.lsr_quick_decode_plan_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.lsr_quick_decode_plan_bytes.restype = ctypes.c_size_t
    lib.lsr_quick_decode_prepare.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp]
    lib.lsr_quick_decode_prepare.restype = ctypes.c_int
    lib.lsr_quick_decode_run.argtypes = [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, _vp, _vp]
    lib.lsr_quick_decode_run.restype = ctypes.c_int
    if hasattr(lib, "lsr_stream_create"):      # (older A/B builds lack it)
        lib.lsr_stream_create.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        lib.lsr_stream_create.restype = ctypes.c_int
        lib.lsr_stream_destroy.argtypes = [ctypes.c_void_p]
        lib.lsr_stream_destroy.restype = ctypes.c_int
    if hasattr(lib, "lsr_quick_pack_codes"):   # (older A/B builds lack it)
        lib.lsr_quick_pack_codes.argtypes = [_vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _vp, _vp]
        lib.lsr_quick_pack_codes.restype = ctypes.c_int
    lib.lsr_topk_code_forward.argtypes = [_vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp,
                                          _vp, ctypes.c_int, ctypes.c_int, _vp]
    lib.lsr_topk_code_forward.restype = ctypes.c_int
    lib.lsr_topk_code_backward.argtypes = [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                           _vp]
    lib.lsr_topk_code_backward.restype = ctypes.c_int
    lib.lsr_topk_code_backward_sparse.argtypes = [_vp, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  _vp, _vp]
    lib.lsr_topk_code_backward_sparse.restype = ctypes.c_int
    lib.lsr_knn_dist2.argtypes = [_vp, ctypes.c_int64, _vp, ALLOC_FN, _vp, _vp]
    lib.lsr_knn_dist2.restype = ctypes.c_int
    _ci = ctypes.c_int
    lib.lsr_lang_loss_forward.argtypes = [_vp, _vp, _ci, _ci, _ci, _ci, _vp, _vp, _ci, _vp, _vp, ALLOC_FN, _vp, _vp]
    lib.lsr_lang_loss_forward.restype = ctypes.c_int
    lib.lsr_lang_loss_backward.argtypes = [_vp, _vp, _ci, _ci, _ci, _ci, _vp, _vp, _ci, _vp, _vp, _vp, _vp,
                                           ALLOC_FN, _vp, _vp]
    lib.lsr_lang_loss_backward.restype = ctypes.c_int
    _cd = ctypes.c_double
    lib.lsr_adam_step.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_int64, _cd, _cd, _cd, _cd, _cd, ctypes.c_int64, _vp]
    lib.lsr_adam_step.restype = ctypes.c_int
    lib.lsr_sh_grad_from_views.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int, _vp, _vp,
                                           _vp, _vp]
    lib.lsr_sh_grad_from_views.restype = ctypes.c_int
    lib.lsr_strerror.argtypes = [ctypes.c_int]
    lib.lsr_strerror.restype = ctypes.c_char_p
    lib.lsr_abi_version.restype = ctypes.c_int
    lib.lsr_max_lang_dim.restype = ctypes.c_int
    lib.lsr_profile_enable.argtypes = [ctypes.c_int]
    lib.lsr_profile_enable.restype = None
    lib.lsr_profile_stages.argtypes = [ctypes.c_char_p]
    lib.lsr_profile_stages.restype = ctypes.c_int
    lib.lsr_profile_reset.restype = None
    lib.lsr_profile_query.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.lsr_profile_query.restype = ctypes.c_int
    if hasattr(lib, "lsr_set_option"):   # (A/B builds of older sources lack the options)
        lib.lsr_set_option.argtypes = [ctypes.c_int, ctypes.c_int64]
        lib.lsr_set_option.restype = ctypes.c_int
        lib.lsr_get_option.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        lib.lsr_get_option.restype = ctypes.c_int
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != LSR_OK:
        msg = load().lsr_strerror(rc).decode()
        raise RuntimeError(f"{what} failed: {msg} (code {rc})")


LSR_OPT_BIN_MODE = 1
BIN_MODES = {"auto": 0, "sorted_tiles": 1}


def set_bin_mode(mode: str) -> str:
    """Select the forward's tile binning process-wide (lsr_set_option
    LSR_OPT_BIN_MODE): "sorted_tiles" or "auto" (the same: one mode is built);
    returns the previous mode."""
    if mode not in BIN_MODES:
        raise ValueError(f"bin mode must be one of {sorted(BIN_MODES)}")
    lib = load()
    prev = ctypes.c_int64(0)
    check(lib.lsr_get_option(LSR_OPT_BIN_MODE, ctypes.byref(prev)), "lsr_get_option")
    check(lib.lsr_set_option(LSR_OPT_BIN_MODE, BIN_MODES[mode]), "lsr_set_option")
    return {v: k for k, v in BIN_MODES.items()}[prev.value]


LSR_OPT_LISTS_MAX_MB = 2


def set_lists_max_mb(mb: int) -> int:
    """Budget (MiB) for the backward's per-block candidate lists a training
    forward writes (lsr_set_option LSR_OPT_LISTS_MAX_MB, default 2048); above
    it the backward re-stages from the tile lists.  Returns the previous value."""
    lib = load()
    prev = ctypes.c_int64(0)
    check(lib.lsr_get_option(LSR_OPT_LISTS_MAX_MB, ctypes.byref(prev)), "lsr_get_option")
    check(lib.lsr_set_option(LSR_OPT_LISTS_MAX_MB, int(mb)), "lsr_set_option")
    return int(prev.value)


LSR_OPT_SPLIT_PREPROCESS = 3


def set_split_preprocess(on: bool) -> bool:
    """SH colour pass of the forward's preprocess on a second stream,
    concurrent with the binning (lsr_set_option LSR_OPT_SPLIT_PREPROCESS,
    default on; results identical).  Returns the previous setting."""
    lib = load()
    prev = ctypes.c_int64(0)
    check(lib.lsr_get_option(LSR_OPT_SPLIT_PREPROCESS, ctypes.byref(prev)), "lsr_get_option")
    check(lib.lsr_set_option(LSR_OPT_SPLIT_PREPROCESS, 1 if on else 0), "lsr_set_option")
    return bool(prev.value)


LSR_OPT_DETERMINISTIC = 4


def set_deterministic(on: bool) -> bool:
    """Bit-reproducible backward (lsr_set_option LSR_OPT_DETERMINISTIC, default
    off): the render backward's cross-block gradient sums in 64-bit fixed point
    (include/lsr.h).  Returns the previous setting."""
    lib = load()
    prev = ctypes.c_int64(0)
    check(lib.lsr_get_option(LSR_OPT_DETERMINISTIC, ctypes.byref(prev)), "lsr_get_option")
    check(lib.lsr_set_option(LSR_OPT_DETERMINISTIC, 1 if on else 0), "lsr_set_option")
    return bool(prev.value)


class deterministic:
    """Context manager: `with deterministic(): loss.backward()` (restores the
    previous setting on exit; process-wide, like torch.use_deterministic_algorithms)."""

    def __init__(self, on: bool = True):
        self.on = on
        self.prev = None

    def __enter__(self):
        self.prev = set_deterministic(self.on)
        return self

    def __exit__(self, *exc):
        set_deterministic(self.prev)
        return False


def nonblocking_stream(device) -> "torch.cuda.ExternalStream":
    """A torch stream object over a non-blocking HIP stream of `device` (no
    implicit synchronisation with the legacy default stream, which
    torch.cuda.Stream() pool streams keep), created by the library's HIP
    runtime (lsr_stream_create).  Kept for the process's lifetime."""
    import torch
    dev = torch.device(device)
    with torch.cuda.device(dev):
        p = ctypes.c_void_p(0)
        check(load().lsr_stream_create(ctypes.byref(p)), "lsr_stream_create")
    s = torch.cuda.ExternalStream(p.value, device=dev)
    _STREAMS.append(s)
    return s


_STREAMS = []


def profile_enable(on: bool = True):
    load().lsr_profile_enable(1 if on else 0)


def profile_stages(names=None):
    """Time only the named stages (None = all); see lsr_profile_stages."""
    arg = None if not names else ",".join(names).encode()
    check(load().lsr_profile_stages(arg), "lsr_profile_stages")


def profile_reset():
    load().lsr_profile_reset()


def profile_query() -> dict:
    """{stage: (total_ms, calls)} since the last reset (synchronises the events)."""
    n = 16
    names = (ctypes.c_char_p * n)()
    ms = (ctypes.c_double * n)()
    calls = (ctypes.c_int64 * n)()
    k = load().lsr_profile_query(names, ms, calls, n)
    if k < 0:
        raise RuntimeError("lsr_profile_query failed")
    return {names[i].decode(): (ms[i], int(calls[i])) for i in range(k)}
