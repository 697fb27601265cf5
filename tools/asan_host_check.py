"""Host-side ASan exercise of liblsr's C ABI (SURVEY §5 "Race detection / sanitizers").

Run with the host-ASan build (make -C langsplatv2_amd/csrc asan) and clang's ASan
runtime preloaded (tests/test_asan.py does both).  No GPU: every call below is
rejected by the host-side validation, or is pure host code (stage-name parsing,
the profiling tables, version queries), before any HIP call.  Prints "ok N" with
the number of calls made; any ASan report aborts the process."""
import ctypes
import importlib.util
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
spec = importlib.util.spec_from_file_location("_lsr_lib", os.path.join(HERE, "..", "langsplatv2_amd", "_lib.py"))
L = importlib.util.module_from_spec(spec)
spec.loader.exec_module(L)   # ctypes structures only; torch is never imported
lib = L.load(os.environ["LSR_LIB"])

rng = random.Random(0)
EINVAL, EUNSUP = 1, 2
calls = 0
buf = (ctypes.c_float * 64)()
P = ctypes.cast(buf, ctypes.c_void_p).value   # a valid host address used as a stand-in pointer (never dereferenced)
ALLOC = L.ALLOC_FN(lambda ctx, n, which: 0)


def settings(**kw):
    d = dict(image_height=64, image_width=64, tanfovx=0.5, tanfovy=0.5, bg=P, scale_modifier=1.0, viewmatrix=P,
             projmatrix=P, sh_degree=3, campos=P, prefiltered=0, debug=0, include_feature=0, quick_render=0,
             quick_dim=0)
    d.update(kw)
    return L.Settings(**d)


def inputs(**kw):
    d = dict(P=10, max_coeffs=16, lang_dim=0, quick_k=0, quick_index_dtype=0, means3D=P, shs=P, colors_precomp=None,
             opacities=P, scales=P, rotations=P, cov3D_precomp=None, language_feature_precomp=None,
             language_feature_weights_quick=None, language_feature_indices=None)
    d.update(kw)
    return L.Inputs(**d)


# forward: every case fails validation (expected code), so no HIP call is made
bad = [
    (dict(image_height=0), {}), (dict(image_width=-3), {}), (dict(bg=None), {}), (dict(campos=None), {}),
    ({}, dict(P=-1)), ({}, dict(means3D=None)), ({}, dict(colors_precomp=P)), ({}, dict(shs=None)),
    ({}, dict(cov3D_precomp=P)), ({}, dict(scales=None)), (dict(sh_degree=4), {}), (dict(sh_degree=-1), {}),
    ({}, dict(max_coeffs=3)), (dict(include_feature=1), dict(lang_dim=16)),
    (dict(quick_render=1), dict(quick_k=4)), (dict(quick_render=1), dict(quick_k=4, language_feature_weights_quick=P,
                                                                          language_feature_indices=P,
                                                                          quick_index_dtype=7)),
]
for skw, ikw in bad:
    out = L.FwdOut(P, P, P)
    rc = lib.lsr_forward(ctypes.byref(settings(**skw)), ctypes.byref(inputs(**ikw)), ctypes.byref(out), ALLOC, None,
                         None)
    assert rc == EINVAL, (skw, ikw, rc)
    calls += 1
# unsupported shapes
for skw, ikw in [({}, dict(max_coeffs=25, sh_degree=3)),
                 (dict(include_feature=1), dict(lang_dim=1000, language_feature_precomp=P)),
                 (dict(quick_render=1, quick_dim=100000), dict(quick_k=4, language_feature_weights_quick=P,
                                                               language_feature_indices=P))]:
    rc = lib.lsr_forward(ctypes.byref(settings(**skw)), ctypes.byref(inputs(**ikw)), ctypes.byref(L.FwdOut(P, P, P)),
                         ALLOC, None, None)
    assert rc in (EINVAL, EUNSUP), (skw, ikw, rc)
    calls += 1
# null structs / outputs
assert lib.lsr_forward(None, None, None, ALLOC, None, None) == EINVAL
assert lib.lsr_forward(ctypes.byref(settings()), ctypes.byref(inputs()), ctypes.byref(L.FwdOut(None, P, P)), ALLOC,
                       None, None) == EINVAL
calls += 2
# backward: missing workspaces / upstream gradients, quick/dense conflicts
for bkw, okw, skw in [(dict(geom=None), {}, {}), (dict(dL_dout_color=None), {}, {}), (dict(image=None), {}, {}),
                      ({}, dict(dL_dlang_weights=P), {}),
                      ({}, dict(dL_dlang=P), dict(quick_render=1))]:
    b = dict(geom=P, binning=P, image=P, num_rendered=0, radii=P, dL_dout_color=P, dL_dout_lang=None)
    b.update(bkw)
    o = L.BwdOut(**okw)
    ikw = dict(quick_k=4, language_feature_weights_quick=P, language_feature_indices=P) if skw else {}
    rc = lib.lsr_backward(ctypes.byref(settings(**skw)), ctypes.byref(inputs(**ikw)), ctypes.byref(L.BwdIn(**b)),
                          ctypes.byref(o), ALLOC, None, None)
    assert rc == EINVAL, (bkw, okw, skw, rc)
    calls += 1
# the other entry points' argument checks
assert lib.lsr_mark_visible(-1, None, None, None, None, None) == EINVAL
assert lib.lsr_quick_decode(None, None, 3, 64, 500, 4, 4, 1, 1e-10, None, ALLOC, None, None) == EINVAL
assert lib.lsr_quick_decode(None, None, 3, 32, 512, 4, 4, 1, 1e-10, None, ALLOC, None, None) == EUNSUP
assert lib.lsr_quick_decode_plan_bytes(3, 32, 512, 1) == 0 and lib.lsr_quick_decode_plan_bytes(3, 64, 512, 1) > 0
assert lib.lsr_quick_decode_prepare(None, -1, 64, 512, 1, None, None) == EINVAL
assert lib.lsr_quick_decode_run(None, 0, None, 3, 64, 17, 4, 4, 1, 1e-10, None, None) == EINVAL
assert lib.lsr_quick_decode_run(None, 2, None, 3, 64, 16, 4, 4, 1, 1e-10, None, None) == EINVAL
assert lib.lsr_knn_dist2(None, -5, None, ALLOC, None, None) == EINVAL
assert lib.lsr_adam_step(None, None, None, None, -1, 0.1, 0.9, 0.999, 1e-8, 0.0, 1, None) == EINVAL
calls += 9
# pure host code: stage-name parsing (random strings), profiling tables, versions
names = ["preprocess", "scan_tiles", "bin_count", "scan_tile_counts", "bin_scatter", "tile_sort", "render_fwd",
         "grad_zero", "render_bwd", "preprocess_bwd", "det_bounds", "det_finish"]
for _ in range(2000):
    parts = [rng.choice(names + ["", "x", "render", "render_bwdx", "a" * rng.randint(0, 300)]) for _ in
             range(rng.randint(0, 6))]
    s = ",".join(parts)
    rc = lib.lsr_profile_stages(s.encode())
    segs = s.split(",")
    if len(segs) > 1 and segs[-1] == "":
        segs = segs[:-1]   # a trailing comma is accepted
    ok = all(p in names for p in segs) if s else True
    assert (rc == 0) == ok, (s, rc)
    calls += 1
lib.lsr_profile_stages(None)
lib.lsr_profile_enable(1)
lib.lsr_profile_reset()
nm = (ctypes.c_char_p * 16)()
ms = (ctypes.c_double * 16)()
cl = (ctypes.c_int64 * 16)()
for k in (0, 1, 5, 10, 16):
    n = lib.lsr_profile_query(nm, ms, cl, k)
    assert n == min(k, len(names)), (k, n)
    calls += 1
lib.lsr_profile_enable(0)
# process-wide options: valid modes round-trip, anything else is rejected
lib.lsr_set_option.argtypes = [ctypes.c_int, ctypes.c_int64]
lib.lsr_get_option.argtypes = [ctypes.c_int, ctypes.c_void_p]
v = ctypes.c_int64(-1)
for mode in (1, 0):
    assert lib.lsr_set_option(1, mode) == 0
    assert lib.lsr_get_option(1, ctypes.byref(v)) == 0 and v.value == mode
    calls += 2
for mb in (0, 4096, 2048):   # LSR_OPT_LISTS_MAX_MB
    assert lib.lsr_set_option(2, mb) == 0
    assert lib.lsr_get_option(2, ctypes.byref(v)) == 0 and v.value == mb
    calls += 2
for on in (1, 0):             # LSR_OPT_DETERMINISTIC
    assert lib.lsr_set_option(4, on) == 0
    assert lib.lsr_get_option(4, ctypes.byref(v)) == 0 and v.value == on
    calls += 2
for opt, val in ((1, 2), (1, 3), (1, -1), (2, -5), (0, 0), (77, 1), (4, 2), (4, -1)):
    assert lib.lsr_set_option(opt, val) != 0
    calls += 1
assert lib.lsr_get_option(1, None) != 0
for code in range(-3, 10):
    assert lib.lsr_strerror(code)
    calls += 1
assert lib.lsr_abi_version() >= 6 and lib.lsr_max_lang_dim() == 64
print("ok", calls)
