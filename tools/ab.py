"""A/B timing of liblsr variants in ONE process: each variant's library is
loaded under its own name and the cfg3 fwd+bwd stage times are measured in
interleaved rounds (cdna guide §5.4 rule 24).  Usage: python tools/ab.py name=path.so[#binmode] ...
(binmode: auto / sorted_tiles, set through lsr_set_option before each of the variant's rounds;
LSR_CFG selects the BASELINE config, default 3)."""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

variants = [a.split("=", 1) for a in sys.argv[1:]]
split0 = {name: path.endswith("#split0") for name, path in variants}
variants = [(name, path[:-len("#split0")] if split0[name] else path) for name, path in variants]
modes = {name: _lib.BIN_MODES[path.split("#", 1)[1]] if "#" in path else None for name, path in variants}
libs = {name: _lib.load(path.split("#", 1)[0]) for name, path in variants}
cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
D = int(os.environ.get("LSR_D", cfg["lang_dim"]))
FWD_ONLY = not cfg["backward"]
dev = torch.device("cuda:0")
cam = make_camera(cfg["W"], cfg["H"])
g0 = make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=D)
keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
if os.environ.get("LSR_SPATIAL") == "y":
    # layout probe: the Gaussians sorted by their projected screen row (y / z)
    # only, so a wave's lanes share rows but spread over the columns
    m = g0["means3D"].double()
    perm = torch.argsort(m[:, 1] / m[:, 2].clamp_min(1e-6))
    g0 = {k: (v[perm] if isinstance(v, torch.Tensor) and v.shape[:1] == perm.shape else v) for k, v in g0.items()}
elif os.environ.get("LSR_SPATIAL"):
    # layout probe: the same Gaussians in a spatial order (3-D Morton code of the
    # means, 10 bits per axis) instead of the generator's random order
    m = g0["means3D"].double()
    lo, hi = m.min(0).values, m.max(0).values
    q = ((m - lo) / (hi - lo).clamp_min(1e-12) * 1023).long().clamp(0, 1023)

    def spread(v):
        out = torch.zeros_like(v)
        for b in range(10):
            out |= ((v >> b) & 1) << (3 * b)
        return out
    code = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
    perm = torch.argsort(code)
    g0 = {k: (v[perm] if isinstance(v, torch.Tensor) and v.shape[:1] == perm.shape else v) for k, v in g0.items()}
g = {k: g0[k].to(dev).requires_grad_(True) for k in keys}
g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
r = GaussianRasterizer(bench.settings(cam, dev, 3, True))
dc = torch.randn(3, cfg["H"], cfg["W"], device=dev)
dl = torch.randn(D, cfg["H"], cfg["W"], device=dev)


def set_split(name):
    # "name=path#split0": the fused preprocess (LSR_OPT_SPLIT_PREPROCESS 0)
    lib = libs[name]
    if hasattr(lib, "lsr_set_option"):
        lib.lsr_set_option.argtypes = [ctypes.c_int, ctypes.c_int64]
        lib.lsr_set_option(3, 0 if split0[name] else 1)


def run(name, steps):
    lib = libs[name]
    _lib._lib = lib
    set_split(name)
    if modes[name] is not None:
        lib.lsr_set_option.argtypes = [ctypes.c_int, ctypes.c_int64]
        assert lib.lsr_set_option(_lib.LSR_OPT_BIN_MODE, modes[name]) == 0
    lib.lsr_profile_reset()
    lib.lsr_profile_enable(1)
    for _ in range(steps):
        for p in g.values():
            p.grad = None
        with torch.set_grad_enabled(not FWD_ONLY):
            c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                        language_feature_precomp=g["language_feature_precomp"], scales=g["scales"],
                        rotations=g["rotations"])
        if not FWD_ONLY:
            torch.autograd.backward([c, l], [dc, dl])
    torch.cuda.synchronize()
    lib.lsr_profile_enable(0)
    q = _lib.profile_query()
    return {k: ms / n for k, (ms, n) in q.items() if n}


def step_ms(name, steps):
    """Whole steps back to back, no stage events (what bench.py times)."""
    _lib._lib = libs[name]
    set_split(name)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        for p in g.values():
            p.grad = None
        with torch.set_grad_enabled(not FWD_ONLY):
            c, l, _ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                        language_feature_precomp=g["language_feature_precomp"], scales=g["scales"],
                        rotations=g["rotations"])
        if not FWD_ONLY:
            torch.autograd.backward([c, l], [dc, dl])
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / steps


res = {name: [] for name, _ in variants}
whole = {name: [] for name, _ in variants}
for name, _ in variants:
    run(name, 3)
    step_ms(name, 3)
for rnd in range(5):
    for name, _ in variants:
        res[name].append(run(name, 5))
        whole[name].append(step_ms(name, 10))
for name, _ in variants:
    stages = res[name][0].keys()
    med = {k: statistics.median(x[k] for x in res[name]) for k in stages}
    print(name, " ".join(f"{k}={v:.4f}" for k, v in med.items()), f"SUM={sum(med.values()):.4f}",
          f"STEP={statistics.median(whole[name]):.4f}")
