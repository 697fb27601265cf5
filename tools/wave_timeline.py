"""Wave timelines of the cfg3 training step's two render kernels (diagnostic
variant only: built by tools/variants/wave_timeline.py, which adds per-wave
s_memrealtime start/end stamps, the HW_ID / XCC_ID registers and a work count
to k_render_bwd_mf<16, ., LD, ., LST> (the block's list count) and to the
training forward k_render_fwd<., true> (the tile's instance count)).

Prints, per kernel: the span, the summed wave time against slots x span (how
much of the machine the waves keep busy), the tail (time from the last moment
the resident waves fill >= 90 % of their peak to the end), per-XCD spans and
work, and the wave-duration vs work fit.
Usage: python tools/wave_timeline.py LIB [OUT.json]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

lib = _lib.load(sys.argv[1])
_lib._lib = lib
lib.lsr_dbg_wave_tl.argtypes = [ctypes.c_void_p]
cfg = CONFIGS[int(os.environ.get("LSR_CFG", "3"))]
dev = torch.device("cuda:0")
cam = make_camera(cfg["W"], cfg["H"])
D = cfg["lang_dim"]
g0 = make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=D)
keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
g = {k: g0[k].to(dev).requires_grad_(True) for k in keys}
g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
r = GaussianRasterizer(bench.settings(cam, dev, 3, True))
dc = torch.randn(3, cfg["H"], cfg["W"], device=dev)
dl = torch.randn(D, cfg["H"], cfg["W"], device=dev)
T = ((cfg["W"] + 15) // 16) * ((cfg["H"] + 15) // 16)
nw = 4 * T
runs = []
for it in range(6):
    col, lang, *_ = r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
                      language_feature_precomp=g["language_feature_precomp"], scales=g["scales"],
                      rotations=g["rotations"])
    torch.autograd.grad([col, lang], [g[k] for k in keys] + [g["means2D"]], [dc, dl])
    torch.cuda.synchronize()
    buf = np.zeros(1 << 20, dtype=np.uint64)
    assert lib.lsr_dbg_wave_tl(buf.ctypes.data) == 0
    w = buf[(1 << 19):(1 << 19) + 4 * nw].reshape(nw, 4).astype(np.int64)
    wf = buf[:4 * nw].reshape(nw, 4).astype(np.int64)
    if it >= 2:
        runs.append((w, wf))

SLOTS = {"bwd": 256 * 16, "fwd": 256 * 24}   # resident waves at each kernel's occupancy (4 / 6 per SIMD)


def analyse(w, slots, work):
    t0, t1 = w[:, 0], w[:, 1]
    ok = t1 > 0
    w, t0, t1, work = w[ok], t0[ok], t1[ok], work[ok]
    base = t0.min()
    s, e = (t0 - base) * 10.0 / 1000.0, (t1 - base) * 10.0 / 1000.0   # 100 MHz -> us
    span = e.max()
    dur = e - s
    busy = dur.sum() / (slots * span)
    bins = np.arange(0.0, span + 0.25, 0.25)
    d = np.zeros(len(bins) + 1)
    np.add.at(d, np.searchsorted(bins, s), 1)
    np.add.at(d, np.searchsorted(bins, e), -1)
    act = np.cumsum(d)[:len(bins)]
    peak = act.max()
    full = np.nonzero(act >= 0.9 * peak)[0]
    tail = span - bins[full[-1]] if len(full) else span
    xcc = (w[:, 2] >> 32) & 0xF
    per_xcd = {int(x): round(float(e[xcc == x].max() - s[xcc == x].min()), 1) for x in np.unique(xcc)}
    A = np.vstack([np.ones_like(work), work]).T.astype(float)
    coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
    late = np.argsort(e)[-200:]
    return dict(waves=int(len(w)), span_us=round(float(span), 1), busy_frac=round(float(busy), 3),
                peak_resident=int(peak), tail_us=round(float(tail), 1),
                mean_wave_us=round(float(dur.mean()), 2), p99_wave_us=round(float(np.percentile(dur, 99)), 1),
                max_wave_us=round(float(dur.max()), 1),
                fit_us=dict(per_wave=round(float(coef[0]), 2), per_work=round(float(coef[1]), 4)),
                late_waves_mean_work=round(float(work[late].mean()), 1), mean_work=round(float(work.mean()), 2),
                work_per_xcd=[int(work[xcc == x].sum()) for x in range(8)], per_xcd_span_us=per_xcd)


out = []
for w, wf in runs:
    out.append(dict(bwd=analyse(w, SLOTS["bwd"], (w[:, 3] + 15) // 16),            # work: 16-candidate groups
                    fwd=analyse(wf, SLOTS["fwd"], wf[:, 3] & 0xFFFFFFFF)))         # work: tile instances
res = dict(what="k_render_bwd_mf<16,.,LD,.,LST> (bwd) and k_render_fwd<., true> (fwd) wave timelines at cfg%d" % int(os.environ.get("LSR_CFG", "3")),
           runs=out)
print(json.dumps(res, indent=1))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump(res, f, indent=1)
    np.save(sys.argv[2].replace(".json", ".npy"), runs[-1][0])
    np.save(sys.argv[2].replace(".json", "_fwd.npy"), runs[-1][1])
