"""Quick-path frame stream: render + decode of F frames, sequential on one
stream vs pipelined over two (frame i's decode overlapping frame i+1's render),
at bench.py's quick_1mpix workload.  The render is latency-bound and the decode
HBM-bound; the pipelined form only helps if the decode, running on part of the
chip, keeps its bandwidth.  Usage: python tools/pipe_quick.py [lib.so] (with
the decncu A/B build, LSR_DEC_NCU sets the decode's CU count)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib, quick  # noqa: E402
from langsplatv2_amd.scenes import make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

if len(sys.argv) > 1:
    _lib._lib = _lib.load(sys.argv[1])
dev = torch.device("cuda:0")
W, H, N = 1280, 800, 1_000_000
cam = make_camera(W, H)
g = make_gaussians(N, cam, seed=0, sh_degree=3, quick_k=4)
t = {k: v.to(dev) for k, v in g.items() if isinstance(v, torch.Tensor)}
r = GaussianRasterizer(bench.settings(cam, dev, 3, False, quick=True, quick_layout=os.environ.get("LSR_AB_LAYOUT", "hwc")))
z = torch.zeros_like(t["means3D"])
cb = torch.randn(3, 64, 512, device=dev)


def render():
    with torch.no_grad():
        return r(means3D=t["means3D"], means2D=z, opacities=t["opacities"], shs=t["shs"],
                 language_feature_weights_quick=t["language_feature_weights_quick"],
                 language_feature_indices=t["language_feature_indices"], scales=t["scales"],
                 rotations=t["rotations"])[1]


def sequential(F):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(F):
        quick.decode_language_features(render(), cb)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / F


s_r, s_d = torch.cuda.Stream(), torch.cuda.Stream()


def pipelined(F):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(F):
        with torch.cuda.stream(s_r):
            m = render()
            ev = torch.cuda.Event()
            ev.record(s_r)
        with torch.cuda.stream(s_d):
            s_d.wait_event(ev)
            quick.decode_language_features(m, cb)
            m.record_stream(s_d)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / F


fs = quick.QuickFeatureStream(cb)


def qfs(F):
    """quick.QuickFeatureStream from the caller's (default) stream."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(F):
        fs.push(render)
    fs.flush()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / F


s_c = torch.cuda.Stream()


def qfs_side(F):
    """The same with the caller on a side stream."""
    with torch.cuda.stream(s_c):
        return qfs(F)


modes = {"seq": sequential, "pipe": pipelined, "qfs": qfs, "qfs_side": qfs_side}
for _ in range(3):
    for f in modes.values():
        f(3)
res = {k: [] for k in modes}
for rnd in range(5):
    for k, f in modes.items():
        res[k].append(f(20))
import statistics  # noqa: E402
ncu = os.environ.get("LSR_DEC_NCU", "all")
print(f"dec_cus={ncu} " + " ".join(f"{k}_ms={1e3 * statistics.median(v):.4f} fps={1 / statistics.median(v):.1f}"
                                    for k, v in res.items()))
