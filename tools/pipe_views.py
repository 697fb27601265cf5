"""cfg5 forwards over a stream of views: one at a time, two in flight from one host
thread (view_stream.ViewStream), and two in flight from two host threads (each
with its own non-blocking stream; the library's per-thread state allows it)."""
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
from langsplatv2_amd.view_stream import ViewStream  # noqa: E402
import bench  # noqa: E402

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "5"))]
dev = torch.device("cuda:0")
cam = make_camera(cfg["W"], cfg["H"])
g = {k: v.to(dev) for k, v in make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=cfg["lang_dim"]).items()
     if isinstance(v, torch.Tensor)}
r = GaussianRasterizer(bench.settings(cam, dev, 3, cfg["lang_dim"] > 0))
z = torch.zeros_like(g["means3D"])


def fwd():
    with torch.no_grad():
        return r(means3D=g["means3D"], means2D=z, opacities=g["opacities"], shs=g["shs"],
                 language_feature_precomp=g.get("language_feature_precomp"), scales=g["scales"],
                 rotations=g["rotations"])


def seq(F):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(F):
        fwd()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / F


vs = ViewStream(dev)


def one_thread(F):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(F):
        vs.push(fwd)
    vs.flush()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / F


streams = [_lib.nonblocking_stream(dev) for _ in range(2)]


def two_threads(F):
    torch.cuda.synchronize()

    def work(k):
        torch.cuda.set_device(dev)
        with torch.cuda.stream(streams[k]):
            for _ in range(F // 2):
                fwd()
    t = time.perf_counter()
    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / F


for f in (seq, one_thread, two_threads):
    f(4)
res = {f.__name__: [] for f in (seq, one_thread, two_threads)}
for _ in range(3):
    for f in (seq, one_thread, two_threads):
        res[f.__name__].append(f(20))
import statistics  # noqa: E402
print(" ".join(f"{k}={1e3 * statistics.median(v):.3f}ms ({1 / statistics.median(v):.1f} fps)" for k, v in res.items()))
