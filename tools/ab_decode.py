"""A/B timing of the quick-path codebook decode (3 x 64 x 512, L2-normalised) of liblsr
variants in one process, 1280x800 and 1920x1080 weight maps.
Usage: python tools/ab_decode.py name=path.so ..."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import _lib, quick  # noqa: E402

NORM = os.environ.get("LSR_DEC_NORM", "1") == "1"
variants = [a.split("=", 1) for a in sys.argv[1:]]
libs = {n: _lib.load(p) for n, p in variants}
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
cb = torch.randn(3, 64, 512, generator=g).to(dev)
for (W, H) in ((1280, 800), (1920, 1080)):
    wm = (torch.rand(192, H, W, generator=g) * (torch.rand(192, H, W, generator=g) < 0.1)).to(dev)
    res = {n: [] for n, _ in variants}
    for rnd in range(6):
        for n, _ in variants:
            _lib._lib = libs[n]
            quick.decode_language_features(wm, cb, normalize=NORM)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                quick.decode_language_features(wm, cb, normalize=NORM)
            torch.cuda.synchronize()
            if rnd:
                res[n].append((time.perf_counter() - t0) / 10 * 1e3)
    print(f"{W}x{H}: " + "  ".join(f"{n}={statistics.median(v):.3f}ms ({3 * 512 * W * H * 4 / (statistics.median(v) * 1e-3) / 1e9:.0f} GB/s)" for n, v in res.items()))
