"""distCUDA2 timing at SfM-like sizes (clustered clouds with outliers and a
uniform cloud).  Prints one JSON line.  Usage: python tools/bench_knn.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_knn._C import distCUDA2  # noqa: E402
from langsplatv2_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    res = {}
    for n, kind in ((100_000, "uniform"), (1_000_000, "uniform"), (1_000_000, "clusters"), (4_000_000, "clusters")):
        g = np.random.default_rng(0)
        if kind == "uniform":
            p = g.uniform(-10, 10, (n, 3))
        else:
            c = g.uniform(-50, 50, (20, 3))
            p = c[g.integers(0, 20, n)] + 0.05 * g.standard_normal((n, 3))
            p[: n // 100] = g.uniform(-1000, 1000, (n // 100, 3))
        x = torch.from_numpy(p.astype(np.float32)).to(dev)
        distCUDA2(x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            distCUDA2(x)
        e.record()
        torch.cuda.synchronize()
        res[f"{kind}_{n}"] = round(s.elapsed_time(e) / 5, 3)
    print(json.dumps({"distCUDA2_ms": res}))


if __name__ == "__main__":
    _lib.load()
    main()
