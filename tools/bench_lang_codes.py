"""Fused top-k soft-code producer vs the reference's PyTorch op chain
(utils/vq_utils.py:9-40, run with torch on the same GPU) at 1M Gaussians.
Algorithmic bytes: dense fwd 4K read + 4K write per row; bwd 8K read
(logits + grad) + 4K write; sparse 4K read + 8k write (weights + fp32 idx).
Prints one JSON line.  Usage: python tools/bench_lang_codes.py [N]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langsplatv2_amd import lang_codes, scenes  # noqa: E402

HBM = 8000.0


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(0)
    res = {"N": N}
    for L, K, k in ((1, 64, 4), (3, 64, 4)):
        x = torch.randn(N, L * K, generator=gen).to(dev)
        g = torch.randn(N, L * K, generator=gen).to(dev)
        xr = x.clone().requires_grad_(True)
        rows = N * L
        fwd = timed(lambda: lang_codes.get_render_weights(x, L, K, k))
        y = lang_codes.get_render_weights(xr, L, K, k)
        bwd = timed(lambda: torch.autograd.grad(y, xr, g, retain_graph=True))
        sp = timed(lambda: lang_codes.quick_inputs(x, k, levels=L))

        def ref_fwd():
            return torch.cat([scenes.softmax_to_topk_soft_code(xr[:, i * K:(i + 1) * K], k) for i in range(L)], -1)

        yr = ref_fwd()
        t_ref_fwd = timed(lambda: ref_fwd())
        t_ref_bwd = timed(lambda: torch.autograd.grad(yr, xr, g, retain_graph=True))

        def ref_sparse():
            ws, ids = [], []
            for i in range(L):
                w, idx = scenes.get_weights_and_indices(x[:, i * K:(i + 1) * K], k)
                ws.append(w)
                ids.append(idx + i * K)
            return torch.cat(ws, 1), torch.cat(ids, 1)

        t_ref_sp = timed(ref_sparse, reps=5)
        b_f, b_b, b_s = rows * K * 8, rows * K * 12, rows * (K * 4 + 8 * k)
        res[f"L{L}K{K}k{k}"] = {
            "dense_fwd_ms": round(fwd, 4), "dense_fwd_GBps": round(b_f / fwd / 1e6, 1),
            "dense_fwd_frac": round(b_f / fwd / 1e6 / HBM, 3),
            "bwd_ms": round(bwd, 4), "bwd_GBps": round(b_b / bwd / 1e6, 1), "bwd_frac": round(b_b / bwd / 1e6 / HBM, 3),
            "sparse_ms": round(sp, 4), "sparse_GBps": round(b_s / sp / 1e6, 1),
            "torch_ref_fwd_ms": round(t_ref_fwd, 4), "torch_ref_bwd_ms": round(t_ref_bwd, 4),
            "torch_ref_sparse_ms": round(t_ref_sp, 4),
        }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
