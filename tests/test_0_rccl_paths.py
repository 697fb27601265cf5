"""The RCCL branches of the view-sharded exchange, executed on a one-GPU box
(VERDICT r03 next #7).

bench.py's multi-GPU step (`--gpus N`, BASELINE cfg3/cfg4's exchange:
train.py:250-263's accumulation over views) runs `dp.ViewShardedExchange`
over the `nccl` backend, which is RCCL on ROCm: the language bucket's
all-reduce started on a side stream from the library's lang-ready event
(`_launch_early`), the main bucket's all-reduce, the view-factored SH
gradient rebuilt from all-gathered colour gradients and camera centres
(`_factored_sh`, `all_gather` into `unbind` views) and the MAX of the radii.
A test box has one GPU, so the exchange is built with `force_collectives=True`
on a world-size-1 RCCL group: every collective branch executes on RCCL, and
the reduced buckets must equal the same step's gradients computed without any
exchange (a sum over one rank), within the GRAD tolerance (the render
backward's float atomics reorder between the two backward calls); the
factored SH gradient must equal the backward's own dL/dSH.  A second worker
runs the identical forced exchange on a gloo group and the two backends'
buckets are compared the same way.

Named to be collected early: the parent never touches the GPU; the workers
are spawned processes."""
import os
import socket
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
W, H, N, D = 256, 192, 20000, 16
KEYS = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _step_inputs(dev):
    sys.path.insert(0, ROOT)
    from langsplatv2_amd.scenes import make_camera, make_gaussians
    cam = make_camera(W, H, yaw_deg=5.0)
    g = make_gaussians(N, cam, seed=21, sh_degree=3, lang_dim=D)
    leaves = [g[k].to(dev).contiguous().requires_grad_(True) for k in KEYS]
    gen = torch.Generator().manual_seed(3)
    dC = torch.randn((3, H, W), generator=gen).to(dev)
    dL = torch.randn((D, H, W), generator=gen).to(dev)
    return cam, leaves, dC, dL


def _forward(cam, leaves, dev):
    import bench
    from diff_gaussian_rasterization import GaussianRasterizer
    rs = bench.settings(cam, dev, 3, True)
    m2d = torch.zeros_like(leaves[0], requires_grad=True)
    color, lang, radii = GaussianRasterizer(rs)(means2D=m2d, **dict(zip(KEYS, leaves)))
    return rs, color, lang, radii, m2d


def _worker(backend, port, outdir):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from langsplatv2_amd import dp
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        cam, leaves, dC, dL = _step_inputs(dev)
        # the same step without any exchange
        rs, color, lang, radii, m2d = _forward(cam, leaves, dev)
        local = torch.autograd.grad([color, lang], leaves + [m2d], [dC, dL])
        local_stats = dp.densify_increment(local[-1], radii)
        # bench.py's zero-copy exchange, every collective branch forced
        ex = dp.ViewShardedExchange(leaves, with_stats=True, names=list(KEYS), force_collectives=True)
        assert ex.world == 1 and ex.collective and ex.sh_idx is not None and ex.early is not None
        rs, color, lang, radii, m2d = _forward(cam, leaves, dev)
        with ex.sink() as sink:
            grads = torch.autograd.grad([color, lang], leaves + [m2d], [dC, dL])
        assert "language_feature_precomp" in sink.used and "shs" in sink.used
        early_started = ex._early_work is not None        # _launch_early ran from the lang-ready callback
        red, stats, max_r = ex.finish(grads[-1], radii, grads[:-1], campos=rs.campos, means3D=leaves[0].detach(),
                                      sh_degree=3)
        torch.cuda.synchronize()
        torch.save({"red": [r.detach().cpu() for r in red], "local": [g.detach().cpu() for g in local[:-1]],
                    "stats": stats.cpu(), "local_stats": local_stats.cpu(), "max_r": max_r.cpu(),
                    "radii": radii.cpu(), "early_started": early_started,
                    "side_stream": ex._side is not None, "backend": dist.get_backend()},
                   os.path.join(outdir, f"{backend}.pt"))
    finally:
        dist.destroy_process_group()


def _close(name, x, z):
    scale = max(1.0, float(z.abs().max()))
    err = float((x - z).abs().max())
    assert err <= 1e-6 + 1e-5 * scale, f"{name}: {err:.3e} vs tolerance {1e-6 + 1e-5 * scale:.3e}"


def test_rccl_exchange_branches_world1(tmp_path):
    import torch.multiprocessing as mp
    if torch.cuda.device_count() == 0:
        pytest.skip("no ROCm GPU visible")
    ctx = mp.get_context("spawn")
    out = str(tmp_path)
    res = {}
    for backend in ("nccl", "gloo"):
        p = ctx.Process(target=_worker, args=(backend, _free_port(), out))
        p.start()
        p.join(timeout=150)
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, f"{backend} worker exit code {p.exitcode}"
        res[backend] = torch.load(os.path.join(out, f"{backend}.pt"), weights_only=True)
    r = res["nccl"]
    assert r["backend"] == "nccl" and r["early_started"] and r["side_stream"]
    for name, x, z in zip(KEYS, r["red"], r["local"]):
        _close(name, x, z)
    assert float(r["local"][1].abs().max()) > 1e-3          # the factored SH gradient is exercised
    assert float(r["local"][5].abs().max()) > 1e-3          # the early (language) bucket too
    torch.testing.assert_close(r["stats"], r["local_stats"], rtol=1e-5, atol=1e-7)
    assert torch.equal(r["max_r"], r["radii"])
    g = res["gloo"]
    for name, x, y in zip(KEYS, r["red"], g["red"]):
        _close(name + " (nccl vs gloo)", x, y)
    torch.testing.assert_close(r["stats"], g["stats"], rtol=1e-5, atol=1e-7)
