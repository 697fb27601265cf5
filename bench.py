"""bench.py — headline benchmark of the MI355X-native language-Gaussian rasterizer.

Metric (BASELINE.json): frames/s fwd+bwd @ 1M Gaussians 1080p 3+16ch; achieved HBM GB/s.
Workload (BASELINE.json configs[2]): 1,000,000 synthetic Gaussians,
1920x1080, SH degree 3 + 16 dense language coefficients (top-4 soft codes), forward +
backward through the drop-in `diff_gaussian_rasterization` surface with EVERY input
requiring grad, upstream gradients ~ N(0,1).

One step = one view per GPU: forward + backward (+ for N > 1 the RCCL all-reduce(SUM) of
all per-Gaussian gradients — the data-parallel exchange of SURVEY.md §8e).  Views shard
one per rank (camera yaw depends on the rank), Gaussians are replicated: weak scaling.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints ONE JSON line.  Extra fields: per-stage HIP-event times (stages_ms), the
roofline of the dominant kernel, whole-step algorithmic HBM GB/s, forward FPS at 1.0 Mpix
(1280x800, the >=450 FPS target), and the CPU baseline (the oracle, timed on this host).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib, dp, layout, rasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402

METRIC = "frames/s fwd+bwd @ 1M Gaussians 1080p 3+16ch; achieved HBM GB/s"
HBM_PEAK_GBPS = 8000.0   # MI355X spec (MI355X_MICROARCH.md chip table)


def settings(cam, dev, sh_degree, include_feature):
    return GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
        projmatrix=cam["projmatrix"].to(dev), sh_degree=sh_degree, campos=cam["campos"].to(dev),
        prefiltered=False, debug=False, include_feature=include_feature, quick_render=False)


def algorithmic_bytes(g, rs, D, S):
    """Per-stage algorithmic HBM bytes of one forward+backward (with this
    build's record layout).  Instance terms use the instances the blend must visit:
    per tile, up to its largest n_contrib (+1 terminating), rounded to the 256-batch."""
    N = g["means3D"].shape[0]
    e = torch.empty(0, device=g["means3D"].device)
    _, _, radii, M, bufs, _, _ = rasterizer._run_forward(
        g["means3D"], g.get("shs", e), g.get("colors_precomp", e), g.get("language_feature_precomp", e), e, e,
        g["opacities"], g.get("scales", e), g.get("rotations", e), e, rs)
    W, H = rs.image_width, rs.image_height
    dec = layout.decode(bufs, N, W, H, M)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    nc = dec["n_contrib"]
    pad = torch.zeros((gy * 16, gx * 16), dtype=nc.dtype, device=nc.device)
    pad[:H, :W] = nc
    tmax = pad.view(gy, 16, gx, 16).amax(dim=(1, 3)).reshape(-1).to(torch.int64)
    cnt = (dec["ranges"][:, 1] - dec["ranges"][:, 0]).to(torch.int64)
    staged_f = torch.minimum(cnt, ((tmax + 1 + 255) // 256) * 256).sum().item()
    staged_b = torch.minimum(cnt, ((tmax + 255) // 256) * 256).sum().item()
    vis = int((radii > 0).sum().item())
    P = W * H
    T = gx * gy
    C = 3 + D
    inst = 4 + 32 + 4 * C     # point_list id + splat record + feature row
    VP = ((12 + D) + 31) // 32 * 32
    chunk = max(1024, (N + 511) // 512)
    chunk = (chunk + 255) // 256 * 256
    B = (N + chunk - 1) // chunk
    b = {
        "preprocess": N * (12 + 12 + 16 + 4 + 4 * S) + N * (16 + 16 + 12 + 4 + 4 + 4 + 4),
        "bin_count": N * 4 + vis * 16 + B * T * 4 * 3 + T * 4,
        "scan_tile_counts": T * 12,
        "bin_scatter": N * 4 + vis * (16 + 4) + B * T * 4 + T * 4 + M * 8,
        "tile_sort": M * (8 + 4),
        "render_fwd": staged_f * inst + T * 8 + P * (4 * C + 8),
        "grad_zero": N * VP * 4,
        "render_bwd": staged_b * inst + T * 8 + P * (4 * C + 8) + vis * (9 + D) * 4,
        "preprocess_bwd": N * ((9 + D) * 4 + 12 + 12 + 16 + 4 * S + 4 + 4) + N * (12 + 4 + 4 * D + 12 + 4 * S + 12 + 16),
    }
    return b, dict(num_rendered=M, visible=vis, staged_fwd=staged_f, staged_bwd=staged_b,
                   mean_n_contrib=float(nc.float().mean().item()))


def pmc_traffic(stage):
    """Measured HBM bytes per launch of `stage`'s kernel from the newest committed
    profiles/r*_pmc_traffic.json (tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes over tools/pmc_step.py = this workload, gfx950-corrected)."""
    import glob
    import re
    # natural order: r01v10 after r01v9
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))])
    if not files:
        return None, None
    with open(files[-1]) as f:
        doc = json.load(f)
    ks = [v for k, v in doc["kernels"].items()
          if k == "k_" + stage or k.startswith("k_" + stage + "<") or k.startswith("k_" + stage + "_mf<")]
    if not ks:
        return None, None
    return int(sum(v["traffic_bytes"] for v in ks)), os.path.relpath(files[-1], ROOT)


def cpu_baseline(cam, gcpu, D, budget_tiles=2048):
    """The oracle (C restatement, single thread) on a bounded sample of the same frame:
    full preprocess + binning + preprocess-bwd, render fwd+bwd on `budget_tiles` seeded
    tiles, the render part extrapolated by T / budget_tiles."""
    from oracle import oracle as O
    O.build()
    pb = O.Problem(cam, gcpu)
    lib = O.load()
    T = pb.gx * pb.gy
    rng = np.random.default_rng(0)
    tiles = np.sort(rng.choice(T, size=min(budget_tiles, T), replace=False)).astype(np.int32)
    t0 = time.perf_counter()
    f = O.forward(pb, nthreads=1, tiles=np.zeros(0, np.int32))   # preprocess + binning only
    t1 = time.perf_counter()
    f2 = O.forward(pb, nthreads=1, tiles=tiles)
    t2 = time.perf_counter()
    t_pre_bin = t1 - t0
    t_rf = (t2 - t1) - t_pre_bin        # f2 repeats preprocess+binning; subtract it
    dcol = rng.standard_normal((3, pb.H, pb.W)).astype(np.float32)
    dlang = rng.standard_normal((pb.D, pb.H, pb.W)).astype(np.float32) if pb.D else None
    t3 = time.perf_counter()
    O.backward(pb, f2, dcol, dlang, tiles=tiles)
    t4 = time.perf_counter()
    t_bwd_sample = t4 - t3              # render bwd on the sample + full preprocess bwd
    scale = T / len(tiles)
    t_frame = t_pre_bin + max(t_rf, 0.0) * scale + t_bwd_sample * scale
    del f
    return dict(value=1.0 / t_frame, unit="frames/s", cores=1, kind="port",
                sample=f"oracle/lsr_oracle.c single-threaded: full preprocess+binning ({t_pre_bin:.2f}s), render "
                       f"fwd {len(tiles)}/{T} seeded tiles ({max(t_rf, 0):.2f}s), render bwd + preprocess bwd on "
                       f"the same tiles ({t_bwd_sample:.2f}s); render + bwd extrapolated x{scale:.1f}",
                seconds_per_frame=t_frame)


def fwd_fps(g, dev, sh_degree, D, W=1280, H=800, iters=20):
    cam = make_camera(W, H)
    rs = settings(cam, dev, sh_degree, D > 0)
    r = GaussianRasterizer(rs)
    with torch.no_grad():
        for _ in range(3):
            r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
              language_feature_precomp=g.get("language_feature_precomp"), scales=g["scales"],
              rotations=g["rotations"])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
              language_feature_precomp=g.get("language_feature_precomp"), scales=g["scales"],
              rotations=g["rotations"])
        torch.cuda.synchronize()
    return iters / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=[3])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fwd-1mpix", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    _lib.load()

    cfg = CONFIGS[args.config]
    N, W, H, D, deg = cfg["N"], cfg["W"], cfg["H"], cfg["lang_dim"], cfg["sh_degree"]
    # one view per rank: yaw offsets within +-20 degrees, Gaussians replicated (seed 0)
    yaw = dp.rank_yaw(rank, world)
    cam0 = make_camera(W, H)
    cam = make_camera(W, H, yaw_deg=yaw)
    gcpu = make_gaussians(N, cam0, seed=0, sh_degree=deg, lang_dim=D)
    leaf_keys = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
    g = {k: gcpu[k].to(dev).requires_grad_(True) for k in leaf_keys}
    g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
    params = [g[k] for k in leaf_keys] + [g["means2D"]]
    gen = torch.Generator(device="cpu").manual_seed(1 + rank)
    dcolor = torch.randn((3, H, W), generator=gen).to(dev)
    dlang = torch.randn((D, H, W), generator=gen).to(dev)
    rs = settings(cam, dev, deg, True)
    rast = GaussianRasterizer(rs)
    leaves = [g[k] for k in leaf_keys]
    exch = dp.ViewShardedExchange(leaves, with_stats=True) if world > 1 else None

    def step():
        for p in params:
            p.grad = None
        color, lang, radii = rast(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"],
                                  shs=g["shs"], language_feature_precomp=g["language_feature_precomp"],
                                  scales=g["scales"], rotations=g["rotations"])
        torch.autograd.backward([color, lang], [dcolor, dlang])
        if exch is not None:
            # one flat all-reduce(SUM) of every gradient + densification stats, one MAX of radii
            exch.exchange([p.grad for p in leaves], g["means2D"].grad, radii)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # per-stage breakdown: a separate untimed pass with every stage bracketed
    # by events (each bracket idles the stream a few us, so the timed region
    # below brackets only the dominant stage, for the live roofline)
    _lib.profile_stages(None)
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(max(2, min(args.steps, 5))):
        step()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    stages = _lib.profile_query()
    per_stage = {k: dict(ms_per_launch=(ms / calls if calls else 0.0), launches=calls)
                 for k, (ms, calls) in stages.items() if calls}
    dom = max(per_stage, key=lambda k: per_stage[k]["ms_per_launch"])
    if world > 1:
        dist.barrier()
    _lib.profile_stages([dom])
    _lib.profile_reset()
    _lib.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _lib.profile_enable(False)
    _lib.profile_stages(None)
    dom_ms_s, dom_calls = _lib.profile_query()[dom]
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        frames = world * args.steps
        value = frames / elapsed
        with torch.no_grad():
            gd = {k: v.detach() for k, v in g.items()}
            bytes_, info = algorithmic_bytes(gd, rs, D, 48)
        dom_ms = dom_ms_s / dom_calls if dom_calls else 0.0
        dom_gbps = bytes_[dom] / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(dom)
        step_ms = elapsed / args.steps * 1e3
        kernel_ms = sum(v["ms_per_launch"] for v in per_stage.values())
        total_bytes = sum(bytes_.values())
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded; SURVEY.md §8d generator)",
            "config": {
                "workload": "BASELINE cfg3: 1M Gaussians, 1920x1080, SH deg 3 + 16 dense language channels, "
                            "fwd+bwd, all inputs require grad; 1 view per GPU",
                "gaussians": N, "width": W, "height": H, "lang_dim": D, "sh_degree": deg,
                "global_batch": world, "parallelism": f"dp{world} (views sharded, RCCL all-reduce of grads)"
                if world > 1 else "single GPU",
            },
            "exchange": ({"bucket_bytes": exch.bucket.nbytes, **dp.allreduce_bound_ms(exch.bucket.nbytes, world)}
                         if exch is not None else None),
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(dom_gbps, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(dom_gbps / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": int(bytes_[dom]),
                "ms_per_launch": round(dom_ms, 4),
                "launches_timed": dom_calls,
            },
            "hbm_step": {"algorithmic_bytes": int(total_bytes),
                         "GBps_over_kernels": round(total_bytes / (kernel_ms * 1e-3) / 1e9, 1) if kernel_ms else 0,
                         "GBps_over_step": round(total_bytes / (step_ms * 1e-3) / 1e9, 1)},
            "stages_ms": {k: round(v["ms_per_launch"], 4) for k, v in per_stage.items()},
            "stage_bytes": {k: int(v) for k, v in bytes_.items()},
            "workload_stats": info,
        }
        if world == 1 and not args.no_fwd_1mpix:
            gg = dict(g)
            out["fwd_fps_1mpix"] = round(fwd_fps({k: v.detach() for k, v in gg.items()}, dev, deg, D), 1)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cam, gcpu, D)
            out["cpu_baseline"]["value"] = round(out["cpu_baseline"]["value"], 5)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
