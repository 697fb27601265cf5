"""bench.py — headline benchmark of the MI355X-native language-Gaussian rasterizer.

Metric (BASELINE.json): frames/s fwd+bwd @ 1M Gaussians 1080p 3+16ch; achieved HBM GB/s.
Workload (BASELINE.json configs[2]): 1,000,000 synthetic Gaussians,
1920x1080, SH degree 3 + 16 dense language coefficients (top-4 soft codes), forward +
backward through the drop-in `diff_gaussian_rasterization` surface with EVERY input
requiring grad, upstream gradients ~ N(0,1).

One step = one view per GPU: forward + backward (+ for N > 1 the RCCL all-reduce(SUM) of
all per-Gaussian gradients — the data-parallel exchange of SURVEY.md §8e, written straight
into the all-reduce buckets, the language bucket started while preprocess_bwd still runs).
Views shard one per rank (camera yaw depends on the rank), Gaussians are replicated: weak
scaling.

  python bench.py [--gpus N --steps K --warmup W]
      N > 1 without WORLD_SIZE in the environment: bench.py starts N ranks itself (a
      torch.distributed.run child, before any GPU call) and exits with its status
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
  python bench.py --gpus 2 --dry-run     # ranks come up on gloo, agree on the world size; no GPU

Rank 0 prints ONE JSON line.  Extra fields: per-stage HIP-event times (stages_ms), the
roofline of the dominant kernel (SURVEY §8d algorithmic bytes / HIP-event time), whole-step
algorithmic HBM GB/s, forward FPS at 1.0 Mpix (1280x800, the >=450 FPS target), the quick
(sparse 192-channel) render + codebook decode FPS at 1 Mpix, and the CPU baseline (the
oracle's C restatement on the host's cores).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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


def settings(cam, dev, sh_degree, include_feature, quick=False, quick_dim=None, quick_layout=None):
    return GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
        projmatrix=cam["projmatrix"].to(dev), sh_degree=sh_degree, campos=cam["campos"].to(dev),
        prefiltered=False, debug=False, include_feature=include_feature, quick_render=quick,
        language_feature_dim=quick_dim, language_feature_layout=quick_layout)


def algorithmic_bytes(g, rs, D, S):
    """Per-stage algorithmic HBM bytes of one forward+backward, SURVEY.md §8d's formula
    (M = measured num_rendered, C = 3 + D, S SH floats), mapped onto this build's stages:
      preprocess     N(44+4S) + 75N
      bin_count      8N [scan] + 20N [duplicate's per-Gaussian reads]
      bin_scatter    12M [duplicate's per-instance key/value writes]
      tile_sort      24M [sort] + 8M [ranges]
      scan_tile_counts 8T [ranges]
      render_fwd     M(28+4C) + P(4C+8)
      render_bwd     M(28+4C) + 8T + P(4C+8) + N(24+4C)
      preprocess_bwd N(12+12+16+4S+4+24+12+8+12+3) + N(12+12+16+4S+12)
      grad_zero      0 (an implementation memset, no §8d term)
    Also returns the instances the blend actually visits ("staged": per tile up to its
    largest n_contrib, rounded to the 256-batch) for context."""
    N = g["means3D"].shape[0]
    e = torch.empty(0, device=g["means3D"].device)
    _, _, radii, M, bufs, _, _, _ = rasterizer._run_forward(
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
    # the reference's instance count for the same frame (its 3-sigma rect lists, A.2);
    # this build's binning drops the instances whose cut ellipse misses the tile
    M_ref = int(dec["tiles_touched"].to(torch.int64)[radii > 0].sum().item())
    P = W * H
    T = gx * gy
    C = 3 + D
    b = {
        "preprocess": N * (44 + 4 * S) + N * 75,
        "bin_count": N * 8 + N * 20,
        "scan_tile_counts": T * 8,
        "bin_scatter": M * 12,
        "tile_sort": M * 24 + M * 8,
        "render_fwd": M * (28 + 4 * C) + P * (4 * C + 8),
        "grad_zero": 0,
        "render_bwd": M * (28 + 4 * C) + T * 8 + P * (4 * C + 8) + N * (24 + 4 * C),
        "preprocess_bwd": N * (12 + 12 + 16 + 4 * S + 4 + 24 + 12 + 8 + 12 + 3) + N * (12 + 12 + 16 + 4 * S + 12),
    }
    return b, dict(num_rendered=M, num_rendered_reference=M_ref, visible=vis, staged_fwd=staged_f,
                   staged_bwd=staged_b, mean_n_contrib=float(nc.float().mean().item()))


def pmc_traffic(stage, prefix="r"):
    """Measured HBM bytes per launch of `stage`'s kernel from the newest committed
    profiles/<prefix>*_pmc_traffic.json (tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes over tools/pmc_step.py = this workload, gfx950-corrected); the
    cfg5 line reads the cfg5_r* files (pmc_step.py with LSR_CFG=5)."""
    import glob
    import re
    # natural order: r01v10 after r01v9
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", prefix + "*_pmc_traffic.json")),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))])
    if not files:
        return None, None
    with open(files[-1]) as f:
        doc = json.load(f)
    ks = [v for k, v in doc["kernels"].items()
          if k == "k_" + stage or k.startswith("k_" + stage + "<") or k.startswith("k_" + stage + "_")]
    if not ks:
        return None, None
    return int(sum(v["traffic_bytes"] for v in ks)), os.path.relpath(files[-1], ROOT)


ROOF_EVERY = 4   # timed-region steps per event-bracketed launch of the roofline kernel
# chip-wide rate of memory-side float atomics (global_atomic_add_f32), bytes added per
# second: /opt/skills/guides/MI355X_MICROARCH.md, "Global float atomics" (1.26-1.36 TB/s)
ATOMIC_PEAK_GBPS = 1300.0


def atomic_floor(stage, ms_per_launch, prefix="r"):
    """render_bwd writes only through memory-side float atomics (the gradient rows):
    its PMC WRITE_SIZE bytes at the chip's atomic rate give a time floor that, unlike
    the HBM roofline, the kernel runs close to."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", prefix + "*_pmc_traffic.json")),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))])
    if not files or ms_per_launch <= 0:
        return None
    with open(files[-1]) as f:
        doc = json.load(f)
    ks = [v for k, v in doc["kernels"].items() if k.startswith("k_" + stage + "<") or k.startswith("k_" + stage + "_")]
    if not ks or "write_bytes" not in ks[0]:
        return None
    wb = int(sum(v["write_bytes"] for v in ks))
    floor_ms = wb / (ATOMIC_PEAK_GBPS * 1e9) * 1e3
    return {"write_bytes": wb, "ceiling_GBps": ATOMIC_PEAK_GBPS, "floor_ms": round(floor_ms, 4),
            "frac": round(floor_ms / ms_per_launch, 4), "source": os.path.relpath(files[-1], ROOT),
            "note": "all of the kernel's HBM writes are buffer/global_atomic_add_f32 into gradient rows; "
                    "rate from MI355X_MICROARCH.md (global float atomics, chip-wide)"}

def rocprof_avg(stage):
    """The stage kernel's average duration under rocprofv3 --kernel-trace --stats from the
    newest committed profile of the cfg3 step ALONE (profiles/r*_kernel_stats.md written by
    `tools/pass.py TAG prof`, title "(cfg3 step alone)"): the HIP-event roofline time's
    cross-check."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats.md")),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))])
    kn = STAGE_KERNEL.get(stage, "k_" + stage)
    for fn in reversed(files):
        with open(fn) as f:
            lines = f.read().splitlines()
        if not lines or "(cfg3 step alone)" not in lines[0]:
            continue
        rows = []
        for ln in lines:
            m = re.match(r"\| `(?:lsr::)?([^`]+)` \| (\d+) \| ([\d.]+) \| ([\d.]+) \|", ln)
            if m and (m.group(1) == kn or m.group(1).startswith(kn + "<")):
                rows.append((float(m.group(3)), m.group(1), int(m.group(2)), float(m.group(4))))
        if rows:
            tot, name, calls, avg = max(rows)
            return {"kernel": name, "avg_ms": round(avg / 1e3, 4), "calls": calls,
                    "source": os.path.relpath(fn, ROOT)}
    return None


STAGE_KERNEL = {"render_bwd": "k_render_bwd_mf", "render_fwd": "k_render_fwd", "preprocess": "k_preprocess",
                "preprocess_bwd": "k_preprocess_bwd", "bin_scatter": "k_bin_scatter", "bin_count": "k_bin_count",
                "tile_sort": "k_tile_sort"}


def pmc_issue(stage, prefix="r"):
    """Issue-rate roofline of `stage`'s kernel from the newest committed
    profiles/<prefix>*_pmc_issue.json (tools/pmc_issue.py over two rocprofv3 SQ passes of
    tools/pmc_step.py = this workload): VALU pipe issue fraction (wave64 VALU = 2 SIMD-32
    cycles), MFMA busy fraction, waves per SIMD, the wave-cycle split (issuing / issue-stalled
    / in s_waitcnt) and instructions per staged (candidate, 8x8-block) pair."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", prefix + "*_pmc_issue.json")),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))])
    if not files:
        return None
    with open(files[-1]) as f:
        doc = json.load(f)
    kn = STAGE_KERNEL.get(stage, "k_" + stage)
    ks = sorted(((k, v) for k, v in doc["kernels"].items() if k == kn or k.startswith(kn + "<")),
                key=lambda kv: -kv[1]["derived"].get("kernel_cycles", 0))
    if not ks:
        return None
    k, v = ks[0]
    d = v["derived"]
    keep = ("valu_issue_frac", "mfma_busy_frac", "valu_active_frac", "salu_issue_frac", "waves_per_simd",
            "wave_issuing_frac", "wave_issue_stalled_frac", "wave_in_waitcnt_frac", "units_per_dispatch",
            "valu_per_unit", "mfma_per_unit", "salu_per_unit", "lds_per_unit")
    out = {"kernel": k, **{x: d[x] for x in keep if x in d}}
    out["bound"] = "issue/latency" if max(d.get("valu_issue_frac", 0), d.get("mfma_busy_frac", 0)) < 0.6 else "issue"
    out["source"] = os.path.relpath(files[-1], ROOT)
    out["units"] = "unit = one staged (candidate, 8x8-block) pair (tools/bwd_work.py census)"
    return out


def host_threads() -> int:
    """CPU threads this process may use: the box's share (OMP_NUM_THREADS is set to it on the
    GPU pool; os.cpu_count() reports the whole machine there), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cam, gcpu, D, cfg_name="cfg3", backward=True, tile_sample=None):
    """The oracle (oracle/lsr_oracle.c: the naive per-pixel serial blend, per-tile loops) on
    the host's cores, the WHOLE frame (or, with `tile_sample`, that many seeded tiles, the
    render time scaled by T / sample -- flagged extrapolated): preprocess + binning
    (single-threaded in the oracle), render forward over the tiles on `threads` OpenMP
    threads, and with `backward` the render backward on the same threads (fp64 atomic
    accumulation) + preprocess backward.  kind "port": the reference's CUDA rasterizer
    source is absent, this is its restatement."""
    from oracle import oracle as O
    O.build()
    threads = host_threads()
    pb = O.Problem(cam, gcpu)
    T = pb.gx * pb.gy
    tiles = None
    if tile_sample is not None and tile_sample < T:
        tiles = np.sort(np.random.default_rng(0).choice(T, size=tile_sample, replace=False)).astype(np.int32)
    scale = T / len(tiles) if tiles is not None else 1.0
    rng = np.random.default_rng(0)
    dcol = rng.standard_normal((3, pb.H, pb.W)).astype(np.float32)
    dlang = rng.standard_normal((pb.D, pb.H, pb.W)).astype(np.float32) if pb.D else None
    tf = {}
    f = O.forward(pb, nthreads=threads, tiles=tiles, timings=tf)
    t2 = time.perf_counter()
    if backward:
        O.backward(pb, f, dcol, dlang, tiles=tiles, nthreads=threads)
    t3 = time.perf_counter()
    t_pre_bin = tf["preprocess_binning"]
    # the render part of the forward scales with the tiles (a sample: x T / sample)
    t_fwd = t_pre_bin + tf["render"] * scale
    t_bwd = (t3 - t2) * scale
    t_frame = t_fwd + t_bwd
    what = "whole" if tiles is None else f"{len(tiles)} of {T} tiles (x{scale:.1f}, extrapolated) of the"
    return dict(value=round(1.0 / t_frame, 5), unit="frames/s", cores=threads, kind="port",
                cpu_model=cpu_model(), host_cpus=os.cpu_count(),
                sample=f"{what} {cfg_name} frame, oracle/lsr_oracle.c on {threads} OpenMP threads: forward {t_fwd:.2f}s "
                       f"(of which preprocess + binning {t_pre_bin:.2f}s, single-threaded)"
                       + (f", backward {t_bwd:.2f}s (render bwd on {threads} threads + preprocess bwd)" if backward else
                          ", forward only"),
                extrapolated=tiles is not None,
                seconds_per_frame=round(t_frame, 3), stages_s=dict(preprocess_binning=round(t_pre_bin, 3),
                                                                  forward=round(t_fwd, 3), backward=round(t_bwd, 3)))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def fwd_fps(g, dev, sh_degree, D, W=1280, H=800, iters=20):
    cam = make_camera(W, H)
    rs = settings(cam, dev, sh_degree, D > 0)
    r = GaussianRasterizer(rs)

    def run():
        with torch.no_grad():
            r(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], shs=g["shs"],
              language_feature_precomp=g.get("language_feature_precomp"), scales=g["scales"],
              rotations=g["rotations"])
    return 1.0 / timeit(run, iters)


def quick_fps(N, dev, W=1280, H=800, iters=20):
    """The evaluation path behind the reference's "450+ FPS" (README.md:1, eval_lerf.py:210-220):
    quick render of 3 levels x top-4 codes into 192 channels, then the 3 x 64 x 512 codebook
    decode + L2 normalise, at 1.0 Mpix.  The headline fields use DEFAULT settings, exactly as the
    reference's unchanged caller builds them (no language_feature_layout: the map is the
    pixel-major (192,H,W) view, which the reference's .view(3, 64, H, W).view(3, 64, H*W) +
    einsum accept unchanged; tests/test_quick_layout.py).  `reference_layout` times the
    contiguous map (language_feature_layout="chw").  render_decode_fps is one view at a time
    (render, then this package's decode); render_decode_stream_fps is the throughput over a
    stream of views with each decode overlapping the next render (quick.QuickFeatureStream);
    `reference_consumer` times the reference's own decode on the same map, torch.einsum +
    /(norm + 1e-10) exactly as eval_lerf.py:214-218."""
    from langsplatv2_amd import quick
    cam = make_camera(W, H)
    g = make_gaussians(N, cam, seed=0, sh_degree=3, quick_k=4)
    t = {k: v.to(dev) for k, v in g.items() if isinstance(v, torch.Tensor)}
    z = torch.zeros_like(t["means3D"])
    cb = torch.randn(3, 64, 512, device=dev)

    def measure(layout, consumer=False):
        r = GaussianRasterizer(settings(cam, dev, 3, False, quick=True, quick_layout=layout))

        def render():
            with torch.no_grad():
                return r(means3D=t["means3D"], means2D=z, opacities=t["opacities"], shs=t["shs"],
                         language_feature_weights_quick=t["language_feature_weights_quick"],
                         language_feature_indices=t["language_feature_indices"], scales=t["scales"],
                         rotations=t["rotations"])[1]

        def both():
            quick.decode_language_features(render(), cb)
        s_render = timeit(render, iters)
        s_total = timeit(both, iters)
        fs = quick.QuickFeatureStream(cb)

        def streamed():
            fs.push(render)
        s_stream = timeit(streamed, iters)
        fs.flush()
        res = dict(render_fps=round(1.0 / s_render, 1), render_decode_fps=round(1.0 / s_total, 1),
                   render_ms=round(s_render * 1e3, 4), decode_ms=round((s_total - s_render) * 1e3, 4),
                   render_decode_stream_fps=round(1.0 / s_stream, 1))
        if consumer:
            cbt = cb.permute(0, 2, 1)

            def reference_consumer():
                with torch.no_grad():
                    m = render()
                    D, Hh, Ww = m.shape
                    m = m.view(3, 64, Hh, Ww).view(3, 64, Hh * Ww)
                    f = torch.einsum('ldk,lkn->ldn', cbt, m).view(3, 512, Hh, Ww)
                    return f / (f.norm(dim=1, keepdim=True) + 1e-10)
            s_ref = timeit(reference_consumer, iters)
            res["reference_consumer"] = dict(
                what="render + the reference's torch.einsum decode + /(norm+1e-10) (eval_lerf.py:214-218)",
                render_decode_fps=round(1.0 / s_ref, 1), decode_ms=round((s_ref - s_render) * 1e3, 4))
        return res
    out = dict(workload=f"{N} Gaussians {W}x{H}, quick 3x top-4 -> 192 ch + 3x64x512 decode + L2 norm",
               layout="default settings (pixel-major quick map view; language_feature_layout unset)")
    out.update(measure(None, consumer=True))
    out["reference_layout"] = measure("chw")
    return out


def deterministic_cost(step, steps):
    """The same fwd+bwd step with the deterministic backward (LSR_OPT_DETERMINISTIC:
    fixed-point cross-block sums, include/lsr.h): its time per step and per stage
    (outside the headline's timed region), and whether two steps' gradients are
    bit-identical."""
    with _lib.deterministic(True):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        _lib.profile_stages(None)
        _lib.profile_reset()
        _lib.profile_enable(True)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        _lib.profile_enable(False)
        st = {k: round(ms / c, 4) for k, (ms, c) in _lib.profile_query().items() if c}
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        a, b = step(), step()
        same = all(torch.equal(x, y) for x, y in zip(a, b) if x is not None)
    return dict(what="fwd+bwd step with lsr_set_option(LSR_OPT_DETERMINISTIC, 1)",
                ms_per_step=round(el / steps * 1e3, 4), frames_per_s=round(steps / el, 1), stages_ms=st,
                bit_identical_runs=bool(same))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks as a torch.distributed.run child (no
    GPU call has happened in this process) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run(world, rank, config=3) -> int:
    """Rank bring-up only (gloo, no GPU): every rank reports (rank, world size, its view's
    yaw) to rank 0."""
    yaw = dp.rank_yaw(rank, world)
    if world > 1:
        dist.init_process_group("gloo")
        seen = [None] * world
        dist.all_gather_object(seen, (rank, dist.get_world_size(), yaw))
        dist.destroy_process_group()
    else:
        seen = [(0, 1, yaw)]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "config": config,
                          "mode": CONFIG_MODES[config], "ranks": sorted(r for r, _, _ in seen),
                          "world_sizes_seen": sorted({w for _, w, _ in seen}),
                          "yaws": [y for _, _, y in sorted(seen)]}), flush=True)
    return 0


# --config 3: the headline (BASELINE metric) — fwd+bwd, views sharded, RCCL gradient exchange.
# --config 5: BASELINE configs[4] — forward only, replicas only (every rank renders its own
#             view of the replicated 5M-Gaussian scene; no data-path collective).
CONFIG_MODES = {1: "fwd+bwd, views sharded + gradient all-reduce (BASELINE configs[0], plumbing size)",
                2: "forward only, replicas (no collective)",
                3: "fwd+bwd, views sharded + RCCL all-reduce of gradients",
                5: "forward only, replicas (no collective)"}
FWD_METRIC = {2: "frames/s fwd @ 100k Gaussians 800x800 3+3ch (BASELINE configs[1], replicas)",
              5: "frames/s fwd @ 5M Gaussians 4K 3+32ch (BASELINE configs[4], replicas)"}
FWD_WORKLOAD = {2: "BASELINE cfg2: 100k Gaussians, 800x800, RGB colours + 3 language channels, forward only; "
                   "1 view per GPU, replicas (no collective)",
                5: "BASELINE cfg5: 5M Gaussians, 3840x2160, SH deg 3 + 32 dense language channels, "
                   "forward only; 1 view per GPU, replicas (no collective)"}
# CPU-baseline tile sample per forward config (None = the whole frame; cfg5's whole
# frame would take minutes of oracle time on the box's 16 threads)
FWD_CPU_TILES = {2: None, 5: 256}


def main_forward_replicas(args, world, rank, dev) -> int:
    """The forward-only BASELINE configs: configs[1] (cfg2: 100k Gaussians, 800x800, RGB
    colours + 3 language channels) and configs[4] (cfg5: 5M Gaussians, 3840x2160, SH degree 3
    + 32 dense language channels); one view per rank (yaw within +-20 degrees), Gaussians
    replicated, nothing exchanged.  value = frames rendered by all ranks / max-over-ranks
    time."""
    cfg = CONFIGS[args.config]
    N, W, H, D, deg = cfg["N"], cfg["W"], cfg["H"], cfg["lang_dim"], cfg["sh_degree"]
    yaw = dp.rank_yaw(rank, world)
    cam0 = make_camera(W, H)
    cam = make_camera(W, H, yaw_deg=yaw)
    gcpu = make_gaussians(N, cam0, seed=0, sh_degree=deg, lang_dim=D)
    keys = [k for k in ("means3D", "shs", "colors_precomp", "opacities", "scales", "rotations",
                        "language_feature_precomp") if k in gcpu]
    g = {k: gcpu[k].to(dev) for k in keys}
    g["means2D"] = torch.zeros_like(g["means3D"])
    rs = settings(cam, dev, deg or 0, D > 0)
    rast = GaussianRasterizer(rs)
    kw = {k: g[k] for k in keys if k not in ("means3D", "opacities")}

    def step():
        with torch.no_grad():
            return rast(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], **kw)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _lib.profile_stages(None)
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(max(2, min(args.steps, 5))):
        step()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    per_stage = {k: ms / calls for k, (ms, calls) in _lib.profile_query().items() if calls}
    dom = "render_fwd"
    _lib.profile_stages([dom])
    _lib.profile_reset()
    _lib.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        _lib.profile_enable(i % ROOF_EVERY == 0)   # as in the training bench
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _lib.profile_enable(False)
    _lib.profile_stages(None)
    dom_ms_s, dom_calls = _lib.profile_query()[dom]
    # the same forwards over a stream of views, two in flight (view_stream.ViewStream):
    # reported beside `value`, which is one view at a time
    from langsplatv2_amd.view_stream import ViewStream
    vs = ViewStream(dev)
    for _ in range(3):
        vs.push(step)
    vs.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        vs.push(step)
    vs.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed_stream = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([elapsed, elapsed_stream], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)   # timing only, not on the data path
        elapsed, elapsed_stream = float(t[0].item()), float(t[1].item())
    if rank == 0:
        S = 3 * (deg + 1) ** 2 if deg is not None else 0
        bytes_, info = algorithmic_bytes(g, rs, D, S)
        dom_ms = dom_ms_s / dom_calls if dom_calls else 0.0
        dom_gbps = bytes_[dom] / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        step_ms = elapsed / args.steps * 1e3
        fwd_keys = ("preprocess", "bin_count", "scan_tile_counts", "bin_scatter", "tile_sort", "render_fwd")
        pre = f"cfg{args.config}_r"
        traffic, traffic_src = pmc_traffic(dom, prefix=pre)
        # §8d charges every instance its 4C-byte feature row (M * 140 B at C = 35), which the
        # kernel re-reads from L2: the algorithmic rate exceeds the HBM peak, so the HBM
        # roofline here is the MEASURED traffic (PMC) over the launch time
        meas_gbps = traffic / (dom_ms * 1e-3) / 1e9 if (traffic and dom_ms > 0) else None
        out = {
            "metric": FWD_METRIC[args.config],
            "value": round(world * args.steps / elapsed, 3),
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
                "workload": FWD_WORKLOAD[args.config],
                "gaussians": N, "width": W, "height": H, "lang_dim": D, "sh_degree": deg,
                "global_batch": world, "parallelism": f"replicas x{world}" if world > 1 else "single GPU",
            },
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "roofline": {
                "bound": "hbm", "kernel": dom,
                "achieved": round(meas_gbps, 1) if meas_gbps is not None else None, "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(meas_gbps / HBM_PEAK_GBPS, 4) if meas_gbps is not None else None,
                "traffic": traffic, "traffic_source": traffic_src,
                "achieved_basis": "measured HBM bytes per launch (PMC FETCH+WRITE) / HIP-event launch time",
                "algorithmic_bytes_per_launch": int(bytes_[dom]),
                "algorithmic_GBps": round(dom_gbps, 1),
                "bytes_formula": "SURVEY.md §8d (bench.py:algorithmic_bytes)",
                "note": "the §8d bytes charge every instance its 4C-byte feature row (M*4C), which the kernel "
                        "re-reads from L2, so the algorithmic rate can exceed the HBM peak and is not an HBM "
                        "fraction; the kernel is VALU/MFMA-issue bound (`issue`)",
                "issue": pmc_issue(dom, prefix=pre),
                "ms_per_launch": round(dom_ms, 4), "launches_timed": dom_calls,
            },
            "stages_ms": {k: round(v, 4) for k, v in per_stage.items()},
            "stage_bytes": {k: int(bytes_[k]) for k in fwd_keys if k in bytes_},
            "workload_stats": info,
            "view_stream_fps": round(world * args.steps / elapsed_stream, 3),
            "view_stream_note": "the same forwards over a stream of views, two in flight on alternating "
                                "HIP streams (langsplatv2_amd.view_stream.ViewStream); `value` is one view at a time",
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cam, gcpu, D, cfg_name=f"cfg{args.config}", backward=False,
                                               tile_sample=FWD_CPU_TILES[args.config])
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 5],
                    help="3: BASELINE cfg3 fwd+bwd (the headline); 1: BASELINE cfg1 fwd+bwd (1k Gaussians, "
                         "128x128, RGB); 2 / 5: BASELINE cfg2 / cfg5 forward-only replicas")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fwd-1mpix", action="store_true")
    ap.add_argument("--no-quick", action="store_true")
    ap.add_argument("--no-det", action="store_true", help="skip the deterministic-backward sub-line")
    ap.add_argument("--dry-run", action="store_true", help="bring the ranks up on gloo and exit (no GPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dry_run:
        return dry_run(world, rank, args.config)
    # rehearsal only (a multi-rank run on a one-GPU box): LSR_BENCH_BACKEND=gloo and
    # LSR_BENCH_SAME_DEVICE=1 put every rank on cuda:0 with a gloo exchange; the
    # driver's runs use neither (RCCL, one GPU per rank)
    if world > 1:
        dist.init_process_group(os.environ.get("LSR_BENCH_BACKEND", "nccl"))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: RCCL sees {dist.get_world_size()} ranks, expected {args.gpus}")
    if os.environ.get("LSR_BENCH_SAME_DEVICE") == "1":
        local = 0
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    _lib.load()
    if args.config in (2, 5):
        return main_forward_replicas(args, world, rank, dev)

    cfg = CONFIGS[args.config]
    N, W, H, D, deg = cfg["N"], cfg["W"], cfg["H"], cfg["lang_dim"], cfg["sh_degree"]
    # one view per rank: yaw offsets within +-20 degrees, Gaussians replicated (seed 0)
    yaw = dp.rank_yaw(rank, world)
    cam0 = make_camera(W, H)
    cam = make_camera(W, H, yaw_deg=yaw)
    gcpu = make_gaussians(N, cam0, seed=0, sh_degree=deg, lang_dim=D)
    leaf_keys = tuple(k for k in ("means3D", "shs", "colors_precomp", "opacities", "scales", "rotations",
                                  "language_feature_precomp") if k in gcpu)
    g = {k: gcpu[k].to(dev).requires_grad_(True) for k in leaf_keys}
    g["means2D"] = torch.zeros_like(g["means3D"], requires_grad=True)
    leaves = [g[k] for k in leaf_keys]
    inputs = leaves + [g["means2D"]]
    gen = torch.Generator(device="cpu").manual_seed(1 + rank)
    dcolor = torch.randn((3, H, W), generator=gen).to(dev)
    dlang = torch.randn((D, H, W), generator=gen).to(dev) if D else None
    rs = settings(cam, dev, deg or 0, D > 0)
    rast = GaussianRasterizer(rs)
    kw = {k: g[k] for k in leaf_keys if k not in ("means3D", "opacities")}
    outs_of = (lambda c, l: [c, l]) if D else (lambda c, l: [c])
    grads_in = [dcolor, dlang] if D else [dcolor]
    exch = dp.ViewShardedExchange(leaves, with_stats=True, names=leaf_keys) if world > 1 else None
    xev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    xms = [0.0, 0]

    def step(timed_exchange=False):
        color, lang, radii = rast(means3D=g["means3D"], means2D=g["means2D"], opacities=g["opacities"], **kw)
        if exch is None:
            return torch.autograd.grad(outs_of(color, lang), inputs, grads_in)
        # gradients land in the all-reduce buckets; the language bucket's all-reduce
        # starts on a side stream as soon as the render backward has finished it
        with exch.sink():
            grads = torch.autograd.grad(outs_of(color, lang), inputs, grads_in)
        if timed_exchange:
            xev[0].record()
        red, _, _ = exch.finish(grads[-1], radii, grads[:-1], campos=rs.campos, means3D=g["means3D"].detach(),
                                sh_degree=deg or 0)
        if timed_exchange:
            xev[1].record()
            xev[1].synchronize()
            xms[0] += xev[0].elapsed_time(xev[1])
            xms[1] += 1
        return red

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # per-stage breakdown (+ the exposed exchange time): a separate untimed pass with every
    # stage bracketed by events (each bracket idles the stream a few us, so the timed region
    # below brackets only the dominant stage, for the live roofline)
    _lib.profile_stages(None)
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(max(2, min(args.steps, 5))):
        step(timed_exchange=True)
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
    for i in range(args.steps):
        # the dominant kernel is bracketed by events on every ROOF_EVERY-th step
        # of the timed region (each bracket idles the stream a few us)
        _lib.profile_enable(i % ROOF_EVERY == 0)
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
            bytes_, info = algorithmic_bytes(gd, rs, D, 3 * (deg + 1) ** 2 if deg is not None else 0)
        dom_ms = dom_ms_s / dom_calls if dom_calls else 0.0
        dom_gbps = bytes_[dom] / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        pre = "r" if args.config == 3 else f"cfg{args.config}_r"
        traffic, traffic_src = pmc_traffic(dom, prefix=pre)
        step_ms = elapsed / args.steps * 1e3
        kernel_ms = sum(v["ms_per_launch"] for v in per_stage.values())
        total_bytes = sum(bytes_.values())
        out = {
            "metric": METRIC if args.config == 3 else
            "frames/s fwd+bwd @ 1k Gaussians 128x128 RGB (BASELINE configs[0]); ms_per_step = its fwd+bwd time",
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
                            "fwd+bwd, all inputs require grad; 1 view per GPU" if args.config == 3 else
                            "BASELINE cfg1: 1k Gaussians, 128x128, RGB colours_precomp, fwd+bwd, all inputs "
                            "require grad; 1 view per GPU",
                "gaussians": N, "width": W, "height": H, "lang_dim": D, "sh_degree": deg,
                "global_batch": world, "parallelism": f"dp{world} (views sharded, RCCL all-reduce of grads)"
                if world > 1 else "single GPU",
            },
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "exchange": ({"bucket_bytes": exch.bucket_bytes, "sh_factored": exch.sh_idx is not None,
                          "early_bucket_bytes": exch.early.nbytes if exch.early is not None else 0,
                          "exposed_ms_per_step": round(xms[0] / max(xms[1], 1), 4),
                          **{k: round(v, 4) for k, v in dp.allreduce_bound_ms(exch.bucket_bytes, world).items()}}
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
                # context: the same §8d formula with the reference's M (its full rect lists) for
                # this frame, i.e. the bytes the reference's algorithm implies for the same output
                "algorithmic_bytes_reference_M": int(bytes_[dom] + (info["num_rendered_reference"] - info["num_rendered"])
                                                     * (28 + 4 * (3 + D))) if dom in ("render_fwd", "render_bwd") else None,
                "bytes_formula": "SURVEY.md §8d (bench.py:algorithmic_bytes)",
                "ms_per_launch": round(dom_ms, 4),
                "launches_timed": dom_calls,
                # the same kernel's average under rocprofv3 in a profile of this step alone
                "rocprof": rocprof_avg(dom) if args.config == 3 else None,
                # the kernel is issue/latency-bound, not HBM-bound: its SQ-counter roofline
                "issue": pmc_issue(dom, prefix=pre),
                # and its writes are memory-side atomics: their rate's floor
                "atomics": atomic_floor("render_bwd_mf", dom_ms, prefix=pre) if dom == "render_bwd" else None,
            },
            "hbm_step": {"algorithmic_bytes": int(total_bytes),
                         "GBps_over_kernels": round(total_bytes / (kernel_ms * 1e-3) / 1e9, 1) if kernel_ms else 0,
                         "GBps_over_step": round(total_bytes / (step_ms * 1e-3) / 1e9, 1),
                         "frac_over_step": round(total_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
            "stages_ms": {k: round(v["ms_per_launch"], 4) for k, v in per_stage.items()},
            "stage_bytes": {k: int(v) for k, v in bytes_.items()},
            "workload_stats": info,
        }
        if world == 1 and args.config == 3 and not args.no_det:
            out["deterministic"] = deterministic_cost(step, args.steps)
        if world == 1 and not args.no_fwd_1mpix and args.config == 3:
            out["fwd_fps_1mpix"] = round(fwd_fps({k: v.detach() for k, v in g.items()}, dev, deg, D), 1)
        if world == 1 and not args.no_quick and args.config == 3:
            out["quick_1mpix"] = quick_fps(N, dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cam, gcpu, D, cfg_name=f"cfg{args.config}")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
