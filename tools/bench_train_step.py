"""Feature-mode training iteration of LangSplatV2 (BASELINE.json cfg4's step,
train.py:139-173 + :261-263 with vq_layer_num 1, codebook_size 64, topk 4,
--cos_loss as in train.sh), synthetic data in place of the LERF scene: the
cfg3 scene (1M Gaussians, 1920x1080) with frozen geometry, per-view segment
maps of coherent regions and an (S, 512) feature table per view.

Per rank and iteration (one view per rank, views sharded across ranks):
  weights = get_render_weights(logits, 1, 64, 4)          fused top-k producer (HIP)
  _, weight_map, _ = rasterizer(..., language_feature_precomp=weights)   (HIP, D = 64)
  loss = language_cos_loss(weight_map, codebooks, seg, feat)             fused loss (HIP)
  loss.backward()                                           -> logits.grad, codebooks.grad
  all-reduce(SUM) of the two gradients in one bucket        (RCCL, world > 1)
  Adam step (FusedAdam, HIP; lr 0.0025 on both, eps 1e-15 as scene/gaussian_model.py:234-255)

--reference runs the same iteration with the reference's torch formulation of
the producer (utils/vq_utils.py:9-24) and of the loss (materialised features +
gathered ground truth + cos_loss), the rasterizer unchanged.
--torch-adam steps with torch.optim.Adam instead of FusedAdam.
--means2d-grad gives means2D requires_grad as render() does
(gaussian_renderer/__init__.py:27-31): the rasterizer then runs its full
backward; feature mode never reads that gradient (train.py:247), and without
it the language-only backward runs.

  python tools/bench_train_step.py [--steps 20 --warmup 5] [--reference] [--means2d-grad]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/bench_train_step.py
Prints one JSON line on rank 0: iterations/s (= optimizer steps/s) and views/s.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from langsplatv2_amd import _lib, dp, lang_codes  # noqa: E402
from langsplatv2_amd.lang_loss import language_cos_loss  # noqa: E402
from langsplatv2_amd.optim import FusedAdam  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians, softmax_to_topk_soft_code  # noqa: E402


def reference_loss(wm, cb, seg, feat):
    K, H, W = wm.shape
    f = (cb[0].T @ wm.reshape(K, -1)).reshape(-1, H, W)
    s = seg.reshape(-1).long()
    mask = (s != -1).reshape(1, H, W)
    gt = feat[s].reshape(H, W, -1).permute(2, 0, 1)
    return 1 - F.cosine_similarity(f * mask, gt * mask, dim=0).mean()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--segments", type=int, default=200)
    ap.add_argument("--reference", action="store_true")
    ap.add_argument("--means2d-grad", action="store_true")
    ap.add_argument("--torch-adam", action="store_true")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    cfg = CONFIGS[3]
    N, W, H = cfg["N"], cfg["W"], cfg["H"]
    K, Df, k = 64, 512, 4
    cam0 = make_camera(W, H)
    cam = make_camera(W, H, yaw_deg=dp.rank_yaw(rank, world))
    g0 = make_gaussians(N, cam0, seed=0, sh_degree=3, lang_dim=0)
    geo = {n: g0[n].to(dev) for n in ("means3D", "shs", "opacities", "scales", "rotations")}
    gen = torch.Generator(device="cpu").manual_seed(7)
    logits = torch.randn(N, K, generator=gen).to(dev).requires_grad_(True)
    codebooks = torch.randn(1, K, Df, generator=gen).to(dev).requires_grad_(True)
    adam = torch.optim.Adam if (a.torch_adam or a.reference) else FusedAdam
    opt = adam([{"params": [logits, codebooks], "lr": 0.0025, "name": "language_feature"}], lr=0.0, eps=1e-15)
    # this rank's view: segment ids in coherent regions, a per-view feature table
    vg = torch.Generator(device="cpu").manual_seed(100 + rank)
    S = a.segments
    feat = torch.randn(S, Df, generator=vg).to(dev)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    seg = (((yy // 60) * 37 + (xx // 80) + rank) % (S + 1) - 1).to(torch.int32).to(dev)
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
        projmatrix=cam["projmatrix"].to(dev), sh_degree=3, campos=cam["campos"].to(dev), prefiltered=False,
        debug=False, include_feature=True, quick_render=False)
    rast = GaussianRasterizer(rs)
    means2D = torch.zeros_like(geo["means3D"], requires_grad=a.means2d_grad)
    exch = dp.ViewShardedExchange([logits, codebooks], with_stats=False) if world > 1 else None

    def step():
        opt.zero_grad(set_to_none=True)
        if a.reference:
            weights = softmax_to_topk_soft_code(logits, k)
        else:
            weights = lang_codes.get_render_weights(logits, 1, K, k)
        _, wmap, _ = rast(means3D=geo["means3D"], means2D=means2D, opacities=geo["opacities"], shs=geo["shs"],
                          language_feature_precomp=weights, scales=geo["scales"], rotations=geo["rotations"])
        loss = reference_loss(wmap, codebooks, seg, feat) if a.reference else \
            language_cos_loss(wmap, codebooks, seg, feat)
        loss.backward()
        if exch is not None:
            grads, _, _ = exch.exchange([logits.grad, codebooks.grad])
            logits.grad, codebooks.grad = grads
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    step()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    stages = {n: round(ms / c, 4) for n, (ms, c) in _lib.profile_query().items() if c}
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({
            "workload": "feature-mode training iteration (cfg4 step shape), synthetic: 1M Gaussians, 1920x1080, "
                        "64 codes x 512-d codebook, top-4 soft codes, cos loss, Adam; 1 view per GPU",
            "variant": "reference torch ops for producer + loss + torch Adam" if a.reference else
                       "fused HIP producer + loss + " + ("torch Adam" if a.torch_adam else "FusedAdam"),
            "means2d_grad": a.means2d_grad, "n_gpus": world, "steps": a.steps,
            "ms_per_iteration": round(el / a.steps * 1e3, 4), "iterations_per_s": round(a.steps / el, 2),
            "views_per_s": round(world * a.steps / el, 2), "rasterizer_stages_ms": stages,
            "last_loss": float(loss.item()),
            "exchange_bytes": exch.bucket.nbytes if exch is not None else 0}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
