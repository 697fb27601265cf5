"""View-sharded data parallelism for the rasterizer step.

One process per GPU; every rank holds the full Gaussian replica and renders
its own view(s).  The only exchange is, once per step (before the optimizer
step), one all-reduce(SUM) of a single flat bucket holding

  * every per-Gaussian parameter gradient (means3D, shs / colors, opacities,
    scales, rotations / cov3D, language features), and
  * the densification statistics the reference accumulates per view
    (`GaussianModel.add_densification_stats`, scene/gaussian_model.py:506-508,
    called from train.py:251): ||dL/d means2D[:, :2]|| and a visibility count,

plus one all-reduce(MAX) of the image-space radii (train.py:250).  Summing
the per-view gradients of R ranks equals `--accum_iter R` on one GPU
(train.py:261-263); only the summation order differs.

One large bucket is deliberate: on MI355X the ranks are joined point to point
by xGMI (7 links per GPU), RCCL's ring/tree channels are link-bound, and a
single ~300 MB message keeps every channel streaming instead of paying
per-collective latency seven times.  Every gradient is produced by the one
rasterizer backward at the end of the step, so there is no earlier point at
which a first bucket could start.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def rank_yaw(rank: int, world: int, spread_deg: float = 40.0) -> float:
    """Camera yaw of the view rank `rank` renders in the synthetic benchmark:
    evenly spaced in [-spread/2, +spread/2] (0 for a single rank)."""
    if world <= 1:
        return 0.0
    return -0.5 * spread_deg + spread_deg * rank / (world - 1)


def view_schedule(num_views: int, world: int, rank: int, seed: int = 0, epoch: int = 0) -> list[int]:
    """Views rank `rank` renders in one pass over the training set: a shared
    seeded permutation, interleaved by rank (rank r takes perm[world*i + r]).
    Every rank computes the same permutation without communicating."""
    g = torch.Generator().manual_seed(seed * 1000003 + epoch)
    perm = torch.randperm(num_views, generator=g).tolist()
    steps = num_views // world
    return [perm[world * i + rank] for i in range(steps)]


class GradBucket:
    """A flat fp32 buffer holding a fixed list of gradient tensors (plus an
    optional (N, 2) densification-statistics block), reduced with ONE
    all_reduce.  After `pack`, `views()` are views of the reduced buffer with
    the parameters' shapes (ready to be installed as `.grad`)."""

    def __init__(self, like: list[torch.Tensor], stats_rows: int = 0):
        self.shapes = [tuple(t.shape) for t in like]
        self.numels = [t.numel() for t in like]
        self.stats_rows = stats_rows
        total = sum(self.numels) + 2 * stats_rows
        dev = like[0].device if like else torch.device("cpu")
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.offsets = []
        o = 0
        for n in self.numels:
            self.offsets.append(o)
            o += n
        self.stats_offset = o

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4

    def pack(self, grads: list[torch.Tensor | None], stats: torch.Tensor | None = None):
        if len(grads) != len(self.numels):
            raise ValueError("GradBucket.pack: wrong number of gradients")
        for g, o, n, shp in zip(grads, self.offsets, self.numels, self.shapes):
            dst = self.flat[o:o + n]
            if g is None:
                dst.zero_()
            else:
                if tuple(g.shape) != shp:
                    raise ValueError(f"GradBucket.pack: gradient shape {tuple(g.shape)} != {shp}")
                dst.copy_(g.reshape(-1))
        if self.stats_rows:
            dst = self.flat[self.stats_offset:]
            if stats is None:
                dst.zero_()
            else:
                dst.copy_(stats.reshape(-1))

    def views(self) -> list[torch.Tensor]:
        return [self.flat[o:o + n].view(shp) for o, n, shp in zip(self.offsets, self.numels, self.shapes)]

    def stats(self) -> torch.Tensor | None:
        if not self.stats_rows:
            return None
        return self.flat[self.stats_offset:].view(self.stats_rows, 2)

    def allreduce(self, group=None, async_op: bool = False):
        return dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


def densify_increment(means2D_grad: torch.Tensor, radii: torch.Tensor) -> torch.Tensor:
    """This view's contribution to (xyz_gradient_accum, denom) as an (N, 2)
    fp32 block: [||dL/d means2D[:, :2]||, 1] where radii > 0, else 0
    (scene/gaussian_model.py:506-508 applied with update_filter = radii > 0)."""
    vis = (radii > 0).to(torch.float32)
    nrm = torch.linalg.vector_norm(means2D_grad[:, :2], dim=-1) * vis
    return torch.stack([nrm, vis], 1)


class ViewShardedExchange:
    """The per-step exchange of one rank: pack this rank's gradients (and
    densification increments), all-reduce once, hand back reduced views.

        ex = ViewShardedExchange(params, with_stats=True)
        ...forward/backward of this rank's view...
        grads, stats, max_radii = ex.exchange([p.grad for p in params], means2D.grad, radii)
    """

    def __init__(self, params: list[torch.Tensor], with_stats: bool = True, group=None):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.group = group
        n = params[0].shape[0] if with_stats else 0
        self.bucket = GradBucket([p.detach() for p in params], stats_rows=n)
        self.with_stats = with_stats

    def exchange(self, grads, means2D_grad=None, radii=None):
        stats = None
        if self.with_stats:
            if means2D_grad is None or radii is None:
                raise ValueError("exchange: densification statistics need means2D.grad and radii")
            stats = densify_increment(means2D_grad, radii)
        self.bucket.pack(grads, stats)
        max_radii = radii
        if self.world > 1:
            work = self.bucket.allreduce(self.group, async_op=True)
            if radii is not None:
                max_radii = radii.clone()
                dist.all_reduce(max_radii, op=dist.ReduceOp.MAX, group=self.group)
            work.wait()
        return self.bucket.views(), self.bucket.stats(), max_radii


def allreduce_bound_ms(nbytes: int, world: int, link_GBps: float = 153.0, links: int = 7) -> dict:
    """Analytic exchange time bounds on xGMI: a single ring is
    bound by one link; multi-channel RCCL spreads over all links."""
    if world <= 1:
        return {"ring_1link_ms": 0.0, "all_links_ms": 0.0}
    vol = 2.0 * (world - 1) / world * nbytes
    return {"ring_1link_ms": vol / (link_GBps * 1e9) * 1e3,
            "all_links_ms": vol / (link_GBps * links * 1e9) * 1e3}


__all__ = ["rank_yaw", "view_schedule", "GradBucket", "densify_increment", "ViewShardedExchange",
           "allreduce_bound_ms"]
