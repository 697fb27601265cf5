"""View-sharded data parallelism for the rasterizer step.

One process per GPU; every rank holds the full Gaussian replica and renders
its own view(s).  The only exchange is, once per step (before the optimizer
step), an all-reduce(SUM) of

  * every per-Gaussian parameter gradient (means3D, shs / colors, opacities,
    scales, rotations / cov3D, language features), and
  * the densification statistics the reference accumulates per view
    (`GaussianModel.add_densification_stats`, scene/gaussian_model.py:506-508,
    called from train.py:251): ||dL/d means2D[:, :2]|| and a visibility count,

plus one all-reduce(MAX) of the image-space radii (train.py:250).  Summing
the per-view gradients of R ranks equals `--accum_iter R` on one GPU
(train.py:261-263); only the summation order differs.

Bucketing for xGMI: the ranks are joined point to point by 7 links per GPU
and RCCL's ring/tree channels are link-bound, so the exchange is a few LARGE
messages, not one per tensor.  Two buckets, by when their gradients are final:
  early  the language gradient(s): final when the render backward ends; the
         library records an event there (lsr_bwd_out.lang_ready_event) and the
         all-reduce starts on a side stream while preprocess_bwd still runs;
  main   everything preprocess_bwd writes + the densification statistics.
Zero-copy: `ViewShardedExchange.sink()` hands the rasterizer backward the
buckets' views as its output buffers (rasterizer.GradSink), so gradients are
written straight into the all-reduce buffers (no ~300 MB pack copy).
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
    Every rank computes the same permutation without communicating.  When
    `world` does not divide `num_views` the permutation is extended by wrapping
    around to its start, so every view is rendered at least once per epoch (the
    reference samples every view, train.py:139-147) and every rank runs the
    same number of steps (ceil(num_views / world))."""
    g = torch.Generator().manual_seed(seed * 1000003 + epoch)
    perm = torch.randperm(num_views, generator=g).tolist()
    if num_views == 0:
        return []
    steps = -(-num_views // world)
    return [perm[(world * i + rank) % num_views] for i in range(steps)]


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


LANG_KEYS = ("language_feature_precomp", "language_feature_weights_quick")


class ViewShardedExchange:
    """The per-step exchange of one rank.

    Copy path (any training loop):
        ex = ViewShardedExchange(params, with_stats=True)
        ...forward / loss.backward() of this rank's view...
        grads, stats, max_radii = ex.exchange([p.grad for p in params], means2D.grad, radii)

    Zero-copy path (named parameters; what bench.py times):
        ex = ViewShardedExchange(params, names=[...])
        with ex.sink():
            grads = torch.autograd.grad(outputs, params + [means2D], grad_outputs)
        grads, stats, max_radii = ex.finish(grads[-1], radii)

    `grads` are views of the reduced buckets in `params` order."""

    def __init__(self, params: list[torch.Tensor], with_stats: bool = True, group=None, names=None):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.group = group
        self.names = list(names) if names is not None else [None] * len(params)
        if len(self.names) != len(params):
            raise ValueError("ViewShardedExchange: one name per parameter")
        n = params[0].shape[0] if with_stats else 0
        self.early_idx = [i for i, nm in enumerate(self.names) if nm in LANG_KEYS]
        self.main_idx = [i for i in range(len(params)) if i not in self.early_idx]
        self.early = GradBucket([params[i].detach() for i in self.early_idx]) if self.early_idx else None
        self.main = GradBucket([params[i].detach() for i in self.main_idx], stats_rows=n)
        self.with_stats = with_stats
        self._early_work = None
        self._ev = None
        self._side = None
        self.cuda = params[0].is_cuda
        if self.cuda and self.early is not None and self.world > 1:
            self._ev = torch.cuda.Event()
            self._side = torch.cuda.Stream(device=params[0].device)

    @property
    def bucket_bytes(self) -> int:
        return self.main.nbytes + (self.early.nbytes if self.early is not None else 0)

    def _views(self) -> list[torch.Tensor]:
        out = [None] * len(self.names)
        for i, v in zip(self.main_idx, self.main.views()):
            out[i] = v
        if self.early is not None:
            for i, v in zip(self.early_idx, self.early.views()):
                out[i] = v
        return out

    def _launch_early(self):
        if self.world <= 1 or self.early is None or self._early_work is not None:
            return
        if self._side is not None:
            self._side.wait_event(self._ev)
            with torch.cuda.stream(self._side):
                self._early_work = self.early.allreduce(self.group, async_op=True)
        else:
            self._early_work = self.early.allreduce(self.group, async_op=True)

    def sink(self):
        """rasterizer.GradSink writing this rank's gradients into the buckets and
        starting the early (language) all-reduce once the library marks it final."""
        from .rasterizer import GradSink
        bufs = {nm: v for nm, v in zip(self.names, self._views()) if nm is not None}
        self._early_work = None
        return GradSink(bufs, lang_ready=self._ev, on_lang_ready=self._launch_early if self._ev is not None else None)

    def finish(self, means2D_grad=None, radii=None, grads=None):
        """Complete the exchange after a `sink()` backward: any gradient in
        `grads` that did not land in its bucket view (e.g. a parameter without
        grad this step) is packed (None -> zeros), the statistics are added, the
        remaining all-reduce runs and every pending one is waited for."""
        views = self._views()
        if grads is not None:
            for i, (g, v) in enumerate(zip(grads, views)):
                if g is None:
                    v.zero_()
                elif g.data_ptr() != v.data_ptr():
                    v.copy_(g.reshape(v.shape))
        if self.with_stats:
            if means2D_grad is None or radii is None:
                raise ValueError("finish: densification statistics need means2D.grad and radii")
            self.main.flat[self.main.stats_offset:].copy_(densify_increment(means2D_grad, radii).reshape(-1))
        max_radii = radii
        if self.world > 1:
            self._launch_early()   # no-op if the backward already started it
            work = self.main.allreduce(self.group, async_op=True)
            if radii is not None:
                max_radii = radii.clone()
                dist.all_reduce(max_radii, op=dist.ReduceOp.MAX, group=self.group)
            work.wait()
            if self._early_work is not None:
                self._early_work.wait()
            self._early_work = None
        return views, self.main.stats(), max_radii

    def exchange(self, grads, means2D_grad=None, radii=None):
        """Copy path: pack `grads` (params order; None -> zeros), all-reduce, return views."""
        if len(grads) != len(self.names):
            raise ValueError("exchange: wrong number of gradients")
        self._early_work = None
        if self.early is not None:
            self.early.pack([grads[i] for i in self.early_idx])
        stats = None
        if self.with_stats:
            if means2D_grad is None or radii is None:
                raise ValueError("exchange: densification statistics need means2D.grad and radii")
            stats = densify_increment(means2D_grad, radii)
        self.main.pack([grads[i] for i in self.main_idx], stats)
        return self._finish_packed(radii)

    def _finish_packed(self, radii):
        max_radii = radii
        if self.world > 1:
            if self.early is not None:
                self._early_work = self.early.allreduce(self.group, async_op=True)
            work = self.main.allreduce(self.group, async_op=True)
            if radii is not None:
                max_radii = radii.clone()
                dist.all_reduce(max_radii, op=dist.ReduceOp.MAX, group=self.group)
            work.wait()
            if self._early_work is not None:
                self._early_work.wait()
            self._early_work = None
        return self._views(), self.main.stats(), max_radii


def allreduce_bound_ms(nbytes: int, world: int, link_GBps: float = 153.0, links: int = 7) -> dict:
    """Analytic exchange time bounds on xGMI: a single ring is
    bound by one link; multi-channel RCCL spreads over all links."""
    if world <= 1:
        return {"ring_1link_ms": 0.0, "all_links_ms": 0.0}
    vol = 2.0 * (world - 1) / world * nbytes
    return {"ring_1link_ms": vol / (link_GBps * 1e9) * 1e3,
            "all_links_ms": vol / (link_GBps * links * 1e9) * 1e3}


__all__ = ["rank_yaw", "view_schedule", "GradBucket", "densify_increment", "ViewShardedExchange",
           "allreduce_bound_ms", "LANG_KEYS"]
