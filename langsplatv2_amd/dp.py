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
The early all-reduce is started from a gradient hook on each language leaf,
which autograd calls once with the leaf's TOTAL gradient (every path summed):
when that is the bucket view itself (the rasterizer is the only path) the
all-reduce waits on the library's lang-ready event and overlaps the preprocess
backward; when another path also reaches the leaf (a regulariser, a second
use) the hook first packs the sum into the view.  So a multi-path gradient is
never dropped or raced, in any mode.

View-factored SH gradient (zero-copy path, SH inputs): the SH coefficient
gradient of a view is an outer product, dL/dsh_k = basis_k(dir) * dL/dRGB
(the clamp-masked colour gradient of the SH evaluation, 3 floats), with dir
fixed by the Gaussian's mean and the view's camera centre.  So instead of
all-reducing the (N, 16, 3) SH gradient (62 % of the bytes at SH degree 3)
each rank all-gathers its (N, 3) dL/dRGB and its camera centre, and every
rank rebuilds the summed SH gradient locally in view order
(lsr_sh_grad_from_views) — identical on all ranks, equal to the all-reduced
sum up to fp32 summation order.  Per GPU the exchange moves
2(R-1)/R * 29 + (R-1)/R * 3R floats per Gaussian instead of 2(R-1)/R * 77:
-47 % at R = 8, -57 % at R = 2.  The backward hands autograd an expanded zero
as the SH gradient (GradSink.sh_return), so a second path into the SH leaf
arrives at its hook as exactly that path's own gradient; the exchange
all-reduces it and adds it to the rebuilt sum.
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

    def __init__(self, params: list[torch.Tensor], with_stats: bool = True, group=None, names=None,
                 factor_sh: bool | None = None, force_collectives: bool = False):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # force_collectives (test hook): take every collective branch even at
        # world size 1 (side-stream early all-reduce, factored SH all-gather,
        # MAX of the radii), so the RCCL code paths run on a one-GPU box
        # (tests/test_rccl_paths.py); the sums over one rank are identities
        if force_collectives and not dist.is_initialized():
            raise ValueError("force_collectives needs an initialised process group")
        self.collective = self.world > 1 or force_collectives
        self.group = group
        self.names = list(names) if names is not None else [None] * len(params)
        if len(self.names) != len(params):
            raise ValueError("ViewShardedExchange: one name per parameter")
        n = params[0].shape[0] if with_stats else 0
        self.early_idx = [i for i, nm in enumerate(self.names) if nm in LANG_KEYS]
        # view-factored SH gradient (see the module docstring): GPU, R > 1, SH parameter present
        sh_i = self.names.index("shs") if "shs" in self.names else None
        if factor_sh is None:
            factor_sh = self.collective and params[0].is_cuda and sh_i is not None
        self.sh_idx = sh_i if factor_sh else None
        if self.sh_idx is not None:
            shp = params[self.sh_idx]
            if shp.dim() != 3 or shp.shape[2] != 3 or shp.shape[1] > 16:
                raise ValueError("ViewShardedExchange: factor_sh needs shs of shape (N, M <= 16, 3)")
            dev = shp.device
            self.sh_grad = torch.empty(tuple(shp.shape), dtype=torch.float32, device=dev)
            self.rgb_mine = torch.empty((shp.shape[0], 3), dtype=torch.float32, device=dev)
            self.rgb_all = torch.empty((self.world, shp.shape[0], 3), dtype=torch.float32, device=dev)
            self.campos_all = torch.empty((self.world, 3), dtype=torch.float32, device=dev)
        self.main_idx = [i for i in range(len(params)) if i not in self.early_idx and i != self.sh_idx]
        self.early = GradBucket([params[i].detach() for i in self.early_idx]) if self.early_idx else None
        self.main = GradBucket([params[i].detach() for i in self.main_idx], stats_rows=n)
        self.with_stats = with_stats
        self._early_work = None
        self._ev = None
        self._side = None
        self.cuda = params[0].is_cuda
        self._params = list(params)
        self._sink = None
        self._hooks = []
        self._early_seen = set()   # early indices whose view holds the leaf's total gradient
        self._early_packed = False
        self._sh_extra = None      # another path's gradient into the factored SH leaf
        self._sh_zero = None
        if self.cuda and self.early is not None and self.collective:
            self._ev = torch.cuda.Event()
            self._ev_pack = torch.cuda.Event()
            self._side = torch.cuda.Stream(device=params[0].device)

    @property
    def bucket_bytes(self) -> int:
        """Bytes all-reduced per step (plus, factored, the all-gathered colour gradients)."""
        b = self.main.nbytes + (self.early.nbytes if self.early is not None else 0)
        if self.sh_idx is not None:
            b += self.rgb_mine.numel() * 4
        return b

    def _views(self) -> list[torch.Tensor]:
        out = [None] * len(self.names)
        for i, v in zip(self.main_idx, self.main.views()):
            out[i] = v
        if self.early is not None:
            for i, v in zip(self.early_idx, self.early.views()):
                out[i] = v
        if self.sh_idx is not None:
            out[self.sh_idx] = self.sh_grad
        return out

    def _early_hook(self, i, view):
        """Gradient hook of early leaf i: `g` is the leaf's total gradient.  The view
        itself: the rasterizer wrote it and nothing else reaches the leaf.  Anything
        else (a multi-path sum, or a gradient that never went through the sink) is
        packed into the view first, on the stream that produced it."""
        def hook(g):
            packed = False
            if g is None:
                view.zero_()
                packed = True
            elif g.data_ptr() != view.data_ptr():
                view.copy_(g.reshape(view.shape))
                packed = True
            self._early_seen.add(i)
            self._early_packed = self._early_packed or packed
            if len(self._early_seen) == len(self.early_idx):
                self._launch_early(after_pack=self._early_packed)
        return hook

    def _sh_hook(self, g):
        """Gradient hook of the factored SH leaf: the rasterizer returns an expanded
        zero (GradSink.sh_return), so anything else is another path's own gradient."""
        if g is not None and g.data_ptr() != self._sh_zero.data_ptr():
            self._sh_extra = g

    def _launch_early(self, after_pack: bool = True):
        if not self.collective or self.early is None or self._early_work is not None:
            return
        if self._side is not None:
            # the library's lang-ready event (before the preprocess backward) when the
            # views are the backward's own output; after a pack, a fresh event
            ev = self._ev
            if after_pack or not ev.cuda_event:
                ev = self._ev_pack
                ev.record(torch.cuda.current_stream(self.early.flat.device))
            self._side.wait_event(ev)
            with torch.cuda.stream(self._side):
                self._early_work = self.early.allreduce(self.group, async_op=True)
        else:
            self._early_work = self.early.allreduce(self.group, async_op=True)

    def _remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def sink(self):
        """rasterizer.GradSink writing this rank's gradients into the buckets; the
        early (language) all-reduce starts from the language leaves' gradient hooks."""
        from .rasterizer import GradSink
        self._remove_hooks()
        views = self._views()
        bufs = {nm: v for nm, v in zip(self.names, views) if nm is not None}
        self._early_work = None
        self._early_seen = set()
        self._early_packed = False
        self._sh_extra = None
        if self.collective:
            for i in self.early_idx:
                p = self._params[i]
                if p.requires_grad:
                    self._hooks.append(p.register_hook(self._early_hook(i, views[i])))
        if self.sh_idx is not None:
            p = self._params[self.sh_idx]
            if self._sh_zero is None:
                self._sh_zero = torch.zeros((1, 1, 1), dtype=torch.float32, device=p.device).expand(tuple(p.shape))
            if p.requires_grad:
                self._hooks.append(p.register_hook(self._sh_hook))
        self._sink = GradSink(bufs, lang_ready=self._ev,
                              rgb_sh=self.rgb_mine if self.sh_idx is not None else None,
                              params={nm: p for nm, p in zip(self.names, self._params) if nm is not None},
                              sh_return=self._sh_zero)
        return self._sink

    def _factored_sh(self, campos, means3D, sh_degree):
        """All-gather the views' colour gradients and camera centres, rebuild the
        summed SH gradient into self.sh_grad (every rank, view order)."""
        if campos is None or means3D is None or sh_degree is None:
            raise ValueError("finish: the factored SH gradient needs campos, means3D and sh_degree")
        cp = torch.as_tensor(campos, dtype=torch.float32, device=self.rgb_mine.device).reshape(3).contiguous()
        if dist.get_backend(self.group) == "gloo":
            # gloo (CPU tests): gather through host copies
            ca = [torch.empty(3) for _ in range(self.world)]
            ra = [torch.empty(tuple(self.rgb_mine.shape)) for _ in range(self.world)]
            dist.all_gather(ca, cp.cpu(), group=self.group)
            dist.all_gather(ra, self.rgb_mine.cpu(), group=self.group)
            self.campos_all.copy_(torch.stack(ca))
            self.rgb_all.copy_(torch.stack(ra))
        else:
            dist.all_gather(list(self.campos_all.unbind(0)), cp, group=self.group)
            dist.all_gather(list(self.rgb_all.unbind(0)), self.rgb_mine, group=self.group)
        sh_grad_from_views(means3D.detach().contiguous(), self.campos_all, self.rgb_all, int(sh_degree), self.sh_grad)

    def finish(self, means2D_grad=None, radii=None, grads=None, campos=None, means3D=None, sh_degree=None):
        """Complete the exchange after a `sink()` backward: any gradient in
        `grads` that did not land in its bucket view (e.g. a parameter without
        grad this step) is packed (None -> zeros); a gradient the backward wrote
        into its view through the sink is taken from the view whatever `grads`
        holds for it (torch.autograd.grad returns the view itself, loss.backward()
        leaves a copy in p.grad); the statistics are added, the
        remaining all-reduce runs and every pending one is waited for.  With the
        factored SH gradient, `campos` (this view's camera centre), `means3D`
        and `sh_degree` (the rasterizer settings') are required."""
        views = self._views()
        used = self._sink.used if self._sink is not None else set()
        self._remove_hooks()
        # factored SH only when the backward wrote dL/dRGB for the bucketed SH leaf;
        # otherwise (e.g. shs = cat(f_dc, f_rest)) the SH gradient is all-reduced as is
        factored = self.sh_idx is not None and "shs" in used
        if grads is not None:
            for i, (g, v) in enumerate(zip(grads, views)):
                if i == self.sh_idx and factored:
                    continue   # rebuilt by _factored_sh below (+ another path's part, _sh_hook)
                if i in self._early_seen:
                    continue   # the hook left the leaf's total gradient in the view
                if g is not None and g.data_ptr() == v.data_ptr():
                    continue
                # the backward wrote this view and `grads` holds a copy (loss.backward()
                # inside `with ex.sink():` leaves AccumulateGrad's copy in p.grad) or
                # autograd's multi-path SUM: packing g is right in both cases; a view
                # the backward did not write is packed too (None -> zeros)
                if g is None:
                    if self.names[i] not in used:
                        v.zero_()
                    continue
                v.copy_(g.reshape(v.shape))
        elif self.sh_idx is not None and not factored:
            raise ValueError("finish: the SH gradient was not factored by the backward; pass grads")
        if self.with_stats:
            if means2D_grad is None or radii is None:
                raise ValueError("finish: densification statistics need means2D.grad and radii")
            self.main.flat[self.main.stats_offset:].copy_(densify_increment(means2D_grad, radii).reshape(-1))
        max_radii = radii
        if self.collective:
            self._launch_early()   # no-op if the backward already started it
            work = self.main.allreduce(self.group, async_op=True)
            if factored:
                self._factored_sh(campos, means3D, sh_degree)
                if self._sh_extra is not None:
                    # another path into the SH leaf (its own gradient, see _sh_hook)
                    extra = self._sh_extra.reshape(self.sh_grad.shape).contiguous()
                    dist.all_reduce(extra, op=dist.ReduceOp.SUM, group=self.group)
                    self.sh_grad.add_(extra)
            elif self.sh_idx is not None:
                dist.all_reduce(self.sh_grad, op=dist.ReduceOp.SUM, group=self.group)
            if radii is not None:
                max_radii = radii.clone()
                dist.all_reduce(max_radii, op=dist.ReduceOp.MAX, group=self.group)
            work.wait()
            if self._early_work is not None:
                self._early_work.wait()
            self._early_work = None
        self._sink = None
        self._sh_extra = None
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
        if self.sh_idx is not None:
            # copy path: the backward produced a full SH gradient; sum it as is
            g = grads[self.sh_idx]
            if g is None:
                self.sh_grad.zero_()
            else:
                self.sh_grad.copy_(g.reshape(self.sh_grad.shape))
        return self._finish_packed(radii)

    def _finish_packed(self, radii):
        max_radii = radii
        if self.collective:
            if self.early is not None:
                self._early_work = self.early.allreduce(self.group, async_op=True)
            if self.sh_idx is not None:
                dist.all_reduce(self.sh_grad, op=dist.ReduceOp.SUM, group=self.group)
            work = self.main.allreduce(self.group, async_op=True)
            if radii is not None:
                max_radii = radii.clone()
                dist.all_reduce(max_radii, op=dist.ReduceOp.MAX, group=self.group)
            work.wait()
            if self._early_work is not None:
                self._early_work.wait()
            self._early_work = None
        return self._views(), self.main.stats(), max_radii


def sh_grad_from_views(means3D: torch.Tensor, campos: torch.Tensor, drgb: torch.Tensor, sh_degree: int,
                       out: torch.Tensor) -> torch.Tensor:
    """out (N, M, 3) <- sum over views r of basis(dir_r) (x) drgb[r] (lsr_sh_grad_from_views):
    the SH coefficient gradient of R views from their (N, 3) colour gradients."""
    from . import _lib
    from .rasterizer import _stream
    N, M = out.shape[0], out.shape[1]
    R = campos.shape[0]
    for t in (means3D, campos, drgb, out):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("sh_grad_from_views: contiguous fp32 ROCm tensors expected (there is no CPU path)")
    if tuple(drgb.shape) != (R, N, 3) or tuple(means3D.shape) != (N, 3) or tuple(campos.shape) != (R, 3):
        raise ValueError("sh_grad_from_views: shapes means3D (N,3), campos (R,3), drgb (R,N,3), out (N,M,3)")
    _lib.check(_lib.load().lsr_sh_grad_from_views(N, M, int(sh_degree), means3D.data_ptr(), R, campos.data_ptr(),
                                                   drgb.data_ptr(), out.data_ptr(), _stream(out.device)),
               "lsr_sh_grad_from_views")
    return out


def allreduce_bound_ms(nbytes: int, world: int, link_GBps: float = 153.0, links: int = 7) -> dict:
    """Analytic exchange time bounds on xGMI: a single ring is
    bound by one link; multi-channel RCCL spreads over all links."""
    if world <= 1:
        return {"ring_1link_ms": 0.0, "all_links_ms": 0.0}
    vol = 2.0 * (world - 1) / world * nbytes
    return {"ring_1link_ms": vol / (link_GBps * 1e9) * 1e3,
            "all_links_ms": vol / (link_GBps * links * 1e9) * 1e3}


__all__ = ["rank_yaw", "view_schedule", "GradBucket", "densify_increment", "ViewShardedExchange",
           "sh_grad_from_views", "allreduce_bound_ms", "LANG_KEYS"]
