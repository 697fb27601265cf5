"""world_size-2 gloo tests of the view-sharded data-parallel exchange
(langsplatv2_amd/dp.py) on CPU.  Each rank's per-view
gradients come from the oracle (the checker), so the test covers exactly the
exchange logic bench.py runs over RCCL on GPUs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from langsplatv2_amd import dp

PARAM_KEYS = ("means3D", "shs", "opacities", "scales", "rotations", "language_feature_precomp")
GRAD_KEYS = {"means3D": "dmeans3D", "shs": "dsh", "opacities": "dopacity", "scales": "dscales",
             "rotations": "drot", "language_feature_precomp": "dlang"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _view_grads(rank, world):
    """Oracle forward+backward of rank's view of the shared (seed 0) cloud."""
    from harness import make_case
    from oracle import oracle as O
    case = make_case(300, 64, 48, seed=0, sh_degree=3, lang_dim=4, yaw=dp.rank_yaw(rank, world))
    for k in ("scales",):
        case["g"][k] = case["g"][k] * 5
    pb = O.Problem(case["cam"], case["g"], bg=case["bg"])
    fwd = O.forward(pb)
    rng = np.random.default_rng(1 + rank)
    dC = rng.standard_normal((3, 48, 64)).astype(np.float32)
    dL = rng.standard_normal((4, 48, 64)).astype(np.float32)
    bwd = O.backward(pb, fwd, dC, dL)
    grads = []
    for k in PARAM_KEYS:
        v = torch.from_numpy(np.ascontiguousarray(bwd[GRAD_KEYS[k]]))
        grads.append(v.view(case["g"][k].shape))
    return case, grads, torch.from_numpy(bwd["dmean2D"]), torch.from_numpy(fwd["radii"])


def _worker(rank, world, port, tests_dir):
    import sys
    sys.path.insert(0, tests_dir)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case, grads, m2d, radii = _view_grads(rank, world)
        params = [case["g"][k] for k in PARAM_KEYS]
        ex = dp.ViewShardedExchange(params, with_stats=True)
        red, stats, max_r = ex.exchange(grads, m2d, radii)

        # expected: every rank's view, summed in rank order (= accum_iter=world on one GPU)
        views = [_view_grads(r, world) for r in range(world)]
        for i, k in enumerate(PARAM_KEYS):
            exp = views[0][1][i].clone()
            for r in range(1, world):
                exp = exp + views[r][1][i]
            assert torch.equal(red[i], exp), k
            assert red[i].shape == params[i].shape
        exp_stats = sum(dp.densify_increment(v[2], v[3]) for v in views)
        assert torch.equal(stats, exp_stats)
        exp_r = views[0][3].clone()
        for v in views[1:]:
            exp_r = torch.maximum(exp_r, v[3])
        assert torch.equal(max_r, exp_r)
        # both views are non-trivial and differ (the shards really are different views)
        assert not torch.equal(views[0][1][0], views[1][1][0])
        assert float(stats[:, 1].max()) == world
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_view_sharded_exchange_gloo_world2(oracle_lib):
    tests_dir = os.path.dirname(os.path.abspath(__file__))
    mp.spawn(_worker, args=(2, _free_port(), tests_dir), nprocs=2, join=True)


def test_grad_bucket_roundtrip():
    like = [torch.zeros(5, 3), torch.zeros(5, 16, 3), torch.zeros(5, 1)]
    b = dp.GradBucket(like, stats_rows=5)
    gs = [torch.randn(5, 3), None, torch.randn(5, 1)]
    st = torch.randn(5, 2)
    b.pack(gs, st)
    v = b.views()
    assert torch.equal(v[0], gs[0]) and torch.equal(v[2], gs[2]) and not v[1].any()
    assert torch.equal(b.stats(), st)
    assert b.nbytes == 4 * (15 + 240 + 5 + 10)
    with pytest.raises(ValueError):
        b.pack([torch.zeros(4, 3), None, None])


def test_view_schedule_partitions_views():
    for world in (1, 2, 4, 8):
        got = [dp.view_schedule(64, world, r, seed=3) for r in range(world)]
        flat = sorted(v for g in got for v in g)
        assert flat == list(range(64))
        assert all(len(g) == 64 // world for g in got)
    assert dp.view_schedule(10, 2, 0, epoch=0) != dp.view_schedule(10, 2, 0, epoch=1)


def test_rank_yaw_and_bounds():
    assert dp.rank_yaw(0, 1) == 0.0
    ys = [dp.rank_yaw(r, 8) for r in range(8)]
    assert ys[0] == -20.0 and ys[-1] == 20.0 and ys == sorted(ys)
    b = dp.allreduce_bound_ms(256 << 20, 8)
    assert 2.5 < b["ring_1link_ms"] < 3.2 and b["all_links_ms"] < b["ring_1link_ms"]


def test_view_schedule_wraps_when_world_does_not_divide():
    for n, world in ((10, 4), (7, 8), (64, 3)):
        got = [dp.view_schedule(n, world, r, seed=1) for r in range(world)]
        steps = -(-n // world)
        assert all(len(g) == steps for g in got)
        assert sorted(set(v for g in got for v in g)) == list(range(n))   # every view at least once


def _finish_worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["means3D", "shs", "opacities", "language_feature_precomp"]
        params = [torch.zeros(6, 3), torch.zeros(6, 16, 3), torch.zeros(6, 1), torch.zeros(6, 16)]
        ex = dp.ViewShardedExchange(params, with_stats=True, names=names)
        assert ex.early is not None and ex.early_idx == [3]
        g = torch.Generator().manual_seed(rank)
        grads = [torch.randn(p.shape, generator=g) for p in params]
        grads[1] = None                                    # a parameter without gradient this step
        m2d = torch.randn(6, 3, generator=g)
        radii = torch.tensor([0, 1, 2, 3, 4, 5], dtype=torch.int32) * (rank + 1)
        red, stats, max_r = ex.finish(m2d, radii, grads)   # the zero-copy path with foreign tensors
        exp = [torch.zeros_like(p) for p in params]
        for r in range(world):
            gr = torch.Generator().manual_seed(r)
            gg = [torch.randn(p.shape, generator=gr) for p in params]
            for i in (0, 2, 3):
                exp[i] += gg[i]
        for i in range(4):
            assert torch.allclose(red[i], exp[i], rtol=0, atol=1e-6), names[i]
        assert torch.equal(max_r, radii // (rank + 1) * world)
        assert float(stats[:, 1].max()) == world
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_exchange_finish_two_buckets_gloo_world2():
    mp.spawn(_finish_worker, args=(2, _free_port()), nprocs=2, join=True)


def test_grad_sink_leaf_identity_and_reuse():
    """GradSink hands out a buffer only for its own leaf (params given) and only
    once per sink (a non-leaf input such as cat(f_dc, f_rest) must
    not receive the bucket view; a second backward must not reuse it)."""
    from langsplatv2_amd.rasterizer import GradSink
    leaf = torch.zeros(4, 3)
    buf = torch.empty(4, 3)
    s = GradSink({"means3D": buf}, params={"means3D": leaf})
    dev = buf.device
    assert s.take("means3D", (4, 3), dev, id(leaf.clone())) is None     # another tensor
    assert s.take("means3D", (4, 2), dev, id(leaf)) is None             # wrong shape
    assert s.take("means3D", (4, 3), dev, id(leaf)) is buf
    assert s.used == {"means3D"}
    with pytest.raises(RuntimeError, match="already written"):
        s.take("means3D", (4, 3), dev, id(leaf))
    s2 = GradSink({"means3D": buf})                                     # no params: any input of that name
    assert s2.take("means3D", (4, 3), dev, 12345) is buf


class _FakeRaster(torch.autograd.Function):
    """What the rasterizer backward does with a GradSink (rasterizer.py backward):
    each input's gradient (2 x upstream) goes into the sink's buffer for that leaf
    when the sink has one, the lang-ready callback runs, and with a factored SH
    sink the colour part goes to rgb_sh and autograd receives sink.sh_return."""

    @staticmethod
    def forward(ctx, names, *xs):
        ctx.names = names
        ctx.ids = [id(x) for x in xs]
        return tuple(x * 2.0 for x in xs)

    @staticmethod
    def backward(ctx, *gs):
        from langsplatv2_amd import rasterizer
        sink = rasterizer._sink()
        out = [None]
        for nm, xid, g in zip(ctx.names, ctx.ids, gs):
            val = 2.0 * g
            buf = sink.take(nm, tuple(g.shape), g.device, xid) if sink is not None else None
            if buf is not None and nm == "shs" and sink.rgb_sh is not None:
                sink.rgb_sh.copy_(val.sum(1))          # the "colour gradient" of this view
                out.append(sink.sh_return if sink.sh_return is not None else buf)
                continue
            if buf is None:
                out.append(val)
            else:
                buf.copy_(val)
                out.append(buf)
        if sink is not None and sink.on_lang_ready is not None:
            sink.on_lang_ready(sink)
        return tuple(out)


def _step(params, names, local, reg, mode):
    """One backward through _FakeRaster whose gradient w.r.t. params[i] is local[i],
    plus (reg not None) a second path adding reg[i]; returns the gradients the
    caller hands finish() (autograd.grad's, or p.grad after loss.backward())."""
    ys = _FakeRaster.apply(names, *params)
    loss = sum((y * (loc / 2.0)).sum() for y, loc in zip(ys, local))
    if reg is not None:
        loss = loss + sum((p * r).sum() for p, r in zip(params, reg))
    if mode == "grad":
        return list(torch.autograd.grad(loss, params))
    for p in params:
        p.grad = None
    loss.backward()
    return [p.grad for p in params]


def test_early_allreduce_starts_from_the_leaf_hook():
    """The early (language) all-reduce starts from the language leaf's gradient
    hook, i.e. only once autograd has the leaf's total gradient, and never
    without a collective."""
    names = ["means3D", "language_feature_precomp"]
    params = [torch.zeros(5, 3, requires_grad=True), torch.zeros(5, 16, requires_grad=True)]
    ex = dp.ViewShardedExchange(params, with_stats=False, names=names)
    assert not ex.collective
    with ex.sink():
        _step(params, names, [torch.ones(5, 3), torch.ones(5, 16)], None, "grad")
    assert ex._early_work is None and ex._hooks == []   # world 1: no hooks, no collective
    ex.collective = True                                # as with force_collectives, minus the process group
    launched = []
    ex._launch_early = lambda after_pack=True: launched.append(after_pack)
    loc = [torch.ones(5, 3), torch.full((5, 16), 3.0)]
    with ex.sink():
        g = _step(params, names, loc, None, "grad")
    assert launched == [False]                           # the view itself: no pack, the lang-ready event
    assert torch.equal(ex._views()[1], loc[1]) and g[1].data_ptr() == ex._views()[1].data_ptr()
    with ex.sink():
        _step(params, names, loc, [torch.zeros(5, 3), torch.ones(5, 16)], "grad")
    assert launched == [False, True]                     # a second path: the sum packed first
    assert torch.equal(ex._views()[1], loc[1] + 1.0)
    ex._remove_hooks()


def _hook_worker(rank, world, port):
    """the zero-copy exchange with loss.backward() or
    autograd.grad, with and without a second gradient path into every bucketed
    leaf (a regulariser).  The early all-reduce starts inside the backward (from
    the language leaf's hook), and every reduced gradient equals the sum over
    ranks of (rasterizer part + regulariser part), in every mode, without any
    debug switch."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["means3D", "opacities", "language_feature_precomp"]
        params = [torch.zeros(7, 3, requires_grad=True), torch.zeros(7, 1, requires_grad=True),
                  torch.zeros(7, 16, requires_grad=True)]
        ex = dp.ViewShardedExchange(params, with_stats=False, names=names)

        def parts(r):
            gr = torch.Generator().manual_seed(10 + r)
            loc = [torch.randn(p.shape, generator=gr) for p in params]
            reg = [torch.randn(p.shape, generator=gr) for p in params]
            return loc, reg
        for mode in ("grad", "backward"):
            for multipath in (False, True):
                loc, reg = parts(rank)
                with ex.sink():
                    grads = _step(params, names, loc, reg if multipath else None, mode)
                assert ex._early_work is not None, (mode, multipath)   # started inside the backward
                red, _, _ = ex.finish(None, None, grads)
                for i in range(3):
                    exp = torch.zeros_like(params[i])
                    for r in range(world):
                        lo, rg = parts(r)
                        exp += lo[i] + (rg[i] if multipath else 0.0)
                    assert torch.allclose(red[i], exp, rtol=0, atol=1e-5), (mode, multipath, names[i])
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_exchange_hooks_multipath_gloo_world2():
    mp.spawn(_hook_worker, args=(2, _free_port()), nprocs=2, join=True)


def _factored_worker(rank, world, port):
    """The view-factored SH leaf with a second gradient path: the backward hands
    autograd an expanded zero (GradSink.sh_return), so the leaf's hook sees exactly
    the other path's gradient, which finish() all-reduces and adds to the rebuilt
    sum (dp.py:_sh_hook).  sh_grad_from_views is replaced by a host stand-in
    (the kernel is GPU code; tests/test_sh_factored.py covers it on the GPU)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def fake_rebuild(means3D, campos, drgb, deg, out):
            out.copy_(drgb.sum(0).unsqueeze(1).expand(out.shape))
            return out
        dp.sh_grad_from_views = fake_rebuild
        names = ["means3D", "shs"]
        params = [torch.zeros(6, 3, requires_grad=True), torch.zeros(6, 4, 3, requires_grad=True)]
        ex = dp.ViewShardedExchange(params, with_stats=False, names=names, factor_sh=True)

        def parts(r):
            gr = torch.Generator().manual_seed(40 + r)
            return [torch.randn(p.shape, generator=gr) for p in params], [torch.randn(p.shape, generator=gr)
                                                                          for p in params]
        for multipath in (False, True):
            loc, reg = parts(rank)
            with ex.sink() as sink:
                grads = _step(params, names, loc, reg if multipath else None, "grad")
            assert "shs" in sink.used
            red, _, _ = ex.finish(None, None, grads, campos=torch.zeros(3), means3D=params[0].detach(), sh_degree=1)
            exp_sh = torch.zeros(6, 4, 3)
            exp_m = torch.zeros(6, 3)
            for r in range(world):
                lo, rg = parts(r)
                exp_sh += lo[1].sum(1, keepdim=True).expand(6, 4, 3)
                exp_m += lo[0]
                if multipath:
                    exp_sh += rg[1]
                    exp_m += rg[0]
            assert torch.allclose(red[1], exp_sh, rtol=0, atol=1e-5), multipath
            assert torch.allclose(red[0], exp_m, rtol=0, atol=1e-5), multipath
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_factored_sh_second_path_gloo_world2():
    mp.spawn(_factored_worker, args=(2, _free_port()), nprocs=2, join=True)
