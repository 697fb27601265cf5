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


def test_early_allreduce_only_when_backward_wrote_the_early_bucket():
    """The early (language) all-reduce is launched from the sink callback only
    when every early-bucket view was written by the backward."""
    names = ["means3D", "language_feature_precomp"]
    params = [torch.zeros(5, 3), torch.zeros(5, 16)]
    ex = dp.ViewShardedExchange(params, with_stats=False, names=names)
    launched = []
    ex._launch_early = lambda: launched.append(1)
    sink = ex.sink()
    ex._on_lang_ready(sink)                       # language input had no grad: nothing written
    assert launched == []
    sink.used.add("language_feature_precomp")
    ex._on_lang_ready(sink)
    assert launched == [1]


def _backward_pattern_worker(rank, world, port):
    """loss.backward() inside `with ex.sink():` -- the backward writes
    the bucket views through the sink (and the early all-reduce starts from the
    lang-ready callback), but AccumulateGrad leaves COPIES of the views in
    p.grad, so finish() receives gradients that are not the views.  It must take
    the views (not raise, not re-pack over the running all-reduce)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["means3D", "opacities", "language_feature_precomp"]
        params = [torch.zeros(7, 3), torch.zeros(7, 1), torch.zeros(7, 16)]
        ex = dp.ViewShardedExchange(params, with_stats=False, names=names)
        g = torch.Generator().manual_seed(10 + rank)
        local = [torch.randn(p.shape, generator=g) for p in params]
        sink = ex.sink()
        for nm, p, loc in zip(names, params, local):      # what the rasterizer backward does
            buf = sink.take(nm, tuple(p.shape), p.device, id(p))
            assert buf is not None
            buf.copy_(loc)
        ex._on_lang_ready(sink)                           # early (language) all-reduce starts now
        assert ex._early_work is not None
        copies = [loc.clone() for loc in local]           # AccumulateGrad's copies in p.grad
        red, _, _ = ex.finish(None, None, copies)
        exp = [torch.zeros_like(p) for p in params]
        for r in range(world):
            gr = torch.Generator().manual_seed(10 + r)
            for i, p in enumerate(params):
                exp[i] += torch.randn(p.shape, generator=gr)
        for i in range(3):
            assert torch.allclose(red[i], exp[i], rtol=0, atol=1e-6), names[i]
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_exchange_finish_after_backward_pattern_gloo_world2():
    mp.spawn(_backward_pattern_worker, args=(2, _free_port()), nprocs=2, join=True)


def _multipath_worker(rank, world, port):
    """a bucketed leaf that ALSO gets gradient from outside the
    rasterizer (a regulariser): autograd hands finish() the SUM, while the
    bucket view holds only the rasterizer's part.  finish() must pack the sum for
    the main bucket; for an early-bucket view whose all-reduce is already in
    flight it cannot, and LSR_DP_DEBUG=1 makes that an error instead of a silent
    drop."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["means3D", "opacities", "language_feature_precomp"]
        params = [torch.zeros(5, 3), torch.zeros(5, 1), torch.zeros(5, 16)]
        ex = dp.ViewShardedExchange(params, with_stats=False, names=names)
        g = torch.Generator().manual_seed(20 + rank)
        local = [torch.randn(p.shape, generator=g) for p in params]
        reg = [torch.randn(p.shape, generator=g) for p in params]
        sink = ex.sink()
        for nm, p, loc in zip(names, params, local):
            sink.take(nm, tuple(p.shape), p.device, id(p)).copy_(loc)
        # no early all-reduce started (e.g. the language input took no lang-ready
        # callback): every view may be packed with autograd's sums
        sums = [loc + rg for loc, rg in zip(local, reg)]
        red, _, _ = ex.finish(None, None, sums)
        exp = [torch.zeros_like(p) for p in params]
        for r in range(world):
            gr = torch.Generator().manual_seed(20 + r)
            lo = [torch.randn(p.shape, generator=gr) for p in params]
            rg = [torch.randn(p.shape, generator=gr) for p in params]
            for i in range(3):
                exp[i] += lo[i] + rg[i]
        for i in range(3):
            assert torch.allclose(red[i], exp[i], rtol=0, atol=1e-5), names[i]
        # the early bucket in flight + a foreign contribution: an error in debug mode
        sink = ex.sink()
        for nm, p, loc in zip(names, params, local):
            sink.take(nm, tuple(p.shape), p.device, id(p)).copy_(loc)
        ex._on_lang_ready(sink)
        assert ex._early_work is not None
        os.environ["LSR_DP_DEBUG"] = "1"
        with pytest.raises(RuntimeError, match="early all-reduce already started"):
            ex.finish(None, None, sums)
        ex._early_work.wait()
        dist.barrier()
    finally:
        os.environ.pop("LSR_DP_DEBUG", None)
        dist.destroy_process_group()


def test_exchange_finish_packs_multipath_sums_gloo_world2():
    mp.spawn(_multipath_worker, args=(2, _free_port()), nprocs=2, join=True)
