"""quick.QuickFeatureStream: render + decode over a stream of views with each
decode overlapping the next render (two HIP streams).  The reference renders
and decodes view after view (eval_lerf.py:210-220, :320-350); the streamed
features must equal that sequence's, frame for frame, bit for bit, and stay
valid after later pushes (the decode stream's outputs are handed to the
caller's stream)."""
import pytest
import torch

from harness import make_case, settings_for

QUICK = dict(N=4000, W=96, H=64, sh_degree=None, quick_k=4, seed=4)


def _renderer(case, gpu, layout):
    from diff_gaussian_rasterization import GaussianRasterizer
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu, layout))
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations") if k in t}

    def render():
        with torch.no_grad():
            return r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                     language_feature_weights_quick=t["language_feature_weights_quick"],
                     language_feature_indices=t["language_feature_indices"], **kw)[1]
    return render


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["chw", None])
def test_stream_equals_view_by_view(gpu, layout):
    from langsplatv2_amd import quick
    renders = [_renderer(make_case(**dict(QUICK, yaw=y)), gpu, layout) for y in (0.0, 6.0, -9.0, 3.0)]
    cb = torch.randn(3, 64, 512, generator=torch.Generator().manual_seed(8)).to(gpu)
    ref = [quick.decode_language_features(f(), cb) for f in renders]
    fs = quick.QuickFeatureStream(cb)
    got = []
    for f in renders:
        prev = fs.push(f)
        if prev is not None:
            got.append(prev)
    assert len(got) == len(renders) - 1
    got.append(fs.flush())
    assert fs.flush() is None
    torch.cuda.synchronize()
    for g_, r_ in zip(got, ref):
        assert torch.equal(g_, r_)


@pytest.mark.gpu
def test_stream_outputs_survive_later_frames(gpu):
    """Outputs handed back stay intact while later frames render and decode
    (their memory is not reused under them), also without a synchronize."""
    from langsplatv2_amd import quick
    render = _renderer(make_case(**QUICK), gpu, "hwc")
    cb = torch.randn(3, 64, 512, generator=torch.Generator().manual_seed(9)).to(gpu)
    ref = quick.decode_language_features(render(), cb).clone()
    fs = quick.QuickFeatureStream(cb, normalize=True)
    outs = [fs.push(render) for _ in range(6)][1:] + [fs.flush()]
    sums = torch.stack([o.double().sum() for o in outs])
    torch.cuda.synchronize()
    assert all(torch.equal(o, ref) for o in outs)
    assert torch.all(sums == ref.double().sum())
