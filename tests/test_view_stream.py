"""view_stream.ViewStream: forwards of a stream of views issued on alternating
HIP streams, two in flight.  The reference renders views one at a time
(eval_lerf.py:320-350); the streamed outputs must equal those, view for view,
bit for bit, and stay valid after later pushes."""
import pytest
import torch

from harness import make_case, settings_for


def _renderer(case, gpu):
    from diff_gaussian_rasterization import GaussianRasterizer
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu))
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations", "language_feature_precomp") if k in t}

    def render():
        with torch.no_grad():
            return r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"], **kw)
    return render


def test_depth_validation():
    from langsplatv2_amd.view_stream import ViewStream
    with pytest.raises(ValueError):
        ViewStream(device="cpu", depth=0)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [1, 2, 3])
def test_stream_equals_view_by_view(gpu, depth):
    from langsplatv2_amd.view_stream import ViewStream
    renders = [_renderer(make_case(N=20000, W=160, H=120, seed=3, sh_degree=3, lang_dim=16, yaw=y), gpu)
               for y in (0.0, 7.0, -5.0, 12.0, 3.0)]
    ref = [tuple(x.clone() for x in f()) for f in renders]
    vs = ViewStream(gpu, depth=depth)
    got = []
    for f in renders:
        out = vs.push(f)
        if out is not None:
            got.append(out)
    got += vs.flush()
    assert len(got) == len(renders) and vs.flush() == []
    torch.cuda.synchronize()
    for g_, r_ in zip(got, ref):
        for a, b in zip(g_, r_):
            assert torch.equal(a, b)
