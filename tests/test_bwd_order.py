"""The list-driven backward's dispatch order (render.hip k_bwd_order,
RenderArgs::border, ImageLayout::border).

A training forward ends by sorting the 8x8 blocks of each XCD dispatch range
(xcd_remap's partition of the backward's 4 T-wave grid) by their list length
in 16-candidate groups, heaviest first.  The backward's wave in slot o then
runs block border[o].  Every block must be run exactly once, so the order is
checked as a permutation that keeps each range's natural block strip, in
non-increasing group count, each entry carrying its block's tile range and
list count; the gradients it produces are covered by the
whole-frame and deterministic tests (each block's partial sums are the same
whatever the dispatch order).  Frames below LSR_BWD_ORDER_MIN_BLOCKS blocks
(lsr_internal.h) keep the band order; the cases here are above it.
"""
import numpy as np
import pytest
import torch

from harness import gpu_inputs, make_case, settings_for

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def xcd_ranges(n):
    """xcd_remap's partition of n dispatch slots (lsr_device.h): XCD x owns [lo, lo + len)."""
    q, r = divmod(n, 8)
    out = []
    for x in range(8):
        lo = x * (q + 1) if x < r else r * (q + 1) + (x - r) * q
        out.append((lo, q + (1 if x < r else 0)))
    return out


@pytest.mark.parametrize("N,W,H", [(60000, 1920, 1080), (20000, 1600, 900), (8000, 1056, 1000)])
def test_block_order_is_a_heavy_first_permutation_per_xcd_range(N, W, H):
    from langsplatv2_amd import _lib, layout, rasterizer
    case = make_case(N=N, W=W, H=H, sh_degree=3, lang_dim=16, seed=3)
    rs = settings_for(case, DEV)
    t = gpu_inputs(case, DEV, requires_grad=False)
    e = torch.empty(0, device=DEV)
    with torch.no_grad():
        _, _, _, M, bufs, _, _, _ = rasterizer._run_forward(
            t["means3D"], t.get("shs", e), t.get("colors_precomp", e), t.get("language_feature_precomp", e), e, e,
            t["opacities"], t.get("scales", e), t.get("rotations", e), t.get("cov3D_precomp", e), rs,
            grad_request=_lib.LSR_GWS_GEOM | _lib.LSR_GWS_LANG)
    torch.cuda.synchronize()
    lists = bufs.get(_lib.LSR_BUF_LISTS)
    assert lists is not None, "a training forward writes the block lists"
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    n = 4 * T
    a256 = lambda x: (x + 255) // 256 * 256  # noqa: E731
    lcount = lists[2 * a256(4 * M * 16):2 * a256(4 * M * 16) + 4 * n].view(torch.int32).cpu().numpy()
    L = layout.image_layout(W * H, T)
    img = bufs[_lib.LSR_BUF_IMAGE]
    ent = img[L["border"]:L["border"] + 16 * n].view(torch.int32).cpu().numpy().astype(np.int64).reshape(n, 4)
    border = ent[:, 0]
    tile_start = img[L["tile_start"]:L["tile_start"] + 4 * (T + 1)].view(torch.int32).cpu().numpy().astype(np.int64)
    # each entry carries its block's tile range and list count (the backward's first load)
    assert np.array_equal(ent[:, 1], tile_start[border >> 2])
    assert np.array_equal(ent[:, 2], tile_start[(border >> 2) + 1])
    assert np.array_equal(ent[:, 3], lcount.astype(np.int64)[border])
    groups = np.minimum((lcount.astype(np.int64) + 15) // 16, 63)
    assert sorted(border.tolist()) == list(range(n)), "every block exactly once"
    for lo, ln in xcd_ranges(n):
        part = border[lo:lo + ln]
        # the XCD's slots hold its natural strip of blocks [lo, lo + ln) ...
        assert part.min() == lo and part.max() == lo + ln - 1
        # ... heaviest list first
        g = groups[part]
        assert np.all(g[:-1] >= g[1:]), "descending group count inside the range"
