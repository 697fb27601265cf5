"""Decoders for the forward workspaces (geom / binning / image buffers) of
liblsr.so — the Python mirror of GeomLayout / ImageLayout / BinLayout in
csrc/lsr_device.h.  Used by the parity tests to compare the GPU's internal
index work (tile lists, ranges, per-Gaussian records) with the oracle."""
from __future__ import annotations

import torch


def _a(x: int) -> int:
    return (x + 255) & ~255


def geom_layout(N: int) -> dict:
    o, L = 0, {}
    for name, nb in (("splatA", N * 16), ("splatB", N * 16), ("rgb", N * 12), ("depth", N * 4), ("tiles", N * 4),
                     ("offsets", N * 4), ("clamped", N * 4), ("scan_part", ((N + 4095) // 4096 + 1) * 8),
                     ("shjac", N * 36), ("flags", 256)):
        L[name] = o
        o += _a(nb)
    L["total"] = o
    return L


def image_layout(P: int, T: int) -> dict:
    o, L = 0, {}
    for name, nb in (("final_T", P * 4), ("n_contrib", P * 4), ("tile_cnt", T * 4), ("tile_start", (T + 1) * 4),
                     ("tile_part", ((T + 63) // 64 + 1) * 8), ("cls_cnt", 512), ("cls_list", T * 6 * 4),
                     ("border", T * 4 * 16)):
        L[name] = o
        o += _a(nb)
    L["total"] = o
    return L


def bin_layout(M: int) -> dict:
    o, L = 0, {}
    for name, nb in (("rank", M * 4), ("keys", M * 8), ("point_list", M * 4)):
        L[name] = o
        o += _a(nb)
    L["total"] = o
    return L


def _view(buf: torch.Tensor, off: int, n: int, dtype) -> torch.Tensor:
    esz = torch.tensor([], dtype=dtype).element_size()
    return buf[off:off + n * esz].view(dtype)


def decode(bufs: dict, N: int, W: int, H: int, M: int) -> dict:
    """bufs: {0: geom, 1: binning, 2: image} uint8 tensors from the allocator."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    G, I, B = geom_layout(N), image_layout(W * H, T), bin_layout(M)
    geom, binning, image = bufs[0], bufs[1], bufs[2]
    sA = _view(geom, G["splatA"], N * 4, torch.float32).view(N, 4)
    sB = _view(geom, G["splatB"], N * 4, torch.float32).view(N, 4)
    out = dict(
        xy=sA[:, :2], conic_opacity=torch.stack([sA[:, 2], sA[:, 3], sB[:, 0], sB[:, 1]], 1), cut=sB[:, 2],
        depth=_view(geom, G["depth"], N, torch.float32),
        rgb=_view(geom, G["rgb"], N * 3, torch.float32).view(N, 3),
        tiles_touched=_view(geom, G["tiles"], N, torch.int32),
        clamped=_view(geom, G["clamped"], N, torch.int32),
        final_T=_view(image, I["final_T"], W * H, torch.float32).view(H, W),
        n_contrib=_view(image, I["n_contrib"], W * H, torch.int32).view(H, W),
        tile_start=_view(image, I["tile_start"], T + 1, torch.int32),
        point_list=_view(binning, B["point_list"], M, torch.int32) if M else torch.zeros(0, dtype=torch.int32),
    )
    ts = out["tile_start"]
    out["ranges"] = torch.stack([ts[:-1], ts[1:]], 1)
    return out
