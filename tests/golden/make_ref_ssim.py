"""Generate tests/golden/ref_ssim.npz by running the REFERENCE's own loss
utilities (utils/loss_utils.py:18-75: l1_loss, ssim) on seeded CPU images.
Pins langsplatv2_amd/train_loop.py's restatement (tests/test_train_loop.py).
Run:  python tests/golden/make_ref_ssim.py   (needs /root/reference; only the
resulting .npz is committed and travels)."""
import os
import sys

import numpy as np
import torch

REF = os.environ.get("LSR_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
from utils import loss_utils  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_ssim.npz")


def main():
    g = torch.Generator().manual_seed(7)
    out = {}
    for i, (h, w) in enumerate(((24, 32), (40, 28), (11, 17))):
        a = torch.rand(3, h, w, generator=g)
        b = (a + 0.2 * torch.randn(3, h, w, generator=g)).clamp(0, 1)
        out[f"a{i}"] = a.numpy()
        out[f"b{i}"] = b.numpy()
        out[f"ssim{i}"] = np.float32(loss_utils.ssim(a, b).item())
        out[f"l1_{i}"] = np.float32(loss_utils.l1_loss(a, b).item())
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sorted(out))


if __name__ == "__main__":
    main()
