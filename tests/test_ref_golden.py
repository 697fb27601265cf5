"""The oracle and the package's edge restatements against golden vectors
produced by the REFERENCE's own Python (tests/golden/make_ref_golden.py)."""
import math
import os

import numpy as np
import pytest
import torch

from langsplatv2_amd import scenes

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_utils.npz"))


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_eval_matches_reference(oracle_lib, deg):
    # reference layout [N, C=3, 16] -> 3DGS/oracle layout [N, 16, 3]
    sh = np.transpose(G["sh_coeffs"], (0, 2, 1))
    got = oracle_lib.sh_eval(deg, sh, G["sh_dirs"])
    ref = G[f"sh_eval_deg{deg}"]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-6)


def test_rotation_and_covariance_match_reference(oracle_lib):
    q = G["cov_quats"].astype(np.float32)
    qn = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)  # caller-normalised (gaussian_model.py:146)
    np.testing.assert_allclose(oracle_lib.quat_to_R(qn), G["rotmat"], rtol=1e-5, atol=1e-6)
    cov = oracle_lib.cov3D(G["cov_scales"], qn)
    scale = np.abs(G["cov3D"]).max(axis=1, keepdims=True)
    np.testing.assert_allclose(cov / scale, G["cov3D"] / scale, atol=2e-6)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_camera_matrices_match_reference(i):
    W, H, fovx_deg, yaw = G[f"cam{i}_params"]
    R, T = G[f"cam{i}_R"], G[f"cam{i}_T"]
    wv = torch.tensor(scenes.get_world2view2(R, T)).transpose(0, 1)
    tx = math.tan(math.radians(fovx_deg) / 2)
    proj = scenes.get_projection_matrix(0.01, 100.0, 2 * math.atan(tx), 2 * math.atan(tx * H / W)).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
    np.testing.assert_allclose(wv.numpy(), G[f"cam{i}_world_view"], rtol=0, atol=0)
    np.testing.assert_allclose(full.numpy(), G[f"cam{i}_full_proj"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(wv.inverse()[3, :3].numpy(), G[f"cam{i}_center"], rtol=1e-6, atol=1e-6)
    if T.any() == 0 and yaw == 0:
        cam = scenes.make_camera(int(W), int(H), fovx_deg)
        np.testing.assert_allclose(cam["viewmatrix"].numpy(), G[f"cam{i}_world_view"], atol=0)


def test_language_codes_match_reference():
    """Input synthesis (scenes.py) and the oracle against utils/vq_utils.py:9-40."""
    logits = torch.from_numpy(G["lang_logits"])
    np.testing.assert_allclose(scenes.softmax_to_topk_soft_code(logits, 4).numpy(), G["lang_topk4"],
                               rtol=1e-6, atol=1e-7)
    w, idx = scenes.get_weights_and_indices(logits, 4)
    np.testing.assert_allclose(w.numpy(), G["lang_quick_w"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(idx.numpy(), G["lang_quick_idx"])
    # indices are fp32-encoded integers in ascending channel order (utils/vq_utils.py:38)
    assert np.all(np.diff(G["lang_quick_idx"], axis=1) > 0)


@pytest.mark.parametrize("k", [1, 4, 8])
def test_oracle_topk_codes_match_reference(k):
    from oracle import oracle as O
    np.testing.assert_allclose(O.topk_soft_code(G["lang_logits"], k), G[f"lang_topk{k}"], rtol=1e-6, atol=1e-7)


def test_oracle_topk_code_grad_matches_reference_autograd():
    from oracle import oracle as O
    d = O.topk_soft_code_backward(G["lang_logits"], G["lang_grad_up"], 4)
    ref = G["lang_topk4_dlogits"]
    np.testing.assert_allclose(d, ref, rtol=0, atol=2e-6 * max(1.0, np.abs(ref).max()))


def test_oracle_multilevel_codes_match_reference():
    from oracle import oracle as O
    x = G["lang3_logits"]
    np.testing.assert_allclose(O.topk_soft_code(x, 4, levels=3), G["lang3_render_weights"], rtol=1e-6, atol=1e-7)
    w, idx = O.weights_and_indices(x, 4, levels=3)
    np.testing.assert_allclose(w, G["lang3_quick_w"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(idx, G["lang3_quick_idx"].astype(np.int64))
