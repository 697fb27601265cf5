"""Generates tests/golden/oracle_*.npz: forward + backward outputs of the C
oracle on seeded synthetic cases (SURVEY.md §8c fixtures cfg1_rgb,
small_lang16, quick192; sizes reduced to keep the files small).

Inputs are generated from seeds by langsplatv2_amd.scenes and STORED in the
fixture (prefix in_ / cam_): torch's CPU transcendental kernels take
ISA-dependent SIMD paths, so regenerating on another host's CPU can change
last bits.  Tests rebuild the case from the stored inputs (`load_case`).

    python tests/golden/make_oracle_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.dirname(HERE)]

CASES = {
    "cfg1_rgb": dict(N=1000, W=128, H=128, seed=0, sh_degree=None),
    "small_lang16": dict(N=4000, W=160, H=128, seed=1, sh_degree=3, lang_dim=16),
    "quick192": dict(N=2000, W=48, H=40, seed=2, sh_degree=3, quick_k=4),
}


def build_case(name):
    from harness import make_case
    return make_case(**CASES[name])


def load_case(npz):
    """The case (camera + Gaussians) exactly as stored in a fixture."""
    import torch
    cam = {k[4:]: (torch.from_numpy(npz[k]) if npz[k].ndim else npz[k].item()) for k in npz if k.startswith("cam_")}
    cam["W"], cam["H"] = int(cam["W"]), int(cam["H"])
    g = {k[3:]: torch.from_numpy(npz[k]) for k in npz if k.startswith("in_")}
    for k in ("sh_degree", "quick_dim"):
        if "meta_" + k in npz:
            g[k] = int(npz["meta_" + k])
    return dict(cam=cam, g=g, bg=tuple(float(x) for x in npz["meta_bg"]),
                scale_modifier=float(npz["meta_scale_modifier"]), quick=bool(npz["meta_quick"]))


def input_digest(case):
    h = hashlib.sha256()
    for k in sorted(case["g"]):
        v = case["g"][k]
        if hasattr(v, "numpy"):
            h.update(k.encode())
            h.update(np.ascontiguousarray(v.numpy()).tobytes())
    for k in ("viewmatrix", "projmatrix", "campos"):
        h.update(np.ascontiguousarray(case["cam"][k].numpy()).tobytes())
    return h.hexdigest()


def upstream_grads(case, seed=1):
    cam, g = case["cam"], case["g"]
    rng = np.random.default_rng(seed)
    dC = rng.standard_normal((3, cam["H"], cam["W"])).astype(np.float32)
    D = g["language_feature_precomp"].shape[1] if ("language_feature_precomp" in g and not case["quick"]) else 0
    dL = rng.standard_normal((D, cam["H"], cam["W"])).astype(np.float32) if D else None
    return dC, dL


def run(name, case=None):
    from oracle import oracle as O
    from harness import oracle_problem
    case = build_case(name) if case is None else case
    pb = oracle_problem(case)
    fwd = O.forward(pb, nthreads=8)
    dC, dL = upstream_grads(case)
    bwd = O.backward(pb, fwd, dC, dL)
    out = dict(digest=np.array(input_digest(case)), num_rendered=np.array(fwd["num_rendered"]),
               meta_bg=np.array(case["bg"], np.float32), meta_scale_modifier=np.array(case["scale_modifier"]),
               meta_quick=np.array(case["quick"]),
               radii=fwd["radii"], color=fwd["color"], lang=fwd["lang"], final_T=fwd["final_T"],
               n_contrib=fwd["n_contrib"], point_list=fwd["point_list"], ranges=fwd["ranges"])
    for k, v in case["g"].items():
        if hasattr(v, "numpy"):
            out["in_" + k] = v.numpy()
        else:
            out["meta_" + k] = np.array(v)
    for k, v in case["cam"].items():
        out["cam_" + k] = v.numpy() if hasattr(v, "numpy") else np.array(v)
    for k in ("dmean2D", "dmeans3D", "dopacity", "dcolors", "dsh", "dscales", "drot", "dlang"):
        if bwd.get(k) is not None:
            out["grad_" + k] = bwd[k]
    return out


if __name__ == "__main__":
    # an existing fixture's stored inputs are reused (regenerating the inputs
    # on another host could change their last bits); --fresh rebuilds them
    fresh = "--fresh" in sys.argv
    for name in CASES:
        path = os.path.join(HERE, f"oracle_{name}.npz")
        case = None if fresh or not os.path.exists(path) else load_case(np.load(path))
        out = run(name, case)
        np.savez_compressed(path, **out)
        print(name, os.path.getsize(path), "bytes", {k: v.shape for k, v in out.items()})
