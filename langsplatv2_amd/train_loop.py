"""RGB-phase training iteration of the reference, over the view-sharded
exchange (BASELINE.json cfg4's loop shape).

What it restates (reference file:line):
  * Gaussian parameters and activations: scene/gaussian_model.py:28-32
    (exp scaling, sigmoid opacity, normalised rotation), :153-157 (features =
    cat(f_dc, f_rest)), :180-182 (oneupSHdegree), the Adam groups and learning
    rates of training_setup :234-255 (eps 1e-15);
  * render(): gaussian_renderer/__init__.py:19-129, RGB mode: the screen-space
    points are `zeros_like(xyz, requires_grad=True) + 0` with retain_grad,
    the (1,) placeholder for the language input, SH evaluated by the rasterizer;
  * the loss (1 - lambda_dssim) L1 + lambda_dssim (1 - SSIM): train.py:166-168,
    utils/loss_utils.py:18-71;
  * per-view bookkeeping: max_radii2D over the visibility filter and
    add_densification_stats (train.py:245-251, scene/gaussian_model.py:506-508);
  * the SH-degree ramp every 1000 iterations (train.py:135-136) and the
    optimizer step every `accum_iter` iterations (train.py:261-263).

Data parallelism: each of R ranks renders one view per step, the exchange
(dp.ViewShardedExchange) all-reduces the gradients and the densification
increments and MAX-reduces the radii, then every rank steps its replica — the
same update as `--accum_iter R` on one GPU with the R views in one
accumulation window (only the gradient summation order differs).  One step
advances the iteration counter by R; the SH ramp is applied at step
granularity (all views of a window use the degree active at its first
iteration, so the replicas stay identical).  densify_and_prune itself (clone /
split / prune, scene/gaussian_model.py:422-505) is outside the rasterizer path
and not restated; its inputs (max_radii2D, xyz_gradient_accum, denom) are.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import dp
from .optim import FusedAdam
from .rasterizer import GaussianRasterizationSettings, GaussianRasterizer

PARAM_NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def inverse_sigmoid(x: torch.Tensor) -> torch.Tensor:
    return torch.log(x / (1 - x))


class GaussianState:
    """The reference GaussianModel's tensors for the RGB phase (no language)."""

    def __init__(self, means3D, shs, opacities, scales, rotations, max_sh_degree: int = 3):
        dev = means3D.device
        self._xyz = means3D.detach().clone().contiguous().requires_grad_(True)
        self._features_dc = shs[:, :1].detach().clone().contiguous().requires_grad_(True)
        self._features_rest = shs[:, 1:].detach().clone().contiguous().requires_grad_(True)
        self._opacity = inverse_sigmoid(opacities.detach().clamp(1e-6, 1 - 1e-6)).contiguous().requires_grad_(True)
        self._scaling = torch.log(scales.detach()).contiguous().requires_grad_(True)
        self._rotation = rotations.detach().clone().contiguous().requires_grad_(True)
        self.max_sh_degree = max_sh_degree
        self.active_sh_degree = 0
        n = means3D.shape[0]
        self.max_radii2D = torch.zeros(n, device=dev)
        self.xyz_gradient_accum = torch.zeros(n, 1, device=dev)
        self.denom = torch.zeros(n, 1, device=dev)

    def params(self) -> list[torch.Tensor]:
        return [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return F.normalize(self._rotation)

    def oneup_sh_degree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    def optimizer(self, spatial_lr_scale: float = 1.0, fused: bool = True):
        """training_setup's groups (scene/gaussian_model.py:234-255, OptimizationParams defaults)."""
        groups = [
            {"params": [self._xyz], "lr": 0.00016 * spatial_lr_scale, "name": "xyz"},
            {"params": [self._features_dc], "lr": 0.0025, "name": "f_dc"},
            {"params": [self._features_rest], "lr": 0.0025 / 20.0, "name": "f_rest"},
            {"params": [self._opacity], "lr": 0.05, "name": "opacity"},
            {"params": [self._scaling], "lr": 0.005, "name": "scaling"},
            {"params": [self._rotation], "lr": 0.001, "name": "rotation"},
        ]
        return FusedAdam(groups, lr=0.0, eps=1e-15) if fused else torch.optim.Adam(groups, lr=0.0, eps=1e-15)


def render_rgb(cam: dict, gs: GaussianState, bg: torch.Tensor, scaling_modifier: float = 1.0) -> dict:
    """gaussian_renderer/__init__.py:19-129 for include_feature = False."""
    screenspace_points = torch.zeros_like(gs.get_xyz, dtype=gs.get_xyz.dtype, requires_grad=True) + 0
    screenspace_points.retain_grad()
    dev = gs.get_xyz.device
    rs = GaussianRasterizationSettings(
        image_height=int(cam["H"]), image_width=int(cam["W"]), tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=bg, scale_modifier=scaling_modifier, viewmatrix=cam["viewmatrix"].to(dev),
        projmatrix=cam["projmatrix"].to(dev), sh_degree=gs.active_sh_degree, campos=cam["campos"].to(dev),
        prefiltered=False, debug=False, include_feature=False)
    rasterizer = GaussianRasterizer(raster_settings=rs)
    placeholder = torch.zeros((1,), dtype=gs.get_opacity.dtype, device=dev)
    image, _lang, radii = rasterizer(means3D=gs.get_xyz, means2D=screenspace_points, shs=gs.get_features,
                                     colors_precomp=None, language_feature_precomp=placeholder,
                                     opacities=gs.get_opacity, scales=gs.get_scaling, rotations=gs.get_rotation,
                                     cov3D_precomp=None)
    return {"render": image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0, "radii": radii}


def l1_loss(out: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    return torch.abs(out - gt).mean()


def _gauss_window(window_size: int, sigma: float, channel: int, like: torch.Tensor) -> torch.Tensor:
    g = torch.tensor([math.exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)])
    g = g / g.sum()
    w2 = (g[:, None] @ g[None, :]).float()
    return w2.expand(channel, 1, window_size, window_size).contiguous().to(like.device, like.dtype)


def ssim(img1: torch.Tensor, img2: torch.Tensor, window_size: int = 11) -> torch.Tensor:
    """utils/loss_utils.py:41-71 (ssim / _ssim: 11x11 Gaussian window, sigma 1.5, mean SSIM)."""
    c = img1.size(-3)
    w = _gauss_window(window_size, 1.5, c, img1)
    pad = window_size // 2
    mu1 = F.conv2d(img1, w, padding=pad, groups=c)
    mu2 = F.conv2d(img2, w, padding=pad, groups=c)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, w, padding=pad, groups=c) - mu1_sq
    s2 = F.conv2d(img2 * img2, w, padding=pad, groups=c) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=pad, groups=c) - mu12
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    return (((2 * mu12 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))).mean()


def view_loss(image: torch.Tensor, gt: torch.Tensor, lambda_dssim: float) -> torch.Tensor:
    return (1.0 - lambda_dssim) * l1_loss(image, gt) + lambda_dssim * (1.0 - ssim(image, gt))


def sh_ramp(gs: GaussianState, iteration: int, window: int, interval: int = 1000):
    """train.py:135-136 (oneupSHdegree when iteration % 1000 == 0) for the window
    of iterations iteration+1 .. iteration+window, applied before its first view."""
    for it in range(iteration + 1, iteration + window + 1):
        if it % interval == 0:
            gs.oneup_sh_degree()


@torch.no_grad()
def apply_view_stats(gs: GaussianState, radii: torch.Tensor, stats: torch.Tensor):
    """max_radii2D over the visibility filter and add_densification_stats with the
    (reduced) per-view increments [||dL/d means2D[:, :2]||, visible]."""
    vis = radii > 0
    gs.max_radii2D[vis] = torch.max(gs.max_radii2D[vis], radii[vis].to(gs.max_radii2D.dtype))
    gs.xyz_gradient_accum += stats[:, :1]
    gs.denom += stats[:, 1:2]


class RGBTrainer:
    """One optimizer step per call: this rank renders `view`, the exchange sums
    the R ranks' gradients and statistics, every rank steps its replica."""

    def __init__(self, gs: GaussianState, bg: torch.Tensor, lambda_dssim: float = 0.2, group=None, fused_adam=True,
                 sh_interval: int = 1000):
        self.gs = gs
        self.sh_interval = sh_interval
        self.bg = bg
        self.lambda_dssim = lambda_dssim
        self.opt = gs.optimizer(fused=fused_adam)
        self.exchange = dp.ViewShardedExchange(gs.params(), with_stats=True, group=group, names=list(PARAM_NAMES))
        self.world = self.exchange.world
        self.iteration = 0

    def step(self, cam: dict, gt: torch.Tensor) -> float:
        sh_ramp(self.gs, self.iteration, self.world, self.sh_interval)
        pkg = render_rgb(cam, self.gs, self.bg)
        loss = view_loss(pkg["render"], gt, self.lambda_dssim)
        loss.backward()
        params = self.gs.params()
        grads, stats, max_radii = self.exchange.exchange([p.grad for p in params],
                                                         pkg["viewspace_points"].grad, pkg["radii"])
        apply_view_stats(self.gs, max_radii, stats)
        for p, g in zip(params, grads):
            p.grad = g
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.iteration += self.world
        return float(loss.detach())


def accumulate_views(gs: GaussianState, opt, cams: list, gts: list, bg: torch.Tensor, lambda_dssim: float = 0.2,
                     iteration: int = 0, sh_interval: int = 1000):
    """The single-GPU reference of one DP step: `len(cams)` iterations with
    accum_iter = len(cams) (train.py:245-263): per view, backward into .grad
    (autograd accumulates), max_radii2D / densification stats; one optimizer
    step at the end of the window."""
    sh_ramp(gs, iteration, len(cams), sh_interval)
    losses = []
    for cam, gt in zip(cams, gts):
        pkg = render_rgb(cam, gs, bg)
        loss = view_loss(pkg["render"], gt, lambda_dssim)
        loss.backward()
        apply_view_stats(gs, pkg["radii"], dp.densify_increment(pkg["viewspace_points"].grad, pkg["radii"]))
        losses.append(float(loss.detach()))
    opt.step()
    opt.zero_grad(set_to_none=True)
    return losses


# ----------------------------------------------------------- feature phase ---
# The language-feature phase (BASELINE.json cfg4's step; train.py:139-173 with
# --include_feature --cos_loss, vq_layer_num 1 as the paper and train.sh use):
# geometry frozen, the trainable parameters are the per-Gaussian code logits
# (N, 64) and the codebooks (1, 64, Df) (scene/gaussian_model.py:238-243), the
# render weights are the top-k soft codes (get_render_weights,
# scene/gaussian_model.py:510-518 -> the fused producer), the loss is the cosine
# loss of the decoded feature map against the view's ground truth under its
# mask (train.py:151-166 -> the fused loss, which never forms the Df-wide map).
# No densification in this phase (train.py:245: `if not opt.include_feature`).

LANG_PARAM_NAMES = ("logits", "codebooks")


class LanguageState:
    """Frozen geometry + the trainable language parameters, Adam groups as
    training_setup with include_feature (lr 0.0025 on both, eps 1e-15)."""

    def __init__(self, means3D, shs, opacities, scales, rotations, logits, codebooks, topk: int = 4):
        self.geo = {"means3D": means3D.detach(), "shs": shs.detach(), "opacities": opacities.detach(),
                    "scales": scales.detach(), "rotations": rotations.detach()}
        self.logits = logits.detach().clone().contiguous().requires_grad_(True)
        self.codebooks = codebooks.detach().clone().contiguous().requires_grad_(True)
        # one codebook level (vq_layer_num 1, train.sh and the paper): L levels of K codes
        # would render L*K dense language channels, past the rasterizer's 64
        if self.codebooks.dim() != 3 or self.codebooks.shape[0] != 1:
            raise ValueError("LanguageState: codebooks must be (1, K, Df): vq_layer_num 1 (the paper's setting)")
        self.topk = topk
        self.active_sh_degree = 3

    def params(self):
        return [self.logits, self.codebooks]

    def optimizer(self, fused: bool = True):
        groups = [{"params": [self.logits, self.codebooks], "lr": 0.0025, "name": "language_feature"}]
        if fused:
            return FusedAdam(groups, lr=0.0, eps=1e-15)
        return torch.optim.Adam(groups, lr=0.0, eps=1e-15)


def render_language(cam: dict, ls: LanguageState, bg: torch.Tensor) -> dict:
    """gaussian_renderer/__init__.py:19-129 for include_feature = True: dense
    top-k render weights, (1,) placeholders for the quick inputs, screen-space
    points `zeros_like(xyz, requires_grad=True) + 0` with retain_grad."""
    from . import lang_codes
    xyz = ls.geo["means3D"]
    dev = xyz.device
    screenspace_points = torch.zeros_like(xyz, requires_grad=True) + 0
    screenspace_points.retain_grad()
    K = ls.codebooks.shape[1]
    weights = lang_codes.get_render_weights(ls.logits, 1, K, ls.topk)
    placeholder = torch.zeros((1,), dtype=xyz.dtype, device=dev)
    rs = GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"], bg=bg,
        scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev), projmatrix=cam["projmatrix"].to(dev),
        sh_degree=ls.active_sh_degree, campos=cam["campos"].to(dev), prefiltered=False, debug=False,
        include_feature=True)
    image, weight_map, radii = GaussianRasterizer(rs)(
        means3D=xyz, means2D=screenspace_points, shs=ls.geo["shs"], colors_precomp=None,
        language_feature_precomp=weights, language_feature_weights_quick=placeholder,
        language_feature_indices=placeholder, opacities=ls.geo["opacities"], scales=ls.geo["scales"],
        rotations=ls.geo["rotations"], cov3D_precomp=None)
    return {"render": image, "language_feature_weight_map": weight_map, "viewspace_points": screenspace_points,
            "radii": radii}


def language_view_loss(pkg: dict, ls: LanguageState, seg: torch.Tensor, features: torch.Tensor,
                       normalize: bool = False, cos: bool = True, l1: bool = False,
                       iteration: int = 0) -> torch.Tensor:
    """train.py:151-167: the decoded feature map of level layer_idx =
    min(int(iteration / 10000 * layer_num), layer_num - 1) (always 0 with the
    single codebook level this phase trains, see LanguageState) against the
    view's ground truth gathered from its (S, Df) table by its segment map,
    under the --normalize / --cos_loss / --l1_loss flags (default: train.sh's
    --cos_loss alone, the fused kernel)."""
    from .lang_loss import language_feature_loss
    layer_num = ls.codebooks.shape[0]
    layer_idx = min(int(iteration / 10000 * layer_num), layer_num - 1)
    return language_feature_loss(pkg["language_feature_weight_map"], ls.codebooks, seg, features,
                                 layer_idx=layer_idx, normalize=normalize, cos=cos, l1=l1)


class LanguageTrainer:
    """One optimizer step per call in the feature phase: this rank renders its
    view, the exchange sums the R ranks' (logits, codebooks) gradients in one
    bucket, every rank steps its replica (= --accum_iter R on one GPU)."""

    def __init__(self, ls: LanguageState, bg: torch.Tensor, group=None, fused_adam: bool = True,
                 normalize: bool = False, cos_loss: bool = True, l1_loss: bool = False):
        self.ls = ls
        self.bg = bg
        self.loss_flags = dict(normalize=normalize, cos=cos_loss, l1=l1_loss)   # train.py --normalize / --cos_loss / --l1_loss
        self.opt = ls.optimizer(fused=fused_adam)
        self.exchange = dp.ViewShardedExchange(ls.params(), with_stats=False, group=group,
                                               names=list(LANG_PARAM_NAMES))
        self.world = self.exchange.world
        self.iteration = 0

    def step(self, cam: dict, seg: torch.Tensor, features: torch.Tensor) -> float:
        pkg = render_language(cam, self.ls, self.bg)
        loss = language_view_loss(pkg, self.ls, seg, features, iteration=self.iteration, **self.loss_flags)
        loss.backward()
        params = self.ls.params()
        grads, _, _ = self.exchange.exchange([p.grad for p in params])
        self.last_grads = grads   # views of the reduced bucket (valid until the next step)
        for p, g in zip(params, grads):
            p.grad = g
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.iteration += self.world
        return float(loss.detach())


def accumulate_language_views(ls: LanguageState, opt, cams: list, segs: list, feats: list, bg: torch.Tensor,
                              grads_out: list | None = None, **loss_flags):
    """Single-GPU reference of one feature-phase DP step: len(cams) iterations
    with accum_iter = len(cams) (train.py:261-263), one optimizer step
    (`grads_out` receives copies of the accumulated gradients it steps with)."""
    losses = []
    for cam, seg, feat in zip(cams, segs, feats):
        pkg = render_language(cam, ls, bg)
        loss = language_view_loss(pkg, ls, seg, feat, **loss_flags)
        loss.backward()
        losses.append(float(loss.detach()))
    if grads_out is not None:
        grads_out[:] = [p.grad.detach().clone() for p in ls.params()]
    opt.step()
    opt.zero_grad(set_to_none=True)
    return losses


__all__ = ["GaussianState", "render_rgb", "sh_ramp", "l1_loss", "ssim", "view_loss", "apply_view_stats", "RGBTrainer",
           "accumulate_views", "PARAM_NAMES", "LanguageState", "render_language", "language_view_loss",
           "LanguageTrainer", "accumulate_language_views", "LANG_PARAM_NAMES"]
