"""The keypoint losses (reference dll/losses/keypoint_loss.py).

* ``AdaptiveHeatmapLoss`` (:202-280) on the device: the forward and its
  gradient with respect to the predicted heatmaps run in one native call
  (``kpd_adaptive_heatmap_loss``: radix-select quantile, fused weighted focal
  MSE, deterministic reduction); autograd receives the gradient through a
  ``torch.autograd.Function``.  There is no CPU path: CPU tensors raise.
* ``KeypointLoss`` = ``ImprovedKeypointLoss`` (:283-393): that heatmap term
  plus the coordinate term (``SpatialCoordinateLoss``, :117-199) and a
  cross-entropy over the 3 visibility classes, mixed by the stateful
  ``DynamicLossBalancer`` (:28-114).  The two small terms are elementwise
  torch ops on [B, P, K] tensors (host-side glue of the eval forward with
  targets, keypoint_model.py:208-209, 509-584); the balancer's weights are
  Python floats, as in the reference.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from .. import _native


class _AdaptiveHeatmapLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, target_weight, kw, bw, adaptive, alpha):
        loss, grad, thr = _native.adaptive_heatmap_loss(pred, gt, target_weight, kw, bw, adaptive, alpha,
                                                        want_grad=pred.requires_grad)
        ctx.save_for_backward(grad if grad is not None else torch.empty(0, device=pred.device))
        ctx.pred_dtype = pred.dtype
        ctx.threshold = thr
        return loss.to(pred.dtype)     # the reference's loss has pred's dtype

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        if grad.numel() == 0:
            return (None,) * 7
        return (grad * g).to(ctx.pred_dtype), None, None, None, None, None, None


class AdaptiveHeatmapLoss(nn.Module):
    """Adaptive heatmap loss with region-specific weighting (keypoint vs
    background regions) and focal weighting of hard examples
    (reference keypoint_loss.py:202-280)."""

    def __init__(self, keypoint_weight: float = 50.0, background_weight: float = 1.0,
                 adaptive_threshold: bool = True, focal_alpha: float = 2.0):
        super().__init__()
        self.keypoint_weight = keypoint_weight
        self.background_weight = background_weight
        self.adaptive_threshold = adaptive_threshold
        self.focal_alpha = focal_alpha

    def _compute_adaptive_threshold(self, gt_heatmaps: torch.Tensor) -> torch.Tensor:
        """clamp(quantile(gt, 0.9), 0.05, 0.3), or 0.1 (reference :229-236)."""
        if not self.adaptive_threshold:
            return torch.tensor(0.1, device=gt_heatmaps.device)
        g = gt_heatmaps if gt_heatmaps.dim() == 4 else gt_heatmaps.reshape(1, 1, 1, -1)
        _, _, thr = _native.adaptive_heatmap_loss(g, g, None, self.keypoint_weight, self.background_weight, True,
                                                  0.0, want_grad=False)
        return thr

    def forward(self, pred_heatmaps: torch.Tensor, gt_heatmaps: torch.Tensor,
                target_weight: Optional[torch.Tensor] = None) -> torch.Tensor:
        # (checked here: inside an autograd Function's forward grad mode is always off)
        if torch.is_grad_enabled() and gt_heatmaps.requires_grad:
            raise NotImplementedError("AdaptiveHeatmapLoss: the gradient with respect to gt_heatmaps is not "
                                      "implemented (only d loss / d pred_heatmaps)")
        return _AdaptiveHeatmapLossFn.apply(pred_heatmaps, gt_heatmaps, target_weight, self.keypoint_weight,
                                            self.background_weight, self.adaptive_threshold, self.focal_alpha)


@dataclass
class LossMetrics:
    """Per-call loss components (reference :19-25)."""
    total_loss: float
    heatmap_loss: float
    coordinate_loss: float
    visibility_loss: float
    loss_weights: Dict[str, float]


class DynamicLossBalancer:
    """Per-component loss weights nudged toward the median component
    (reference :28-114).  Every call appends the components to a 100-deep
    history; every 10th call (once the heatmap history holds 10 values) each
    weight is scaled by 1 + rate * (median / mean_last_10 - 1), clamped to
    [min_weight, max_weight].  The mean divides by 10 whatever the history
    length (reference quirk kept)."""

    HISTORY = 100
    PERIOD = 10

    def __init__(self, initial_weights: Optional[Dict[str, float]] = None, adaptation_rate: float = 0.1,
                 min_weight: float = 0.1, max_weight: float = 10.0):
        self.adaptation_rate = adaptation_rate
        self.min_weight, self.max_weight = min_weight, max_weight
        self.weights = dict(initial_weights) if initial_weights else {"heatmap": 1.0, "coordinate": 1.0,
                                                                     "visibility": 1.0}
        self.loss_history = {k: [] for k in self.weights}
        self.update_count = 0

    def update_weights(self, loss_components: Dict[str, float]) -> Dict[str, float]:
        self.update_count += 1
        for k, v in loss_components.items():
            h = self.loss_history.get(k)
            if h is not None:
                h.append(v)
                del h[:-self.HISTORY]
        if self.update_count % self.PERIOD == 0:
            self._adapt_weights()
        return dict(self.weights)

    def _adapt_weights(self) -> None:
        if len(self.loss_history["heatmap"]) < self.PERIOD:
            return
        recent = {k: (sum(self.loss_history[k][-self.PERIOD:]) / self.PERIOD if self.loss_history[k] else 1.0)
                  for k in self.weights}
        ordered = sorted(recent.values())
        target = ordered[len(ordered) // 2]
        for k, w in self.weights.items():
            if recent[k] > 0:
                scaled = w * (1.0 + (target / recent[k] - 1.0) * self.adaptation_rate)
                self.weights[k] = max(self.min_weight, min(self.max_weight, scaled))


class SpatialCoordinateLoss(nn.Module):
    """Visible-keypoint coordinate loss (reference :117-199): per-coordinate
    smooth-L1 (or MSE / Huber) summed over x, y, masked by visibility > 0,
    scaled by clamp(|pred - gt| / distance_threshold, 1, 3) and
    pixel_weight_scale, summed and divided by the visible count + 1e-8.
    Shapes broadcast exactly as the reference's do (a [B, K] mask against
    [B, P, K] terms)."""

    _CRITERIA = {"smooth_l1": nn.SmoothL1Loss, "mse": nn.MSELoss, "huber": nn.HuberLoss}

    def __init__(self, loss_type: str = "smooth_l1", pixel_weight_scale: float = 100.0,
                 distance_threshold: float = 5.0):
        super().__init__()
        if loss_type not in self._CRITERIA:
            raise ValueError(f"Unsupported loss type: {loss_type}")
        self.loss_type = loss_type
        self.pixel_weight_scale = pixel_weight_scale
        self.distance_threshold = distance_threshold
        self.criterion = self._CRITERIA[loss_type](reduction="none")

    def forward(self, pred_coords: torch.Tensor, gt_coords: torch.Tensor, visibility: torch.Tensor,
                image_size: Tuple[int, int] = (224, 224)) -> torch.Tensor:
        mask = (visibility > 0).float()
        if mask.sum() == 0:
            return torch.tensor(0.0, device=pred_coords.device, requires_grad=True)
        per_kpt = self.criterion(pred_coords, gt_coords).sum(dim=-1) * mask
        dist = torch.norm(pred_coords - gt_coords, dim=-1)
        per_kpt = per_kpt * torch.clamp(dist / self.distance_threshold, min=1.0, max=3.0)
        per_kpt = per_kpt * self.pixel_weight_scale
        return per_kpt.sum() / (mask.sum() + 1e-8)


class ImprovedKeypointLoss(nn.Module):
    """Heatmap + coordinate + visibility loss with dynamic weights (reference
    :283-389).  ``forward(predictions, targets) -> (total, loss_dict)``;
    predictions: 'heatmaps' [B,K,H,W], 'keypoints', 'visibilities' (or
    'visibility') [.., 3]; targets: 'heatmaps', 'keypoints', 'visibility'
    (or 'visibilities') class indices, optional 'target_weight'.  A missing
    pair contributes a 0 term.  Initial weights: heatmap
    config.lambda_keypoint, coordinate 5, visibility config.lambda_visibility."""

    def __init__(self, num_keypoints: int, config, device: Optional[torch.device] = None):
        super().__init__()
        self.num_keypoints = num_keypoints
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.heatmap_loss = AdaptiveHeatmapLoss()
        self.coordinate_loss = SpatialCoordinateLoss()
        self.visibility_loss = nn.CrossEntropyLoss()
        self.loss_balancer = DynamicLossBalancer(initial_weights={
            "heatmap": getattr(config, "lambda_keypoint", 1.0), "coordinate": 5.0,
            "visibility": getattr(config, "lambda_visibility", 1.0)})

    def forward(self, predictions: Dict[str, torch.Tensor], targets: Dict[str, torch.Tensor]):
        ph, pk = predictions.get("heatmaps"), predictions.get("keypoints")
        pv = predictions.get("visibility", predictions.get("visibilities"))
        gh, gk = targets.get("heatmaps"), targets.get("keypoints")
        gv = targets.get("visibilities", targets.get("visibility"))
        zero = lambda: torch.tensor(0.0, device=self.device)  # noqa: E731
        parts = {
            "heatmap": self.heatmap_loss(ph, gh, targets.get("target_weight"))
            if ph is not None and gh is not None else zero(),
            "coordinate": self.coordinate_loss(pk, gk, gv) if pk is not None and gk is not None and gv is not None
            else zero(),
            "visibility": self.visibility_loss(pv.view(-1, pv.size(-1)), gv.view(-1).long())
            if pv is not None and gv is not None else zero(),
        }
        values = {k: v.item() for k, v in parts.items()}
        weights = self.loss_balancer.update_weights(values)
        total = sum(weights[k] * parts[k] for k in parts)
        t = total.item()
        return total, {
            "keypoint_loss": values["heatmap"], "heatmap_loss": values["heatmap"],
            "visibility_loss": values["visibility"], "coordinate_loss": values["coordinate"],
            "total_loss": t, "loss_weights": weights,
            "loss_metrics": LossMetrics(total_loss=t, heatmap_loss=values["heatmap"],
                                        coordinate_loss=values["coordinate"],
                                        visibility_loss=values["visibility"], loss_weights=weights),
        }


KeypointLoss = ImprovedKeypointLoss
