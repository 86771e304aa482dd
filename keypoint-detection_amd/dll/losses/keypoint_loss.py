"""AdaptiveHeatmapLoss on the device (reference dll/losses/keypoint_loss.py:202-280).

Same constructor and forward signature as the reference module.  The forward
and its gradient with respect to the predicted heatmaps run in one native call
(``kpd_adaptive_heatmap_loss``: radix-select quantile, fused weighted focal
MSE, deterministic reduction); autograd receives the gradient through a
``torch.autograd.Function``.  There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

from typing import Optional

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
