"""Plain-PyTorch CPU restatement of ``AdaptiveHeatmapLoss`` (training loss,
SURVEY §8(f) rank 4).

TEST INFRASTRUCTURE ONLY -- see ``oracle/__init__.py``.  Checked against
goldens from the reference's own module (tests/golden/make_loss_golden.py).

Reference anchors (all paths under /root/reference):
  * AdaptiveHeatmapLoss.__init__ ............ dll/losses/keypoint_loss.py:208-226
  * _compute_adaptive_threshold ............. dll/losses/keypoint_loss.py:228-236
  * forward (masks, MSE, weights, focal, tw) dll/losses/keypoint_loss.py:238-280
torch.quantile (linear interpolation) is restated from its published
definition: sorted values v, rank r = q * (n - 1) in the input dtype,
lerp(v[floor r], v[ceil r], r - floor r).
"""
from __future__ import annotations

from typing import Optional

import torch


def quantile_linear(x: torch.Tensor, q: float) -> torch.Tensor:
    """torch.quantile(x.flatten(), q) for fp32 x (no NaNs): the rank and the
    interpolation weight in fp32, like q converted to the input's dtype."""
    v = torch.sort(x.flatten().float()).values
    n = v.numel()
    rank = torch.tensor(q, dtype=torch.float32) * (n - 1)
    lo = int(rank.floor().item())
    hi = int(rank.ceil().item())
    w = rank - lo
    return torch.lerp(v[lo], v[hi], w)


def adaptive_threshold(gt: torch.Tensor, adaptive: bool = True) -> torch.Tensor:
    """keypoint_loss.py:228-236."""
    if not adaptive:
        return torch.tensor(0.1)
    return torch.clamp(quantile_linear(gt, 0.9), min=0.05, max=0.3)


def adaptive_heatmap_loss(pred: torch.Tensor, gt: torch.Tensor, target_weight: Optional[torch.Tensor] = None,
                          keypoint_weight: float = 50.0, background_weight: float = 1.0, adaptive: bool = True,
                          focal_alpha: float = 2.0) -> torch.Tensor:
    """keypoint_loss.py:238-280 (differentiable w.r.t. pred)."""
    thr = adaptive_threshold(gt, adaptive)
    km = (gt > thr).float()
    bm = (gt <= thr).float()
    mse = (pred - gt) ** 2
    wl = mse * km * keypoint_weight + mse * bm * background_weight
    if focal_alpha > 0:
        wl = wl * (1 - torch.exp(-mse)) ** focal_alpha
    if target_weight is not None:
        wl = wl * target_weight.view(wl.shape[0], wl.shape[1], 1, 1)
    return wl.mean()
