"""Seeded inputs of the AdaptiveHeatmapLoss golden cases (shared by
make_loss_golden.py and the tests, so the fixture stores outputs + a checksum
of the inputs only)."""
from __future__ import annotations

import torch

# (name, B, K, H, W, gt kind, target weight?, loss kwargs)
CASES = [
    ("gauss_default", 2, 4, 32, 24, "gauss", False, {}),
    ("gauss_tw_alpha15", 2, 4, 32, 24, "gauss", True, {"focal_alpha": 1.5}),
    ("fixed_thr_nofocal", 1, 3, 20, 16, "gauss", False, {"adaptive_threshold": False, "focal_alpha": 0.0}),
    ("uniform_interp", 1, 5, 17, 13, "uniform", True, {"keypoint_weight": 20.0, "background_weight": 2.0}),
    ("ties", 2, 2, 8, 8, "ties", False, {}),
    ("uniform_high", 1, 2, 16, 16, "uniform_high", False, {}),
]


def make_inputs(B, K, H, W, kind, with_tw, seed):
    g = torch.Generator().manual_seed(seed)
    if kind == "gauss":
        ys = torch.arange(H, dtype=torch.float32).view(1, 1, H, 1)
        xs = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W)
        cy = torch.rand(B, K, 1, 1, generator=g) * H
        cx = torch.rand(B, K, 1, 1, generator=g) * W
        gt = torch.exp(-((ys - cy) ** 2 + (xs - cx) ** 2) / (2 * 2.0 ** 2))
    elif kind == "uniform":      # 0.9-quantile inside (0.05, 0.3): the interpolated value is the threshold
        gt = torch.rand(B, K, H, W, generator=g) * 0.25
    elif kind == "uniform_high":  # quantile above 0.3: clamped
        gt = torch.rand(B, K, H, W, generator=g)
    else:                         # few distinct values: the quantile lands on ties
        gt = (torch.randint(0, 4, (B, K, H, W), generator=g).float() * 0.1)
    pred = (gt + 0.2 * torch.randn(B, K, H, W, generator=g)).clamp(0, 1)
    tw = (torch.rand(B, K, generator=g) > 0.3).float() if with_tw else None
    return pred, gt, tw
