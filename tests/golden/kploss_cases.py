"""Seeded inputs of the KeypointLoss / eval-with-targets golden sequence
(shared by make_kploss_golden.py and tests/test_loss.py; the fixture stores
outputs + an input checksum only).

One sequence of calls on ONE loss instance, so the DynamicLossBalancer's
history and its every-10th-call adaptation are part of what is pinned."""
from __future__ import annotations

import torch

K = 17
# (B, P, gt heatmaps as [B,P,K,56,56]?, visible fraction).  The reference's
# coordinate term multiplies [B,P,K] by a [B,K] mask, so P must be 1 or B
# (or B = 1): other shapes raise there, and here (test_kploss_bad_shape)
SEQ = [(2, 1, True, 0.7), (3, 3, False, 0.5), (2, 2, True, 0.9), (1, 1, False, 0.6), (2, 2, True, 0.0),
       (4, 1, False, 0.8), (2, 2, True, 0.4), (3, 1, True, 0.7), (1, 3, False, 0.5), (1, 2, True, 1.0),
       (2, 1, False, 0.6), (3, 3, True, 0.3), (2, 2, False, 0.7)]


def make_call(i):
    """(outputs, batch) for call i: model-shaped predictions (one-hot 3-class
    visibilities, sigmoid-range heatmaps) and dataloader-shaped targets."""
    B, P, gt5, frac = SEQ[i]
    g = torch.Generator().manual_seed(1000 + i)
    heat = torch.rand(B, P, K, 56, 56, generator=g)
    kpts = torch.rand(B, P, 1, K, 2, generator=g)
    cls = torch.randint(0, 3, (B, P, 1, K), generator=g)
    vis = torch.nn.functional.one_hot(cls, 3).float()
    ys = torch.arange(56.0).view(1, 1, 1, 56, 1)
    xs = torch.arange(56.0).view(1, 1, 1, 1, 56)
    c = torch.rand(B, P, K, 2, generator=g) * 56
    gt = torch.exp(-((ys - c[..., 1:2, None]) ** 2 + (xs - c[..., 0:1, None]) ** 2) / 8.0)
    gvis = (torch.rand(B, P, K, generator=g) < frac).long() * torch.randint(1, 3, (B, P, K), generator=g)
    batch = {"image": torch.zeros(B, 3, 8, 8), "keypoints": torch.rand(B, P, K, 2, generator=g),
             "visibilities": gvis, "heatmaps": gt if gt5 else gt.max(dim=1)[0]}
    return {"heatmap": heat, "keypoints": kpts, "visibilities": vis}, batch


def checksum(outputs, batch):
    s = sum(float(t.double().sum()) for t in outputs.values())
    return s + sum(float(batch[k].double().sum()) for k in ("keypoints", "visibilities", "heatmaps"))
