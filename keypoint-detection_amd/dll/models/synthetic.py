"""Deterministic synthetic weights for a MultiPersonKeypointModel state dict.

There are no trained weights (the reference's outputs/best_model.pth is a
missing blob and the torchvision ImageNet weights are a network download), so
benchmarks and parity fixtures use weights drawn from a seeded CPU generator,
visiting the state dict in key order.  BN running statistics are made
non-trivial so that BN folding is exercised.  Rules, by parameter role:
  conv weight   N(0, sqrt(2 / fan_out))          (torchvision / reference init)
  conv bias     N(0, 0.05)
  linear weight U(-1/sqrt(fan_in), 1/sqrt(fan_in))  (nn.Linear default)
  linear bias   U(-1/sqrt(fan_in), 1/sqrt(fan_in))
  norm weight   U(0.5, 1.5); norm bias N(0, 0.1)
  running_mean  N(0, 0.1);   running_var U(0.5, 1.5)
  anchors / num_batches_tracked: left as constructed
``head_gain`` scales the last heatmap 1x1 conv so heatmaps are not flat.
"""
from __future__ import annotations

import math
from typing import Dict

import torch


def synthetic_state_dict(sd: Dict[str, torch.Tensor], seed: int = 0, head_gain: float = 4.0) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    out: Dict[str, torch.Tensor] = {}
    keys = list(sd.keys())
    for k in keys:
        t = sd[k]
        if not t.is_floating_point() or k.endswith("anchors"):
            out[k] = t.detach().clone().cpu()
            continue
        shape = tuple(t.shape)
        base = k.rsplit(".", 1)[0]
        leaf = k.rsplit(".", 1)[1]
        is_norm = (base + ".running_mean") in sd or (len(shape) == 1 and leaf == "weight" and
                                                     (base + ".bias") in sd and (base + ".weight") in sd and
                                                     sd[base + ".weight"].dim() == 1)
        if leaf == "running_mean":
            v = torch.randn(shape, generator=g) * 0.1
        elif leaf == "running_var":
            v = torch.rand(shape, generator=g) + 0.5
        elif is_norm and leaf == "weight":
            v = torch.rand(shape, generator=g) + 0.5
        elif is_norm and leaf == "bias":
            v = torch.randn(shape, generator=g) * 0.1
        elif leaf == "weight" and len(shape) == 4:
            fan_out = shape[0] * shape[2] * shape[3]
            v = torch.randn(shape, generator=g) * math.sqrt(2.0 / fan_out)
        elif leaf == "weight" and len(shape) == 2:
            b = 1.0 / math.sqrt(shape[1])
            v = (torch.rand(shape, generator=g) * 2 - 1) * b
        elif leaf == "bias":
            w = sd.get(base + ".weight")
            if w is not None and w.dim() == 2:
                b = 1.0 / math.sqrt(w.shape[1])
                v = (torch.rand(shape, generator=g) * 2 - 1) * b
            else:
                v = torch.randn(shape, generator=g) * 0.05
        else:
            v = torch.randn(shape, generator=g) * 0.05
        if k.startswith("heatmap_head.final_layer.3."):
            v = v * head_gain
        out[k] = v.to(torch.float32)
    return out


def weights_checksum(sd: Dict[str, torch.Tensor]) -> float:
    """Order-independent fingerprint used by the golden fixtures."""
    s = 0.0
    for i, k in enumerate(sorted(sd)):
        t = sd[k]
        if t.is_floating_point():
            s += float(t.double().abs().sum()) * (1.0 + 1e-3 * i)
    return s


_MEAN = (0.485, 0.456, 0.406)
_STD = (0.229, 0.224, 0.225)


def synthetic_images(batch: int, channels: int = 3, height: int = 256, width: int = 192, seed: int = 1234,
                     device=None) -> torch.Tensor:
    """U[0,1) images (seed 1234) then ImageNet Normalize (1-channel: mean .5 std .5,
    as ITransform's grayscale pipeline), fp32 NCHW (BASELINE.md protocol)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(batch, channels, height, width, generator=g)
    if channels == 3:
        m = torch.tensor(_MEAN).view(1, 3, 1, 1)
        s = torch.tensor(_STD).view(1, 3, 1, 1)
    else:
        m = torch.full((1, channels, 1, 1), 0.5)
        s = torch.full((1, channels, 1, 1), 0.5)
    x = (x - m) / s
    return x if device is None else x.to(device)


def synthetic_boxes(batch: int, persons: int = 1, seed: int = 1235, device=None) -> torch.Tensor:
    """[B,P,4] cxcywh: cx,cy ~ U(0.3,0.7), w ~ U(0.15,0.5), h ~ U(0.3,0.9) (seed 1235)."""
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(batch, persons, 4, generator=g)
    b = torch.empty_like(u)
    b[..., 0] = 0.3 + 0.4 * u[..., 0]
    b[..., 1] = 0.3 + 0.4 * u[..., 1]
    b[..., 2] = 0.15 + 0.35 * u[..., 2]
    b[..., 3] = 0.3 + 0.6 * u[..., 3]
    return b if device is None else b.to(device)
