"""Validation metrics on the device: ADE and PCK exactly as the reference's
``Trainer._calculate_validation_metrics`` (dll/training/trainer.py:384-429)
defines them, computed by ``kpd_keypoint_metrics`` (csrc/data_kernels.hip).

* predicted [B,P,1,K,2] is squeezed to [B,P,K,2]; against a [B,K,2] ground
  truth the first person is taken; any other shape mismatch returns the
  default (all-zero) metrics, as does any error;
* ADE = mean L2 distance over keypoints with visibility > 0;
* PCK@t = #(distance <= t and visible) / #keypoints (all of them -- the
  reference's denominator), 0 when nothing is visible.

Accumulation is in double on the device, so the values agree with the
reference's fp32 reductions to ~1e-7 relative.
"""
from __future__ import annotations

import ctypes
import logging
from typing import Dict, Sequence

import torch

from .. import _native
from ..configs.training_config import TrainingConfig

DEFAULT_PCK_THRESHOLDS = tuple(TrainingConfig().pck_thresholds)


def get_default_metrics(pck_thresholds: Sequence[float] = DEFAULT_PCK_THRESHOLDS) -> Dict[str, float]:
    """Reference ``_get_default_metrics`` (trainer.py:431-436)."""
    out = {"avg_ADE": 0.0}
    out.update({f"pck_{t}": 0.0 for t in pck_thresholds})
    return out


def _metrics_on_device(pred: torch.Tensor, gt: torch.Tensor, vis: torch.Tensor, thresholds: Sequence[float]):
    _native._require_cuda(pred, "pred keypoints")
    dev = pred.device
    p = pred.float().contiguous()
    g = gt.to(dev).float().contiguous()
    v = vis.to(dev).float().contiguous()
    if v.numel() != p.numel() // 2:
        raise ValueError(f"visibilities {tuple(vis.shape)} do not match keypoints {tuple(pred.shape)}")
    out = torch.empty(1 + len(thresholds), device=dev, dtype=torch.float32)
    thr = (ctypes.c_float * max(len(thresholds), 1))(*thresholds)
    lib = _native.load()
    with torch.cuda.device(dev):
        rc = lib.kpd_keypoint_metrics(_native._ptr(p), _native._ptr(g), _native._ptr(v), p.numel() // 2, thr,
                                      len(thresholds), _native._ptr(out), _native._stream(dev))
    _native.check(rc, "kpd_keypoint_metrics")
    return out.tolist()


def calculate_validation_metrics(outputs: Dict[str, torch.Tensor], batch: Dict[str, torch.Tensor],
                                 pck_thresholds: Sequence[float] = DEFAULT_PCK_THRESHOLDS) -> Dict[str, float]:
    try:
        pred, gt, vis = outputs["keypoints"], batch["keypoints"], batch["visibilities"]
        if pred.dim() == 5:
            pred = pred.squeeze(2)
        if pred.dim() == 4 and gt.dim() == 3:
            pred = pred[:, 0, :, :]
        if pred.shape != gt.shape:
            return get_default_metrics(pck_thresholds)
        vals = _metrics_on_device(pred, gt, vis, list(pck_thresholds))
        out = {"avg_ADE": vals[0]}
        out.update({f"pck_{t}": vals[1 + i] for i, t in enumerate(pck_thresholds)})
        return out
    except _native.KpdNativeError:
        raise                                   # no silent CPU fallback for a missing library / device
    except Exception as e:   # noqa: BLE001 -- reference behaviour: log and return defaults
        logging.warning(f"Error calculating validation metrics: {e}")
        return get_default_metrics(pck_thresholds)
