"""MultiPersonKeypointModel -- drop-in for the reference's eval forward.

Reference: dll/models/keypoint_model.py:49-210.  Same constructor
(``MultiPersonKeypointModel(ModelConfig, TrainingConfig)``), same submodule /
state-dict names, same ``forward(batch)`` contract and output dict:

    {'heatmap': [B,P,17,56,56], 'keypoints': [B,P,1,17,2],
     'visibilities': [B,P,1,17,3], 'boxes': <per-image box list>}

including the reference's quirks: all-zero boxes are skipped and the
remaining persons compacted, images without a valid box get a dummy person
(visibility class 0), P stays the padded person count, and a batch where
every image has zero boxes returns zeros with a 2-D ``visibilities`` [B,1,17]
(:123-135).

Everything numeric runs in libkpd.so (csrc/) on the input's HIP device; the
Python layer only normalises arguments, allocates outputs and calls the C
ABI.  There is no CPU fallback: CPU inputs or a missing library raise.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .. import _native
from ..configs.model_config import ModelConfig
from ..configs.training_config import TrainingConfig
from .backbone import MobileNetV3Wrapper
from .heatmap_head import HeatmapHead
from .keypoint_head import KEYPOINT_HEAD
from .person_head import PERSON_HEAD

HEATMAP_SIDE = 56


class ChannelAttention(nn.Module):
    """sigmoid(fc(avgpool) + fc(maxpool)), fc = Linear(C, C//16) ReLU Linear (reference :18-44)."""

    def __init__(self, in_channels: int, reduction_ratio: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        red = max(1, in_channels // reduction_ratio)
        self.fc = nn.Sequential(nn.Linear(in_channels, red), nn.ReLU(), nn.Linear(red, in_channels))


def normalize_bboxes(batch, batch_size: int, device) -> Optional[List[torch.Tensor]]:
    """Reference :93-113.  Returns the per-image box list, or None when the
    person-detector branch would be taken."""
    if not (isinstance(batch, dict) and "bboxes" in batch):
        return None
    bb = batch["bboxes"]
    if isinstance(bb, list) and len(bb) > 0:
        t = bb[0]
        if t.dim() == 3:
            return [t[i] for i in range(t.size(0))]
        if t.dim() == 2:
            return [t]
        raise ValueError(f"Invalid bboxes tensor format: {t.shape}")
    if isinstance(bb, torch.Tensor):
        if bb.dim() == 3 and bb.size(-1) == 4:
            return [bb[i] for i in range(bb.size(0))]
        raise ValueError(f"Invalid bboxes format: {bb.shape}")
    return [torch.zeros(0, 4, device=device) for _ in range(batch_size)]


class MultiPersonKeypointModel(nn.Module):
    """Multi-person keypoint detection model (native MI355X inference path).

    Extra keyword arguments (not in the reference):
      precision: "fp32" -- every conv on fp32-input MFMA (exact fp32 products);
                 "mixed" -- heatmap-head convs on bf16 MFMA with fp32
                 accumulation; the backbone/FPN feeding the order-critical
                 channel top-k stays fp32.
      dual_head: also instantiate KEYPOINT_HEAD (not wired in the reference).
    """

    def __init__(self, config: ModelConfig, training_config: TrainingConfig, precision: str = "fp32",
                 dual_head: bool = False, max_persons: int = 5, streams: int = 1):
        super().__init__()
        if precision not in _native.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_native.PRECISIONS)}")
        self.config = config
        self.training_config = training_config
        self.backbone = MobileNetV3Wrapper(config.backbone)
        self.person_detector = PERSON_HEAD(config.person_head)
        self.heatmap_head = HeatmapHead(config.heatmap_head)
        self.channel_attention = ChannelAttention(config.backbone.out_channels, reduction_ratio=16)
        self.dual_head = dual_head
        if dual_head:
            self.keypoint_head = KEYPOINT_HEAD(config.keypoint_head)
        self.max_persons = max_persons
        self.num_keypoints = config.num_keypoints
        self.precision = precision
        self.streams = streams          # sub-batch streams for B >= 32 (kpd_plan_set_streams)
        self._plan: Optional[_native.Plan] = None
        self._plan_key = None
        self._state_tensors: Optional[List[torch.Tensor]] = None
        if config.num_keypoints != 17 or config.heatmap_head.in_channels != 64 \
                or config.backbone.out_channels != 128:
            raise ValueError("the native path is built for 17 keypoints, 64 selected channels, 128 FPN channels")

    # ------------------------------------------------------------------ plan
    def _weights_key(self, device: torch.device) -> Tuple:
        # The state tensors are listed once (a module walk costs ~0.7 ms per
        # forward); storage or in-place changes show in (data_ptr, _version).
        # Replacing a Parameter object goes through load_state_dict / _apply
        # (both reset the list) or needs invalidate_plan().
        if self._state_tensors is None:
            self._state_tensors = list(self.state_dict(keep_vars=True).values())
        vers = tuple((t.data_ptr(), t._version) for t in self._state_tensors)
        return (device, self.precision, self.streams, vers)

    def _apply(self, fn, *args, **kwargs):
        self._state_tensors = None
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        self._state_tensors = None
        return super().load_state_dict(*args, **kwargs)

    def native_plan(self, device: torch.device) -> _native.Plan:
        """Build (or reuse) the packed-weight plan for ``device``."""
        key = self._weights_key(device)
        if self._plan is None or self._plan_key != key:
            plan = _native.Plan(device, self.config.backbone.in_channels)
            for name, t in self.state_dict().items():
                if t.is_floating_point():
                    plan.set_tensor(name, t)
            plan.finalize(_native.PRECISIONS[self.precision])
            ph = self.config.person_head
            plan.set_detector(ph.conf_threshold, ph.nms_iou_threshold)
            plan.set_streams(self.streams)
            self._plan, self._plan_key = plan, key
        return self._plan

    def invalidate_plan(self) -> None:
        self._plan, self._plan_key, self._state_tensors = None, None, None

    # ------------------------------------------------------------------ forward
    def forward(self, batch) -> Dict[str, torch.Tensor]:
        x = batch["image"] if isinstance(batch, dict) else batch
        if not isinstance(x, torch.Tensor):
            raise TypeError("Input must be a tensor or a dict with 'image' key containing a tensor")
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training forward/loss is outside the accelerated path; "
                                      "call model.eval() (inference only)")
        if not x.is_cuda:
            raise _native.KpdNativeError("MultiPersonKeypointModel runs on the HIP device only; "
                                         "move the model input to 'cuda'")
        B = x.size(0)
        K = self.num_keypoints
        dev = x.device
        boxes = normalize_bboxes(batch, B, dev)
        plan = self.native_plan(dev)
        image = x.float().contiguous()
        flags = _native.FLAG_DUAL_HEAD if self.dual_head else 0
        if boxes is None:
            # person-detector branch (reference :114-119 is broken; build-defined
            # glue: FPN0 -> 56x56 pool -> box/cls heads -> decode -> NMS,
            # DESIGN.md §C3).  Detected boxes are zero padded to max_persons.
            P = self.max_persons
            bt = torch.zeros(B, P, 4, device=dev)
            scores = torch.zeros(B, P, device=dev)
            out = self._run(plan, image, bt, B, P, flags | _native.FLAG_DETECT, scores)
            out["boxes"] = [bt[i] for i in range(B)]
            out["box_scores"] = scores
            return out
        if not boxes or all(len(b) == 0 for b in boxes):
            return {"keypoints": torch.zeros(B, 1, K, 2, device=dev),
                    "visibilities": torch.zeros(B, 1, K, device=dev),
                    "heatmap": torch.zeros(B, 1, K, HEATMAP_SIDE, HEATMAP_SIDE, device=dev),
                    "boxes": boxes}
        nb = len(boxes)
        if nb > B:
            raise ValueError(f"bboxes describe {nb} images but the batch has {B}")
        P = max(len(b) for b in boxes)
        # boxes given as one [B,P,4] float32 device tensor: read in place (the
        # per-image list above is views of it), no stack copy
        bb = batch["bboxes"]
        t3 = bb if isinstance(bb, torch.Tensor) else bb[0]
        if (t3.dim() == 3 and t3.dtype == torch.float32 and t3.device == dev and t3.is_contiguous()
                and t3.size(0) == nb and t3.size(1) == P):
            bt = t3
        else:
            bt = torch.stack([b.to(dev, torch.float32) for b in boxes]).contiguous()   # [nb,P,4]
        if bt.dim() != 3 or bt.size(-1) != 4:
            raise ValueError(f"Invalid bboxes format: {tuple(bt.shape)}")
        out = self._run(plan, image, bt, nb, P, flags)
        out["boxes"] = boxes
        return out

    def _run(self, plan, image, bt, nb, P, flags, box_scores=None) -> Dict[str, torch.Tensor]:
        dev, K = image.device, self.num_keypoints
        kpts = torch.empty(nb, P, 1, K, 2, device=dev)
        vis = torch.empty(nb, P, 1, K, 3, device=dev)
        heat = torch.empty(nb, P, K, HEATMAP_SIDE, HEATMAP_SIDE, device=dev)
        kh_k = kh_v = None
        if flags & _native.FLAG_DUAL_HEAD:
            kh_k = torch.empty(nb, P, 1, K, 2, device=dev)
            kh_v = torch.empty(nb, P, 1, K, 3, device=dev)
        plan.forward(image, bt, kpts, vis, heat, flags, kh_k, kh_v, box_scores)
        out = {"heatmap": heat, "keypoints": kpts, "visibilities": vis}
        if kh_k is not None:
            out["kh_keypoints"], out["kh_visibilities"] = kh_k, kh_v
        return out
