"""PERSON_HEAD (reference: dll/models/person_head.py:7-166).

Parameters and the ``anchors`` buffer keep the reference names
(``box_heads.{0-3}``, ``cls_heads.{0-3}``, ``anchors`` [56*56*9, 4]).
``box_iou`` and ``non_max_suppression`` keep the reference signatures;
``non_max_suppression`` runs the native greedy NMS (csrc/nms.hip) for device
tensors.
"""
import torch
import torch.nn as nn

from .. import _native
from ..configs.model_config import PersonDetectionConfig


class PERSON_HEAD(nn.Module):
    def __init__(self, config: PersonDetectionConfig):
        super().__init__()
        c = config.in_channels
        self.num_classes = config.num_classes
        self.conf_threshold = config.conf_threshold
        self.nms_iou_threshold = config.nms_iou_threshold
        self.anchor_sizes = list(config.anchor_sizes)
        self.grid_size = (56, 56)
        self.aspect_ratios = [0.5, 1.0, 2.0]
        na = len(self.anchor_sizes) * len(self.aspect_ratios)
        self.box_heads = nn.ModuleList([nn.Conv2d(c, 4 * na, 1) for _ in range(4)])
        self.cls_heads = nn.ModuleList([nn.Conv2d(c, self.num_classes * na, 1) for _ in range(4)])
        self.register_buffer("anchors", self._generate_anchors())

    def _generate_anchors(self) -> torch.Tensor:
        """(cx, cy, size*ar, size/ar) per grid cell, sizes in pixels (reference quirk, :39-52)."""
        h, w = self.grid_size
        j = (torch.arange(w, dtype=torch.float64) + 0.5) / w
        i = (torch.arange(h, dtype=torch.float64) + 0.5) / h
        cy, cx = torch.meshgrid(i, j, indexing="ij")
        wh = torch.tensor([[s * r, s / r] for s in self.anchor_sizes for r in self.aspect_ratios],
                          dtype=torch.float64)
        na = wh.shape[0]
        a = torch.empty(h, w, na, 4, dtype=torch.float64)
        a[..., 0] = cx[..., None]
        a[..., 1] = cy[..., None]
        a[..., 2] = wh[:, 0]
        a[..., 3] = wh[:, 1]
        return a.reshape(-1, 4).to(torch.float32)

    @staticmethod
    def box_iou(boxes1: torch.Tensor, boxes2: torch.Tensor) -> torch.Tensor:
        """IoU of cxcywh boxes, (N,4) x (M,4) -> (N,M) (reference :54-94)."""
        def corners(b):
            return b[:, 0] - b[:, 2] / 2, b[:, 1] - b[:, 3] / 2, b[:, 0] + b[:, 2] / 2, b[:, 1] + b[:, 3] / 2
        ax1, ay1, ax2, ay2 = corners(boxes1)
        bx1, by1, bx2, by2 = corners(boxes2)
        iw = torch.clamp(torch.min(ax2[:, None], bx2) - torch.max(ax1[:, None], bx1), min=0)
        ih = torch.clamp(torch.min(ay2[:, None], by2) - torch.max(ay1[:, None], by1), min=0)
        inter = iw * ih
        return inter / ((ax2 - ax1) * (ay2 - ay1))[:, None].add((bx2 - bx1) * (by2 - by1)).sub(inter).add(1e-16)

    def non_max_suppression(self, boxes, scores, iou_threshold=0.2, max_output_size=None):
        """Greedy NMS (reference :96-139) on the device; returns a CPU int64 index
        tensor like the reference."""
        return _native.nms(boxes, scores, iou_threshold, max_output_size or 0).cpu()

    def forward(self, features, targets=None):
        """Reference :141-166: with training targets the last FPN level and the
        target boxes pass through; otherwise every level's box head runs and the
        last level's prediction [B, 36, h, w] is returned (the reference keeps
        only that one, so only that one is computed here; kpd_conv1x1)."""
        if self.training and targets is not None and "bboxes" in targets:
            return features[-1], targets["bboxes"]
        # zip(features, box_heads): at most 4 levels; a plain tensor iterates its
        # batch dim (unbatched [C, h, w] maps), as in the reference
        feats = list(features)[: len(self.box_heads)]
        head, x = self.box_heads[len(feats) - 1], feats[-1]
        if x.dim() == 3:
            return _native.conv1x1(x.unsqueeze(0), head.weight, head.bias).squeeze(0)
        return _native.conv1x1(x, head.weight, head.bias)
