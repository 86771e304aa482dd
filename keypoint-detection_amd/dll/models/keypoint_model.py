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
from ..losses import KeypointLoss
from .backbone import MobileNetV3Wrapper
from .heatmap_head import HeatmapHead
from .keypoint_head import KEYPOINT_HEAD
from .person_head import PERSON_HEAD

HEATMAP_SIDE = 56


class ChannelAttention(nn.Module):
    """sigmoid(fc(avgpool) + fc(maxpool)), fc = Linear(C, C//16) ReLU Linear (reference :18-44).
    ``forward`` runs the native channel statistics + FC kernel (kpd_channel_attention)
    on the module's own plan (``channel_attention.`` prefix); built for C = 128."""

    def __init__(self, in_channels: int, reduction_ratio: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        red = max(1, in_channels // reduction_ratio)
        self.fc = nn.Sequential(nn.Linear(in_channels, red), nn.ReLU(), nn.Linear(red, in_channels))
        self._plans = _native.PlanCache("channel_attention.")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, C, H, W] -> attention scores [B, C] in (0, 1)."""
        return self.native_select(x, select=False)[0]

    def native_select(self, x: torch.Tensor, k: int = 64, select: bool = True):
        """(scores [B, C], top-k channel indices [B, k], x[b, topk[b]] [B, k, H, W] or None)."""
        return self._plans.get(self, x.device, "fp32").channel_attention(x, k, select)


def box_center_to_corners(box: torch.Tensor) -> torch.Tensor:
    """[cx, cy, w, h] (normalised) -> [x1, y1, x2, y2] clamped to [0, 1] (reference :630-638)."""
    cx, cy, w, h = box.unbind()
    return torch.stack([torch.clamp(cx - w / 2, 0, 1), torch.clamp(cy - h / 2, 0, 1),
                        torch.clamp(cx + w / 2, 0, 1), torch.clamp(cy + h / 2, 0, 1)])


def pad_to_length(tensor_list, length):
    """Truncate / zero-pad a list of tensors to ``length`` (reference :640-651)."""
    if len(tensor_list) == 0:
        return []
    if len(tensor_list) >= length:
        return tensor_list[:length]
    template = tensor_list[0]
    return tensor_list + [torch.zeros_like(template).detach() for _ in range(length - len(tensor_list))]


def select_top_k_channels(features: torch.Tensor, channel_attention: nn.Module, k: int = 64) -> torch.Tensor:
    """features[b, topk(channel_attention(features)[b], k)] -> [B, k, H, W]
    (reference :653-661): scores, sorted top-k (ties to the lower channel) and
    the gather in one native call."""
    if not isinstance(channel_attention, ChannelAttention):
        raise TypeError("select_top_k_channels runs the native ChannelAttention; pass the model's "
                        "channel_attention module")
    return channel_attention.native_select(features, k, select=True)[2]


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
      precision: "split" (default) -- fp32-accurate: FPN level 0 and the
                 heatmap-head convs as three f16 MFMA products of hi/lo
                 operand splits (fp32 tolerances: keypoints 1e-5, heatmaps
                 5e-5, identical top-k / visibility); everything else fp32;
                 "fp32" -- every conv on fp32-input MFMA (exact fp32 products);
                 "mixed" -- heatmap-head convs on bf16 MFMA with fp32
                 accumulation (keypoints within 1e-3); the backbone/FPN feeding
                 the order-critical channel top-k stays fp32-accurate.
      dual_head: also instantiate KEYPOINT_HEAD (not wired in the reference).

    Attribute ``full_level0`` (default False): with caller boxes the native
    path stores FPN level 0 only where the ROI aligns read it; True stores
    the whole map (for inspecting ``native_plan(dev).debug_buffer("feat0")``).
    Outputs are identical either way.
    """

    def __init__(self, config: ModelConfig, training_config: TrainingConfig, precision: str = "split",
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
        # no parameters: the state dict is unchanged (reference :65-69)
        self.loss_fn = KeypointLoss(num_keypoints=config.num_keypoints, config=training_config,
                                    device=torch.device("cuda"))
        self.dual_head = dual_head
        if dual_head:
            self.keypoint_head = KEYPOINT_HEAD(config.keypoint_head)
        self.max_persons = max_persons
        self.num_keypoints = config.num_keypoints
        self.precision = precision      # (property: also sets the submodules' own plans' precision)
        self.streams = streams          # sub-batch streams for B >= 32 (kpd_plan_set_streams)
        self.full_level0 = False        # store all of FPN level 0 (debug copy), not just the ROI footprints
        self._plan: Optional[_native.Plan] = None
        self._plan_key = None
        self._plan_streams: Optional[int] = None
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
        ph = self.config.person_head
        return (device, self.precision, ph.conf_threshold, ph.nms_iou_threshold, vers)

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
            self._plan, self._plan_key, self._plan_streams = plan, key, None
        if self._plan_streams != self.streams:   # a scheduling setting: no re-pack of the weights
            self._plan.set_streams(self.streams)
            self._plan_streams = self.streams
        return self._plan

    def invalidate_plan(self) -> None:
        self._plan, self._plan_key, self._state_tensors = None, None, None

    # ------------------------------------------------------------------ forward
    @property
    def precision(self) -> str:
        return self._precision

    @precision.setter
    def precision(self, value: str) -> None:
        if value not in _native.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_native.PRECISIONS)}")
        self._precision = value
        for m in (self.backbone, self.heatmap_head):
            m.precision = value

    def forward(self, batch) -> Dict[str, torch.Tensor]:
        """The eval forward (reference :73-210).  A dict batch that also
        carries 'keypoints' and 'visibilities' (the trainer's validation
        loop) gets the loss and its components added (:208-209, 509-584):
        the heatmap term on the device, the balancer's state advancing per
        call as in the reference."""
        out = self._forward(batch)
        if isinstance(batch, dict) and "keypoints" in batch and "visibilities" in batch:
            out = self._compute_loss_and_metrics(out, batch)
        return out

    def _compute_loss_and_metrics(self, outputs, batch):
        """Reference :509-584: the person axis is max-reduced for the heatmaps
        and visibilities (prediction and target), the keypoints keep it; the
        target heatmaps are batch['heatmaps'] or zeros of
        heatmap_head.heatmap_size."""
        K = self.num_keypoints
        hs = tuple(self.config.heatmap_head.heatmap_size)
        ph = outputs["heatmap"]
        if ph.dim() == 5:
            ph = ph.max(dim=1)[0]
        elif ph.dim() != 4:
            ph = ph.reshape(ph.size(0) if ph.dim() == 3 else batch["image"].size(0), K, *hs)
        if "heatmaps" in batch:
            gh = batch["heatmaps"]
            if gh.dim() == 5:
                gh = gh.max(dim=1)[0]
        else:
            gh = torch.zeros(batch["image"].size(0), K, *hs, device=batch["image"].device, dtype=torch.float32)
        if tuple(gh.shape) != tuple(ph.shape):
            raise RuntimeError(f"target heatmaps {tuple(gh.shape)} do not match the predicted {tuple(ph.shape)} "
                               "(the reference's mse_loss fails the same way)")
        pv = outputs["visibilities"]
        if pv.dim() == 5:
            pv = pv.squeeze(2)
        if pv.dim() == 4:
            pv = pv.max(dim=1)[0]
        elif pv.dim() == 3 and pv.size(-1) != 3:
            v3 = torch.zeros(pv.size(0), pv.size(2), 3, device=pv.device)
            v3[:, :, 2] = pv.max(dim=1)[0]
            pv = v3
        gv = batch["visibilities"]
        if gv.dim() == 3:
            gv = gv.max(dim=1)[0]
        pk = outputs["keypoints"]
        if pk.dim() == 5:
            pk = pk.squeeze(2)
        loss, parts = self.loss_fn(predictions={"heatmaps": ph, "visibilities": pv, "keypoints": pk},
                                   targets={"heatmaps": gh, "visibility": gv, "keypoints": batch["keypoints"]})
        outputs["loss"] = loss
        outputs.update(parts)
        return outputs

    def _forward(self, batch) -> Dict[str, torch.Tensor]:
        x = batch["image"] if isinstance(batch, dict) else batch
        if not isinstance(x, torch.Tensor):
            raise TypeError("Input must be a tensor or a dict with 'image' key containing a tensor")
        if self.training:
            raise NotImplementedError("training mode (batch-statistics BatchNorm, dropout, the loss) is outside "
                                      "the accelerated inference path; call model.eval()")
        if not x.is_cuda:
            raise _native.KpdNativeError("MultiPersonKeypointModel runs on the HIP device only; "
                                         "move the model input to 'cuda'")
        B = x.size(0)
        K = self.num_keypoints
        dev = x.device
        boxes = normalize_bboxes(batch, B, dev)
        plan = self.native_plan(dev)
        image = x.float().contiguous()
        flags = (_native.FLAG_DUAL_HEAD if self.dual_head else 0) | \
            (_native.FLAG_FULL_LEVEL0 if self.full_level0 else 0)
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

    # ------------------------------------------------------------------ helpers (reference :212-313)
    def extract_roi_features(self, features: torch.Tensor, box: torch.Tensor, output_size=(56, 56)) -> torch.Tensor:
        """roi_align of one cxcywh box on [1, C, H, W] features -> [1, C, oh, ow]
        (reference :212-228: corners clamped to [0, 1], scaled to the map,
        spatial_scale 1, sampling_ratio -1, aligned False)."""
        B, C, H, W = features.shape
        corners = box_center_to_corners(box.to(features.device, torch.float32))
        scale = torch.tensor([W, H, W, H], device=features.device, dtype=torch.float32)
        rois = torch.cat([torch.zeros(1, device=features.device), corners * scale]).unsqueeze(0)
        return _native.roi_align(features, rois, output_size)

    def convert_to_original_coords(self, keypoints: torch.Tensor, box) -> torch.Tensor:
        """ROI-normalised keypoints -> image-normalised, clamped to [0, 1] (reference :230-248)."""
        shape = keypoints.shape
        kp = keypoints.view(-1, 2) if keypoints.dim() == 3 else keypoints
        cx, cy, w, h = box
        x = torch.clamp(kp[:, 0] * w + (cx - w / 2), 0, 1)
        y = torch.clamp(kp[:, 1] * h + (cy - h / 2), 0, 1)
        return torch.stack([x, y], dim=-1).view(shape)

    def decode_heatmap(self, heatmap: torch.Tensor, threshold: float = 0.1):
        """Soft-argmax keypoints [B, K, 2] and one-hot 3-class visibility
        [B, K, 3] from sigmoid(max) < 0.3 / < 0.7 / else (reference :250-282);
        one device kernel (kpd_decode_heatmaps)."""
        kp, _, vis = _native.decode_heatmaps(heatmap, _native.DECODE_MODEL)
        return kp, vis

    def _soft_argmax(self, heatmap: torch.Tensor) -> torch.Tensor:
        """E[x] / (W - 1), E[y] / (H - 1) under softmax over each map (reference :284-313)."""
        return _native.decode_heatmaps(heatmap, _native.DECODE_SOFTARGMAX, 1.0)[0]
