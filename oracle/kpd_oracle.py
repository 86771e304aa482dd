"""Plain-PyTorch CPU restatement of ``MultiPersonKeypointModel.forward`` (eval).

TEST INFRASTRUCTURE ONLY -- see ``oracle/__init__.py``.  Everything here is a
functional restatement written against a *state dict* that uses the
reference's own parameter names, so the same weights feed the reference
(for goldens), this oracle, and the HIP product path.

Reference anchors (all paths under /root/reference):
  * forward orchestration ........ dll/models/keypoint_model.py:73-210
  * ChannelAttention (model) ..... dll/models/keypoint_model.py:18-44
  * select_top_k_channels ........ dll/models/keypoint_model.py:653-661
  * extract_roi_features ......... dll/models/keypoint_model.py:212-228
  * box_center_to_corners ........ dll/models/keypoint_model.py:630-638
  * convert_to_original_coords ... dll/models/keypoint_model.py:230-248
  * decode_heatmap / _soft_argmax  dll/models/keypoint_model.py:250-313
  * pad_to_length ................ dll/models/keypoint_model.py:640-651
  * MobileNetV3Wrapper / FPN ..... dll/models/backbone.py:7-39, 247-264
  * HeatmapHead (+attention) ..... dll/models/heatmap_head.py:20-151
  * PERSON_HEAD box_iou / NMS .... dll/models/person_head.py:39-139
  * KEYPOINT_HEAD ................ dll/models/keypoint_head.py:9-90
Third-party (torchvision, unpinned version per setup.py:13) restated from the
published algorithm: mobilenet_v3_small features topology and roi_align
(aligned=False, sampling_ratio=-1).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]

NUM_KEYPOINTS = 17
HEATMAP_SIZE = 56
TOPK_CHANNELS = 64

# torchvision mobilenet_v3_small inverted-residual table
# (in, kernel, expanded, out, use_se, activation, stride)
MBV3_SMALL_BNECK: Tuple[Tuple[int, int, int, int, bool, str, int], ...] = (
    (16, 3, 16, 16, True, "RE", 2),
    (16, 3, 72, 24, False, "RE", 2),
    (24, 3, 88, 24, False, "RE", 1),
    (24, 5, 96, 40, True, "HS", 2),
    (40, 5, 240, 40, True, "HS", 1),
    (40, 5, 240, 40, True, "HS", 1),
    (40, 5, 120, 48, True, "HS", 1),
    (48, 5, 144, 48, True, "HS", 1),
    (48, 5, 288, 96, True, "HS", 2),
    (96, 5, 576, 96, True, "HS", 1),
    (96, 5, 576, 96, True, "HS", 1),
)
MBV3_TAPS = (0, 3, 8, 12)          # backbone.py:253 return_nodes
FPN_IN_CHANNELS = (16, 24, 48, 576)  # backbone.py:255
BN_EPS_BODY = 1e-3                 # torchvision mobilenet_v3 norm_layer eps
BN_EPS = 1e-5                      # nn.BatchNorm2d default (FPN / heads)


def make_divisible(v: float, divisor: int = 8) -> int:
    """torchvision ``_make_divisible`` (SE squeeze width)."""
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


# --------------------------------------------------------------------------
# small helpers
# --------------------------------------------------------------------------
def _bn(x: Tensor, sd: SD, p: str, eps: float) -> Tensor:
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], False, 0.0, eps)


def _act(x: Tensor, act: Optional[str]) -> Tensor:
    if act == "RE":
        return F.relu(x)
    if act == "HS":
        return F.hardswish(x)
    return x


# --------------------------------------------------------------------------
# backbone: MobileNetV3-Small body (torchvision restatement) + LightweightFPN
# --------------------------------------------------------------------------
def mbv3_small_taps(x: Tensor, sd: SD, prefix: str = "backbone.body.") -> List[Tensor]:
    """features.0..12 of mobilenet_v3_small; returns taps 0, 3, 8, 12."""
    taps = []
    f = prefix + "features."
    # features.0: conv3x3 s2 + BN + hardswish
    x = F.conv2d(x, sd[f + "0.0.weight"], None, 2, 1)
    x = F.hardswish(_bn(x, sd, f + "0.1", BN_EPS_BODY))
    taps.append(x)
    for i, (cin, k, exp, cout, se, act, s) in enumerate(MBV3_SMALL_BNECK, start=1):
        p = f"{f}{i}.block."
        inp = x
        j = 0
        if exp != cin:
            x = F.conv2d(x, sd[f"{p}{j}.0.weight"])
            x = _act(_bn(x, sd, f"{p}{j}.1", BN_EPS_BODY), act)
            j += 1
        x = F.conv2d(x, sd[f"{p}{j}.0.weight"], None, s, (k - 1) // 2, 1, exp)
        x = _act(_bn(x, sd, f"{p}{j}.1", BN_EPS_BODY), act)
        j += 1
        if se:
            sc = F.adaptive_avg_pool2d(x, 1)
            sc = F.relu(F.conv2d(sc, sd[f"{p}{j}.fc1.weight"], sd[f"{p}{j}.fc1.bias"]))
            sc = F.hardsigmoid(F.conv2d(sc, sd[f"{p}{j}.fc2.weight"], sd[f"{p}{j}.fc2.bias"]))
            x = sc * x
            j += 1
        x = F.conv2d(x, sd[f"{p}{j}.0.weight"])
        x = _bn(x, sd, f"{p}{j}.1", BN_EPS_BODY)
        if s == 1 and cin == cout:
            x = x + inp
        if i in MBV3_TAPS:
            taps.append(x)
    x = F.conv2d(x, sd[f + "12.0.weight"])
    x = F.hardswish(_bn(x, sd, f + "12.1", BN_EPS_BODY))
    taps.append(x)
    return taps


def fpn_laterals(taps: Sequence[Tensor], sd: SD, prefix: str = "backbone.fpn.") -> List[Tensor]:
    """backbone.py:33-37 -- 1x1 laterals then nearest top-down add."""
    lat = [F.conv2d(t, sd[f"{prefix}lateral_convs.{i}.weight"]) for i, t in enumerate(taps)]
    for i in range(len(lat) - 1, 0, -1):
        up = F.interpolate(lat[i], size=lat[i - 1].shape[2:], mode="nearest")
        lat[i - 1] = lat[i - 1] + up
    return lat


def fpn_level(lat: Tensor, sd: SD, level: int, prefix: str = "backbone.fpn.") -> Tensor:
    """backbone.py:20-27,39 -- 3x3 conv (no bias) + BN + ReLU."""
    p = f"{prefix}fpn_convs.{level}."
    y = F.conv2d(lat, sd[p + "0.weight"], None, 1, 1)
    return F.relu(_bn(y, sd, p + "1", BN_EPS))


def backbone_level0(x: Tensor, sd: SD) -> Tensor:
    """Only FPN level 0 is consumed by forward (keypoint_model.py:86-90)."""
    return fpn_level(fpn_laterals(mbv3_small_taps(x, sd), sd)[0], sd, 0)


# --------------------------------------------------------------------------
# channel attention + top-k (keypoint_model.py:18-44, 653-661)
# --------------------------------------------------------------------------
def _fc2(v: Tensor, sd: SD, p: str) -> Tensor:
    h = F.relu(F.linear(v, sd[p + "fc.0.weight"], sd[p + "fc.0.bias"]))
    return F.linear(h, sd[p + "fc.2.weight"], sd[p + "fc.2.bias"])


def channel_scores(feat: Tensor, sd: SD, p: str = "channel_attention.") -> Tensor:
    avg = feat.mean(dim=(2, 3))
    mx = feat.amax(dim=(2, 3))
    return torch.sigmoid(_fc2(avg, sd, p) + _fc2(mx, sd, p))


def select_top_k(feat: Tensor, sd: SD, k: int = TOPK_CHANNELS) -> Tuple[Tensor, Tensor]:
    scores = channel_scores(feat, sd)
    _, idx = torch.topk(scores, min(k, feat.shape[1]), dim=1)
    b = torch.arange(feat.shape[0])[:, None].expand(-1, idx.shape[1])
    return feat[b, idx], idx


# --------------------------------------------------------------------------
# ROI align (torchvision.ops.roi_align, aligned=False, sampling_ratio=-1)
# --------------------------------------------------------------------------
def box_center_to_corners(box: Tensor) -> Tensor:
    cx, cy, w, h = box.unbind()
    return torch.stack([torch.clamp(cx - w / 2, 0, 1), torch.clamp(cy - h / 2, 0, 1),
                        torch.clamp(cx + w / 2, 0, 1), torch.clamp(cy + h / 2, 0, 1)])


def _bilinear_axis(coord: Tensor, size: int):
    """Per-axis part of torchvision's bilinear_interpolate (CPU pre_calc)."""
    valid = (coord >= -1.0) & (coord <= size)
    c = torch.clamp(coord, min=0.0)
    lo = c.floor().to(torch.int64)
    at_edge = lo >= size - 1
    lo = torch.where(at_edge, torch.full_like(lo, size - 1), lo)
    hi = torch.where(at_edge, lo, lo + 1)
    c = torch.where(at_edge, lo.to(c.dtype), c)
    l = c - lo.to(c.dtype)
    return valid, lo, hi, 1.0 - l, l


def roi_align_one(feat: Tensor, x1: Tensor, y1: Tensor, x2: Tensor, y2: Tensor,
                  out: int = HEATMAP_SIZE) -> Tensor:
    """feat [C,H,W]; box in feature-pixel coords -> [C,out,out].  Vectorized,
    separable in y/x; same sample points and weights as torchvision."""
    C, H, W = feat.shape
    roi_w = torch.clamp(x2 - x1, min=1.0)
    roi_h = torch.clamp(y2 - y1, min=1.0)
    bin_w = roi_w / out
    bin_h = roi_h / out
    gw = int(math.ceil(float(roi_w) / out))
    gh = int(math.ceil(float(roi_h) / out))
    count = max(gw * gh, 1)
    ph = torch.arange(out, dtype=torch.float32)
    iy = torch.arange(gh, dtype=torch.float32)
    ix = torch.arange(gw, dtype=torch.float32)
    ys = y1 + ph[:, None] * bin_h + (iy[None, :] + 0.5) * bin_h / gh      # [out, gh]
    xs = x1 + ph[:, None] * bin_w + (ix[None, :] + 0.5) * bin_w / gw      # [out, gw]
    vy, ylo, yhi, hy, ly = _bilinear_axis(ys.reshape(-1), H)
    vx, xlo, xhi, hx, lx = _bilinear_axis(xs.reshape(-1), W)
    vy = vy.float(); vx = vx.float()
    # gather rows then columns: [C, Ny, W] then [C, Ny, Nx]
    r_lo = feat[:, ylo, :]
    r_hi = feat[:, yhi, :]
    v11 = r_lo[:, :, xlo]; v12 = r_lo[:, :, xhi]
    v21 = r_hi[:, :, xlo]; v22 = r_hi[:, :, xhi]
    w1 = (hy[:, None] * hx[None, :]); w2 = (hy[:, None] * lx[None, :])
    w3 = (ly[:, None] * hx[None, :]); w4 = (ly[:, None] * lx[None, :])
    val = w1 * v11 + w2 * v12 + w3 * v21 + w4 * v22
    val = val * (vy[:, None] * vx[None, :])
    val = val.view(C, out, gh, out, gw).sum(dim=(2, 4))
    return val / count


def roi_align_loop(feat: Tensor, x1: float, y1: float, x2: float, y2: float,
                   out: int = HEATMAP_SIZE) -> Tensor:
    """Slow scalar-loop restatement of torchvision roi_align_forward_kernel_impl
    (CPU), vectorized only over channels.  Used by tests to pin the vectorized
    version and by the golden shim."""
    f32 = lambda v: torch.tensor(v, dtype=torch.float32)
    C, H, W = feat.shape
    x1, y1, x2, y2 = f32(x1), f32(y1), f32(x2), f32(y2)
    roi_w = torch.clamp(x2 - x1, min=1.0); roi_h = torch.clamp(y2 - y1, min=1.0)
    bin_w = roi_w / out; bin_h = roi_h / out
    gw = int(math.ceil(float(roi_w) / out)); gh = int(math.ceil(float(roi_h) / out))
    count = max(gw * gh, 1)
    res = torch.zeros(C, out, out)
    for ph in range(out):
        for pw in range(out):
            acc = torch.zeros(C)
            for iy in range(gh):
                y = y1 + ph * bin_h + f32(iy + 0.5) * bin_h / gh
                for ix in range(gw):
                    x = x1 + pw * bin_w + f32(ix + 0.5) * bin_w / gw
                    if y < -1.0 or y > H or x < -1.0 or x > W:
                        continue
                    yy = torch.clamp(y, min=0.0); xx = torch.clamp(x, min=0.0)
                    yl = int(yy); xl = int(xx)
                    if yl >= H - 1:
                        yh = yl = H - 1; yy = f32(yl)
                    else:
                        yh = yl + 1
                    if xl >= W - 1:
                        xh = xl = W - 1; xx = f32(xl)
                    else:
                        xh = xl + 1
                    ly = yy - yl; lx = xx - xl; hy = 1.0 - ly; hx = 1.0 - lx
                    acc = acc + (hy * hx) * feat[:, yl, xl] + (hy * lx) * feat[:, yl, xh] \
                        + (ly * hx) * feat[:, yh, xl] + (ly * lx) * feat[:, yh, xh]
            res[:, ph, pw] = acc / count
    return res


def extract_roi_features(feat1: Tensor, box: Tensor) -> Tensor:
    """keypoint_model.py:212-228 -- feat1 [1,C,H,W], box cxcywh -> [1,C,56,56]."""
    _, C, H, W = feat1.shape
    c = box_center_to_corners(box) * torch.tensor([W, H, W, H], dtype=torch.float32)
    return roi_align_one(feat1[0], c[0], c[1], c[2], c[3])[None]


# --------------------------------------------------------------------------
# HeatmapHead (heatmap_head.py:81-151)
# --------------------------------------------------------------------------
def heatmap_head(x: Tensor, sd: SD, p: str = "heatmap_head.") -> Tensor:
    cw = torch.sigmoid(_fc2(x.mean(dim=(2, 3)), sd, p + "channel_attention.")
                       + _fc2(x.amax(dim=(2, 3)), sd, p + "channel_attention."))
    x = x * cw[:, :, None, None]
    sa = torch.cat([x.mean(dim=1, keepdim=True), x.amax(dim=1, keepdim=True)], dim=1)
    sw = torch.sigmoid(F.conv2d(sa, sd[p + "spatial_attention.conv.weight"],
                                sd[p + "spatial_attention.conv.bias"], 1, 3))
    x = x * sw
    d = p + "deconv_layers."
    x = F.relu(_bn(F.conv2d(x, sd[d + "0.weight"], sd[d + "0.bias"], 1, 1), sd, d + "1", BN_EPS))
    x = F.relu(_bn(F.conv2d(x, sd[d + "4.weight"], sd[d + "4.bias"], 1, 1), sd, d + "5", BN_EPS))
    f = p + "final_layer."
    x = F.relu(_bn(F.conv2d(x, sd[f + "0.weight"], sd[f + "0.bias"], 1, 1), sd, f + "1", BN_EPS))
    x = F.conv2d(x, sd[f + "3.weight"], sd[f + "3.bias"])
    return torch.sigmoid(x)


# --------------------------------------------------------------------------
# decode (keypoint_model.py:250-313) and coordinate transform (:230-248)
# --------------------------------------------------------------------------
def soft_argmax(hm: Tensor) -> Tensor:
    B, K, H, W = hm.shape
    p = torch.softmax(hm.view(B, K, -1), dim=-1).view(B, K, H, W)
    xs = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W)
    ys = torch.arange(H, dtype=torch.float32).view(1, 1, H, 1)
    ex = (p * xs).sum(dim=(2, 3)) / (W - 1)
    ey = (p * ys).sum(dim=(2, 3)) / (H - 1)
    return torch.stack([ex, ey], dim=-1)


def visibility_classes(hm: Tensor) -> Tensor:
    B, K = hm.shape[:2]
    conf = torch.sigmoid(hm.view(B, K, -1).amax(dim=2))
    cls = torch.where(conf < 0.3, 0, torch.where(conf < 0.7, 1, 2))
    return F.one_hot(cls, 3).to(torch.float32)


def decode_heatmap(hm: Tensor) -> Tuple[Tensor, Tensor]:
    return soft_argmax(hm), visibility_classes(hm)


def to_image_coords(kpts: Tensor, box: Tensor) -> Tensor:
    shape = kpts.shape
    k = kpts.reshape(-1, 2)
    cx, cy, w, h = box
    x = torch.clamp(k[:, 0] * w + (cx - w / 2), 0, 1)
    y = torch.clamp(k[:, 1] * h + (cy - h / 2), 0, 1)
    return torch.stack([x, y], dim=-1).view(shape)


def pad_to_length(ts: List[Tensor], n: int) -> List[Tensor]:
    if not ts:
        return []
    if len(ts) >= n:
        return ts[:n]
    return ts + [torch.zeros_like(ts[0]) for _ in range(n - len(ts))]


# --------------------------------------------------------------------------
# bbox-argument normalisation (keypoint_model.py:93-113)
# --------------------------------------------------------------------------
def normalize_bboxes(batch, batch_size: int) -> Optional[List[Tensor]]:
    """Returns the per-image box list, or None when the person-detector branch
    would be taken (no 'bboxes' key / non-dict batch)."""
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
    return [torch.zeros(0, 4) for _ in range(batch_size)]


# --------------------------------------------------------------------------
# full eval forward with caller-given boxes (keypoint_model.py:73-210)
# --------------------------------------------------------------------------
@torch.no_grad()
def forward(sd: SD, batch, return_debug: bool = False, dual_head: bool = False, kh_size: int = 56,
            detect: Optional[dict] = None):
    """Eval forward.  ``detect`` (dict of person_detect kwargs) enables the
    build-defined detector glue when the batch carries no 'bboxes';
    ``dual_head`` also runs KEYPOINT_HEAD ("keypoint_head." weights) on the
    128-channel ROI features (outputs 'kh_keypoints' / 'kh_visibilities')."""
    x = batch["image"] if isinstance(batch, dict) else batch
    if not isinstance(x, torch.Tensor):
        raise TypeError("Input must be a tensor or a dict with 'image' key containing a tensor")
    x = x.float()
    B = x.size(0)
    feat0 = backbone_level0(x, sd)
    feats, topk = select_top_k(feat0, sd)
    boxes = normalize_bboxes(batch, B)
    det_s = None
    if boxes is None:
        if detect is None:
            raise NotImplementedError("person-detector branch: pass detect=dict(...)")
        det, det_s = person_detect(feat0, sd, x.shape[2], x.shape[3], **detect)
        boxes = [det[b] for b in range(B)]
    K = NUM_KEYPOINTS
    if not boxes or all(len(b) == 0 for b in boxes):
        out = {"keypoints": torch.zeros(B, 1, K, 2), "visibilities": torch.zeros(B, 1, K),
               "heatmap": torch.zeros(B, 1, K, 56, 56), "boxes": boxes}
        if return_debug:
            out["_feat0"] = feat0; out["_topk"] = topk
        return out
    pmax = max(len(b) for b in boxes)
    ph, pk, pv, pkk, pkv = [], [], [], [], []
    for bi, bx in enumerate(boxes):
        hs, ks, vs, kks, kvs = [], [], [], [], []
        for box in bx:
            box = box.float()
            if torch.all(box == 0) or box.shape[-1] != 4:
                continue
            roi = extract_roi_features(feats[bi:bi + 1], box)
            hm = heatmap_head(roi, sd)
            kp, vis = decode_heatmap(hm)
            kp = to_image_coords(kp, box)
            hs.append(hm); ks.append(kp); vs.append(vis)
            if dual_head:
                r128 = extract_roi_features(feat0[bi:bi + 1], box)
                a, v = keypoint_head(r128, sd, "keypoint_head.", K, kh_size, kh_size)
                kks.append(a); kvs.append(v)
        if not ks:
            dv = torch.zeros(1, K, 3); dv[:, :, 0] = 1.0
            ks.append(torch.zeros(1, K, 2)); hs.append(torch.zeros(1, K, 56, 56)); vs.append(dv)
            kks.append(torch.zeros(1, K, 2)); kvs.append(torch.zeros(1, K, 3))
        ks, hs, vs = pad_to_length(ks, pmax), pad_to_length(hs, pmax), pad_to_length(vs, pmax)
        pk.append(torch.stack(ks)); ph.append(torch.stack(hs)); pv.append(torch.stack(vs))
        if dual_head:
            pkk.append(torch.stack(pad_to_length(kks, pmax))); pkv.append(torch.stack(pad_to_length(kvs, pmax)))
    out = {"heatmap": torch.stack(ph).squeeze(2), "keypoints": torch.stack(pk),
           "visibilities": torch.stack(pv), "boxes": boxes}
    if dual_head:
        out["kh_keypoints"] = torch.stack(pkk)
        out["kh_visibilities"] = torch.stack(pkv)
    if det_s is not None:
        out["box_scores"] = det_s
    if return_debug:
        out["_feat0"] = feat0; out["_topk"] = topk
    return out


# --------------------------------------------------------------------------
# PERSON_HEAD pieces (person_head.py:39-139)
# --------------------------------------------------------------------------
def generate_anchors(grid_h: int = 56, grid_w: int = 56, sizes=(32, 64, 128),
                     ratios=(0.5, 1.0, 2.0)) -> Tensor:
    a = []
    for i in range(grid_h):
        for j in range(grid_w):
            cx = (j + 0.5) / grid_w
            cy = (i + 0.5) / grid_h
            for s in sizes:
                for r in ratios:
                    a.append([cx, cy, s * r, s / r])
    return torch.tensor(a, dtype=torch.float32)


def box_iou_cxcywh(b1: Tensor, b2: Tensor) -> Tensor:
    def corners(b):
        return (b[:, 0] - b[:, 2] / 2, b[:, 1] - b[:, 3] / 2,
                b[:, 0] + b[:, 2] / 2, b[:, 1] + b[:, 3] / 2)
    ax1, ay1, ax2, ay2 = corners(b1)
    bx1, by1, bx2, by2 = corners(b2)
    iw = torch.clamp(torch.min(ax2[:, None], bx2) - torch.max(ax1[:, None], bx1), min=0)
    ih = torch.clamp(torch.min(ay2[:, None], by2) - torch.max(ay1[:, None], by1), min=0)
    inter = iw * ih
    a1 = (ax2 - ax1) * (ay2 - ay1)
    a2 = (bx2 - bx1) * (by2 - by1)
    return inter / (a1[:, None] + a2 - inter + 1e-16)


def nms(boxes: Tensor, scores: Tensor, iou_threshold: float = 0.2,
        max_output_size: Optional[int] = None, stable: bool = False) -> Tensor:
    """Greedy NMS exactly as person_head.py:96-139 (IoU > thr suppressed; the
    sort order of ``scores.sort(descending=True)`` decides ties).  stable=True
    breaks ties by the lower index (a stable sort: one of the orders the
    reference's unstable sort may produce, and the one the HIP kernel uses)."""
    if stable:
        _, order = torch.sort(scores, dim=0, descending=True, stable=True)
    else:
        _, order = scores.sort(0, descending=True)
    keep: List[int] = []
    while order.numel() > 0:
        if order.numel() == 1:
            keep.append(int(order.item()))
            break
        i = order[0]
        keep.append(int(i.item()))
        if max_output_size and len(keep) >= max_output_size:
            break
        order = order[1:]
        iou = box_iou_cxcywh(boxes[i].unsqueeze(0), boxes[order])
        order = order[(iou <= iou_threshold).squeeze(0)]
    return torch.tensor(keep, dtype=torch.int64)


# --------------------------------------------------------------------------
# Person-detector glue (build-defined; the reference's PERSON_HEAD.forward
# never decodes boxes nor runs NMS, person_head.py:141-166 -- DESIGN.md §C3):
#   1. FPN level 0 (128 ch) adaptive-avg-pooled to the anchor grid 56x56
#   2. box_heads[0] / cls_heads[0] 1x1 convs (36 = 9 anchors x 4, 9 logits)
#   3. score = sigmoid(logit); candidates score > conf_threshold
#   4. decode against the reference's anchors buffer, anchor w/h in pixels
#      normalised by the input width/height:
#        cx = ax + dx*aw, cy = ay + dy*ah, w = aw*exp(min(dw, 4.135)), h = ...
#   5. greedy NMS (person_head.py:96-139), keep <= max_persons, zero padded
# --------------------------------------------------------------------------
BBOX_CLIP = math.log(1000.0 / 16)


def person_detect(feat0: Tensor, sd: SD, img_h: int, img_w: int, conf_threshold: float = 0.3,
                  iou_threshold: float = 0.3, max_persons: int = 5,
                  p: str = "person_detector.") -> Tuple[Tensor, Tensor]:
    B = feat0.shape[0]
    g = F.adaptive_avg_pool2d(feat0, (56, 56))
    box = F.conv2d(g, sd[p + "box_heads.0.weight"], sd[p + "box_heads.0.bias"])     # [B,36,56,56]
    cls = F.conv2d(g, sd[p + "cls_heads.0.weight"], sd[p + "cls_heads.0.bias"])     # [B,9,56,56]
    box = box.permute(0, 2, 3, 1).reshape(B, -1, 4)                                  # [(i,j,a)] order
    score = torch.sigmoid(cls.permute(0, 2, 3, 1).reshape(B, -1))
    anc = sd[p + "anchors"]
    aw = anc[:, 2] / img_w
    ah = anc[:, 3] / img_h
    cx = anc[:, 0] + box[..., 0] * aw
    cy = anc[:, 1] + box[..., 1] * ah
    w = aw * torch.exp(torch.clamp(box[..., 2], max=BBOX_CLIP))
    h = ah * torch.exp(torch.clamp(box[..., 3], max=BBOX_CLIP))
    dec = torch.stack([cx, cy, w, h], dim=-1)
    out = torch.zeros(B, max_persons, 4)
    out_s = torch.zeros(B, max_persons)
    for b in range(B):
        cand = torch.nonzero(score[b] > conf_threshold).flatten()
        if cand.numel() == 0:
            continue
        keep = nms(dec[b, cand], score[b, cand], iou_threshold, max_persons)
        k = cand[keep]
        out[b, :len(k)] = dec[b, k]
        out_s[b, :len(k)] = score[b, k]
    return out, out_s


# --------------------------------------------------------------------------
# KEYPOINT_HEAD (keypoint_head.py:9-90), eval mode
# --------------------------------------------------------------------------
def _resblock(x: Tensor, sd: SD, p: str) -> Tensor:
    out = F.conv2d(x, sd[p + "conv1.0.weight"], sd[p + "conv1.0.bias"], 1, 1)
    out = F.relu6(_bn(out, sd, p + "conv1.1", BN_EPS))
    out = F.relu6(_bn(out, sd, p + "bn1", BN_EPS))
    if (p + "downsample.0.weight") in sd:
        idn = _bn(F.conv2d(x, sd[p + "downsample.0.weight"], sd[p + "downsample.0.bias"]),
                  sd, p + "downsample.1", BN_EPS)
    else:
        idn = x
    return F.relu6(out + idn)


def keypoint_head(x: Tensor, sd: SD, p: str, num_kpts: int = NUM_KEYPOINTS,
                  height: int = 56, width: int = 56) -> Tuple[Tensor, Tensor]:
    B = x.shape[0]
    s = p + "spatial_attention."
    att = F.relu6(F.conv2d(x, sd[s + "0.weight"], sd[s + "0.bias"]))
    att = torch.sigmoid(F.conv2d(att, sd[s + "2.weight"], sd[s + "2.bias"]))
    x = x * att
    r = p + "regression_branch."
    y = _resblock(x, sd, r + "0.")
    y = _resblock(y, sd, r + "1.")
    y = F.relu6(_bn(F.conv2d(y, sd[r + "2.weight"], sd[r + "2.bias"], 1, 1), sd, r + "3", BN_EPS))
    y = F.adaptive_avg_pool2d(y, (height // 4, width // 4)).flatten(1)
    y = F.linear(y, sd[r + "7.weight"], sd[r + "7.bias"])
    y = F.relu6(F.layer_norm(y, (y.shape[-1],), sd[r + "8.weight"], sd[r + "8.bias"]))
    y = F.linear(y, sd[r + "11.weight"], sd[r + "11.bias"])
    kp = torch.sigmoid(y).view(B, num_kpts, 2)
    v = p + "visibility_branch."
    z = F.relu6(_bn(F.conv2d(x, sd[v + "0.weight"], sd[v + "0.bias"], 1, 1), sd, v + "1", BN_EPS))
    z = F.adaptive_avg_pool2d(z, (4, 4)).flatten(1)
    z = F.linear(z, sd[v + "5.weight"], sd[v + "5.bias"])
    z = F.relu6(F.layer_norm(z, (z.shape[-1],), sd[v + "6.weight"], sd[v + "6.bias"]))
    z = F.linear(z, sd[v + "9.weight"], sd[v + "9.bias"])
    vis = torch.sigmoid(z).view(B, num_kpts, 3)
    return kp, vis
