"""HeatmapHead (reference: dll/models/heatmap_head.py:20-151) and the heatmap
decoders (:265-413).

Same submodule names as the reference -- ``channel_attention.fc.{0,2}``,
``spatial_attention.conv``, ``deconv_layers.{0,1,4,5}``,
``final_layer.{0,1,3}`` -- so state dicts load unchanged.  ``forward`` runs
the native HIP path on the input's device (csrc/: the attention kernels, the
three 3x3 convs on MFMA and the fused final 1x1 + sigmoid, kpd_heatmap_head):
the module packs its own weights into a plan under the model's
``heatmap_head.`` prefix.  The decoders are device kernels
(kpd_decode_heatmaps).  There is no CPU fallback: CPU inputs raise.
"""
import ctypes
import weakref
from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import _native
from ..configs.model_config import HeatmapHeadConfig


class ChannelAttention(nn.Module):
    """sigmoid(fc(avgpool) + fc(maxpool)), returned as [B, C, 1, 1] (reference :115-136).
    Runs through the owning HeatmapHead's native plan."""

    def __init__(self, in_channels: int, reduction_ratio: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.fc = nn.Sequential(nn.Linear(in_channels, in_channels // reduction_ratio), nn.ReLU(inplace=True),
                                nn.Linear(in_channels // reduction_ratio, in_channels))
        self._owner = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        head = _owner(self)
        _, cw, _ = head._plan(x.device).heatmap_head(x, _native.HEAD_CHANNEL_ATT)
        return cw.view(x.size(0), -1, 1, 1)


class SpatialAttention(nn.Module):
    """sigmoid(conv7x7([mean_c, max_c])) as [B, 1, H, W] (reference :138-151)."""

    def __init__(self, kernel_size: int = 7):
        super().__init__()
        self.conv = nn.Conv2d(2, 1, kernel_size=kernel_size, padding=kernel_size // 2)
        self._owner = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        head = _owner(self)
        _, _, sw = head._plan(x.device).heatmap_head(x, _native.HEAD_SPATIAL_ATT)
        return sw.unsqueeze(1)


def _owner(m: nn.Module) -> "HeatmapHead":
    head = m._owner() if m._owner is not None else None
    if head is None:
        raise NotImplementedError(f"{type(m).__name__}.forward runs through its HeatmapHead's native plan; "
                                  "use it as a HeatmapHead submodule (or call HeatmapHead.forward)")
    return head


class HeatmapHead(nn.Module):
    precision = "split"   # "fp32" | "split" (fp32-accurate) | "mixed" (bf16 convs); the model sets its own

    def __init__(self, config: HeatmapHeadConfig):
        super().__init__()
        self.config = config
        if config.use_attention:
            self.channel_attention = ChannelAttention(config.in_channels)
            self.spatial_attention = SpatialAttention()
            self.channel_attention._owner = weakref.ref(self)
            self.spatial_attention._owner = weakref.ref(self)
        layers = []
        for i in range(config.num_deconv_layers):
            cin = config.in_channels if i == 0 else config.deconv_channels[i - 1]
            layers += [nn.Conv2d(cin, config.deconv_channels[i], 3, 1, 1), nn.BatchNorm2d(config.deconv_channels[i]),
                       nn.ReLU(inplace=True), nn.Dropout2d(config.dropout_rate)]
        self.deconv_layers = nn.Sequential(*layers)
        self.final_layer = nn.Sequential(
            nn.Conv2d(config.deconv_channels[-1], config.hidden_channels, 3, padding=1),
            nn.BatchNorm2d(config.hidden_channels), nn.ReLU(inplace=True),
            nn.Conv2d(config.hidden_channels, config.num_keypoints, 1))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self._plans = _native.PlanCache("heatmap_head.")

    def _plan(self, device: torch.device) -> "_native.Plan":
        if self.training:
            raise NotImplementedError("HeatmapHead runs the eval path only (BatchNorm running statistics, no "
                                      "dropout); call .eval()")
        return self._plans.get(self, device, self.precision)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, Optional[Tuple[torch.Tensor, torch.Tensor]]]:
        """x [B, 64, 56, 56] ROI features -> (heatmaps [B, 17, 56, 56] in (0, 1),
        (channel weights [B, 64, 1, 1], spatial weights [B, 1, 56, 56]) or None
        without attention) -- reference :81-113."""
        parts = _native.HEAD_ALL if self.config.use_attention else _native.HEAD_CONVS
        heat, cw, sw = self._plan(x.device).heatmap_head(x, parts)
        att = (cw.view(x.size(0), -1, 1, 1), sw.unsqueeze(1)) if self.config.use_attention else None
        return heat, att


def _ensure_batch(heatmaps: torch.Tensor) -> Tuple[torch.Tensor, bool]:
    if heatmaps.dim() == 3:
        return heatmaps.unsqueeze(0), True
    return heatmaps, False


def _remove_batch(t: torch.Tensor, was_3d: bool) -> torch.Tensor:
    return t.squeeze(0) if was_3d else t


def decode_heatmaps(heatmaps: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Argmax decode (reference :265-296): normalised (x, y) of each map's
    maximum (first index on ties, as torch.max) and the maximum as the score.
    [B,K,H,W] -> ([B,K,2], [B,K]); a [K,H,W] input drops the batch dim."""
    h, was_3d = _ensure_batch(heatmaps)
    kp, sc, _ = _native.decode_heatmaps(h, _native.DECODE_ARGMAX)
    return _remove_batch(kp, was_3d), _remove_batch(sc, was_3d)


def decode_heatmaps_subpixel(heatmaps: torch.Tensor, window_size: int = 3) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mass-weighted mean over the window around each maximum (reference
    :298-370); the window's maximum as the score, zeros where the window's
    mass is not positive.  Keeps the reference's shape quirk: a [K,H,W] input
    returns [1,K,2] / [1,K] (its batch-dim removal never triggers)."""
    h = heatmaps.unsqueeze(0) if heatmaps.dim() == 3 else heatmaps
    kp, sc, _ = _native.decode_heatmaps(h, _native.DECODE_SUBPIXEL, float(window_size))
    return kp, sc


def decode_heatmaps_soft_argmax(heatmaps: torch.Tensor, temperature: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Soft-argmax (integral regression) over softmax(h / temperature)
    (reference :372-413); the raw maximum as the score."""
    h, was_3d = _ensure_batch(heatmaps)
    kp, sc, _ = _native.decode_heatmaps(h, _native.DECODE_SOFTARGMAX, float(temperature))
    return _remove_batch(kp, was_3d), _remove_batch(sc, was_3d)


def generate_target_heatmap(keypoints: torch.Tensor, heatmap_size: Tuple[int, int], sigma: float = 3.0) -> torch.Tensor:
    """Gaussian training targets (reference heatmap_head.py:163-224) on the
    device (``kpd_target_heatmaps``).  [B,P,K,2] input is flattened to B*P
    rows of which the reference fills the first B (its loop runs over B);
    [B,K,2] gives one plane set per row.  Returns [B,K,H,W] fp32.  Values
    match the reference within fp32 rounding of the normalised kernel."""
    if keypoints.dim() == 4:
        B, P, K, _ = keypoints.shape
        kp = keypoints.reshape(B * P, K, -1)[:B]
    elif keypoints.dim() == 3:
        B, K, _ = keypoints.shape
        kp = keypoints
    else:
        raise ValueError(f"Unexpected keypoints shape: {keypoints.shape}")
    _native._require_cuda(keypoints, "keypoints")
    H, W = int(heatmap_size[0]), int(heatmap_size[1])
    kp = kp[..., :2].float().contiguous()
    out = torch.empty(B, K, H, W, device=kp.device, dtype=torch.float32)
    lib = _native.load()
    with torch.cuda.device(kp.device):
        rc = lib.kpd_target_heatmaps(_native._ptr(kp), B * K, H, W, ctypes.c_float(sigma), _native._ptr(out),
                                     _native._stream(kp.device))
    _native.check(rc, "kpd_target_heatmaps")
    return out


def generate_target_heatmap_adaptive(keypoints: torch.Tensor, heatmap_size: Tuple[int, int],
                                     base_sigma: float = 3.0, adaptive: bool = True) -> torch.Tensor:
    """Reference :226-252: sigma scaled with min(H, W) / 56, floored at 0.8x."""
    sigma = base_sigma * max(0.8, min(heatmap_size) / 56.0) if adaptive else base_sigma
    return generate_target_heatmap(keypoints, heatmap_size, sigma)
