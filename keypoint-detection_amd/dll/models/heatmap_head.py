"""HeatmapHead parameter container (reference: dll/models/heatmap_head.py:20-151).

Same submodule names as the reference -- ``channel_attention.fc.{0,2}``,
``spatial_attention.conv``, ``deconv_layers.{0,1,4,5}``,
``final_layer.{0,1,3}`` -- so state dicts load unchanged.  The arithmetic
(attention, the three 3x3 convs on MFMA, the 1x1 + sigmoid) runs inside the
native plan for all ROIs of a batch at once (csrc/head_kernels.hip,
csrc/conv_mfma.hip).
"""
import ctypes
from typing import Tuple

import torch
import torch.nn as nn

from .. import _native
from ..configs.model_config import HeatmapHeadConfig


class ChannelAttention(nn.Module):
    def __init__(self, in_channels: int, reduction_ratio: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.fc = nn.Sequential(nn.Linear(in_channels, in_channels // reduction_ratio), nn.ReLU(inplace=True),
                                nn.Linear(in_channels // reduction_ratio, in_channels))


class SpatialAttention(nn.Module):
    def __init__(self, kernel_size: int = 7):
        super().__init__()
        self.conv = nn.Conv2d(2, 1, kernel_size=kernel_size, padding=kernel_size // 2)


class HeatmapHead(nn.Module):
    def __init__(self, config: HeatmapHeadConfig):
        super().__init__()
        self.config = config
        if config.use_attention:
            self.channel_attention = ChannelAttention(config.in_channels)
            self.spatial_attention = SpatialAttention()
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
