"""HeatmapHead parameter container (reference: dll/models/heatmap_head.py:20-151).

Same submodule names as the reference -- ``channel_attention.fc.{0,2}``,
``spatial_attention.conv``, ``deconv_layers.{0,1,4,5}``,
``final_layer.{0,1,3}`` -- so state dicts load unchanged.  The arithmetic
(attention, the three 3x3 convs on MFMA, the 1x1 + sigmoid) runs inside the
native plan for all ROIs of a batch at once (csrc/head_kernels.hip,
csrc/conv_mfma.hip).
"""
import torch.nn as nn

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
