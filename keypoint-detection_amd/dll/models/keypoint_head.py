"""KEYPOINT_HEAD (reference: dll/models/keypoint_head.py:9-90).

Submodule names match the reference (``spatial_attention.{0,2}``,
``regression_branch.{0,1,2,3,7,8,11}``, ``visibility_branch.{0,1,5,6,9}``,
``ResidualBlock.{conv1.{0,1},bn1,downsample.{0,1}}``).  ``forward`` runs the
native HIP path (kpd_keypoint_head: spatial attention, the residual blocks
and 3x3 convs on MFMA with fused BN / ReLU6 / residual epilogues, pooling,
both Linear layers as GEMMs, LayerNorm + sigmoid heads) on the module's own
plan under the ``keypoint_head.`` prefix.  Not instantiated by
``MultiPersonKeypointModel`` unless ``dual_head=True`` (the reference never
wires it in, keypoint_model.py:55-57).
"""
import torch
import torch.nn as nn

from .. import _native
from ..configs.model_config import KeypointHeadConfig


class ResidualBlock(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv2d(in_channels, out_channels, 3, padding=1), nn.BatchNorm2d(out_channels),
                                   nn.ReLU6(inplace=True))
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.downsample = None
        if in_channels != out_channels:
            self.downsample = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1), nn.BatchNorm2d(out_channels))


class KEYPOINT_HEAD(nn.Module):
    precision = "split"   # the convs run fp32 in every precision; kept for a uniform plan key

    def __init__(self, config: KeypointHeadConfig):
        super().__init__()
        self._plans = _native.PlanCache("keypoint_head.")
        self.num_keypoints = config.num_keypoints
        c = config.in_channels
        self.height, self.width = config.height, config.width
        self.spatial_attention = nn.Sequential(nn.Conv2d(c, c // 2, 1), nn.ReLU6(inplace=True),
                                               nn.Conv2d(c // 2, 1, 1), nn.Sigmoid())
        rc = config.regression_channels
        ph, pw = config.height // 4, config.width // 4
        self.regression_branch = nn.Sequential(
            ResidualBlock(c, config.fine_branch_channels),
            ResidualBlock(config.fine_branch_channels, rc),
            nn.Conv2d(rc, rc // 2, 3, padding=1), nn.BatchNorm2d(rc // 2), nn.ReLU6(inplace=True),
            nn.AdaptiveAvgPool2d((ph, pw)), nn.Flatten(),
            nn.Linear(rc // 2 * ph * pw, 256), nn.LayerNorm(256), nn.ReLU6(inplace=True),
            nn.Dropout(config.dropout_rate), nn.Linear(256, self.num_keypoints * 2))
        vc = config.visibility_channels
        self.visibility_branch = nn.Sequential(
            nn.Conv2d(c, vc, 3, padding=1), nn.BatchNorm2d(vc), nn.ReLU6(inplace=True),
            nn.AdaptiveAvgPool2d((4, 4)), nn.Flatten(),
            nn.Linear(vc * 16, 128), nn.LayerNorm(128), nn.ReLU6(inplace=True),
            nn.Dropout(config.dropout_rate), nn.Linear(128, self.num_keypoints * 3))

    def forward(self, x: torch.Tensor):
        """x [B, 128, 56, 56] -> (keypoints [B, 17, 2], visibility [B, 17, 3]),
        both sigmoid outputs (reference :50-62).  Eval only (BatchNorm running
        statistics, dropout off)."""
        if self.training:
            raise NotImplementedError("KEYPOINT_HEAD runs the eval path only; call .eval()")
        if x.dim() != 4 or x.size(2) != self.height or x.size(3) != self.width:
            raise ValueError(f"expected [B, C, {self.height}, {self.width}] input, got {tuple(x.shape)}")
        return self._plans.get(self, x.device, self.precision).keypoint_head(x)
