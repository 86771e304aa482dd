"""Backbone: MobileNetV3-Small body + LightweightFPN.

The modules keep the reference's state-dict names (``backbone.body.features.N...``
from torchvision's mobilenet_v3_small via ``create_feature_extractor``;
``backbone.fpn.{lateral_convs,fpn_convs}``) so that reference checkpoints load
unchanged.  ``MobileNetV3Wrapper.forward`` runs the native HIP plan
(kpd_backbone: csrc/ folds BN and repacks to NHWC at load time) and returns
the four FPN levels as the reference does.  ``body(x)`` (the feature
extractor's four taps, kpd_backbone_body) and ``fpn(taps)`` (kpd_backbone_fpn)
are native on their own too, for callers of the reference's sub-modules.

Reference: dll/models/backbone.py:7-39 (LightweightFPN), :247-264
(MobileNetV3Wrapper); torchvision mobilenet_v3_small topology restated in
oracle/kpd_oracle.py:MBV3_SMALL_BNECK.
"""
from collections import OrderedDict
from typing import List

import torch.nn as nn

from .. import _native
from ..configs.model_config import BackboneConfig

# (in, kernel, expanded, out, use_se, activation, stride) -- torchvision table
MBV3_SMALL_BNECK = (
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
FPN_IN_CHANNELS = [16, 24, 48, 576]
BODY_BN_EPS = 1e-3


def squeeze_width(c: int, divisor: int = 8) -> int:
    """SE squeeze channels = torchvision _make_divisible(c // 4, 8)."""
    v = c // 4
    n = max(divisor, int(v + divisor / 2) // divisor * divisor)
    return n + divisor if n < 0.9 * v else n


class ConvBN(nn.Sequential):
    """``N.0`` conv (no bias) + ``N.1`` BatchNorm (eps 1e-3)."""

    def __init__(self, cin, cout, k, stride=1, groups=1):
        super().__init__(nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
                         nn.BatchNorm2d(cout, eps=BODY_BN_EPS, momentum=0.01))


class SqueezeExcitation(nn.Module):
    def __init__(self, c: int, sq: int):
        super().__init__()
        self.fc1 = nn.Conv2d(c, sq, 1)
        self.fc2 = nn.Conv2d(sq, c, 1)


class InvertedResidual(nn.Module):
    def __init__(self, cin, k, exp, cout, se, stride):
        super().__init__()
        layers: List[nn.Module] = []
        if exp != cin:
            layers.append(ConvBN(cin, exp, 1))
        layers.append(ConvBN(exp, exp, k, stride, groups=exp))
        if se:
            layers.append(SqueezeExcitation(exp, squeeze_width(exp)))
        layers.append(ConvBN(exp, cout, 1))
        self.block = nn.Sequential(*layers)


class MobileNetV3SmallBody(nn.Module):
    """features.0..12 of mobilenet_v3_small (the part create_feature_extractor keeps)."""

    RETURN_NODES = (("features.0", "feat0"), ("features.3", "feat1"), ("features.8", "feat2"),
                    ("features.12", "feat3"))

    def forward(self, x):
        """The feature extractor's call (backbone.py:253-254, 259): x [B,C,H,W] ->
        OrderedDict feat0 [B,16,H/2,W/2], feat1 [B,24,H/8,W/8], feat2
        [B,48,H/16,W/16], feat3 [B,576,H/32,W/32] (kpd_backbone_body; eval only)."""
        if self.training:
            raise NotImplementedError("the backbone runs the eval path only; call .eval()")
        taps = self._plans.get(self, x.device, "fp32").body_taps(x)
        return OrderedDict((name, t) for (_, name), t in zip(self.RETURN_NODES, taps))

    def __init__(self, in_channels: int = 3):
        super().__init__()
        mods: List[nn.Module] = [ConvBN(in_channels, 16, 3, 2)]
        for cin, k, exp, cout, se, _act, s in MBV3_SMALL_BNECK:
            mods.append(InvertedResidual(cin, k, exp, cout, se, s))
        mods.append(ConvBN(96, 576, 1))
        self.features = nn.Sequential(*mods)
        self._plans = _native.PlanCache("backbone.body.", in_channels)


class LightweightFPN(nn.Module):
    def forward(self, features):
        """features: the four taps [B,c_i,h_i,w_i] -> four [B,128,h_i,w_i] levels
        (backbone.py:29-39; kpd_backbone_fpn, eval only)."""
        if len(features) != len(self.lateral_convs):
            raise ValueError(f"Expected {len(self.lateral_convs)} features, got {len(features)}")
        if self.training:
            raise NotImplementedError("the FPN runs the eval path only; call .eval()")
        return self._plans.get(self, features[0].device, "fp32").fpn(list(features))

    def __init__(self, in_channels_list, out_channels):
        super().__init__()
        if not isinstance(in_channels_list, list):
            raise ValueError("in_channels_list must be a list of input channel sizes")
        self.lateral_convs = nn.ModuleList(
            [nn.Conv2d(c, out_channels, 1, bias=False) for c in in_channels_list])
        self.fpn_convs = nn.ModuleList([
            nn.Sequential(nn.Conv2d(out_channels, out_channels, 3, 1, 1, bias=False),
                          nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))
            for _ in in_channels_list])
        self._plans = _native.PlanCache("backbone.fpn.")


class MobileNetV3Wrapper(nn.Module):
    precision = "split"   # FPN level 0 as the fp32-accurate f16 split ("fp32": fp32 MFMA)
    """Same attribute names as the reference wrapper: ``body`` and ``fpn``.

    ``weights=MobileNet_V3_Small_Weights.DEFAULT`` is a network download in the
    reference (backbone.py:250); here the body starts from the deterministic
    initialisation and real weights come from ``load_state_dict``."""

    def __init__(self, config: BackboneConfig, out_channels: int = 128, attention_module=None):
        super().__init__()
        self.body = MobileNetV3SmallBody(config.in_channels)
        self.fpn = LightweightFPN(list(FPN_IN_CHANNELS), out_channels)
        self.attention_module = attention_module
        self.in_channels = config.in_channels
        self._plans = _native.PlanCache("backbone.", config.in_channels)

    def forward(self, x):
        """x [B, C, H, W] -> the four FPN outputs [B, 128, h_i, w_i] at strides
        2 / 8 / 16 / 32 (reference backbone.py:258-264, LightweightFPN :29-39).
        Eval only (BatchNorm running statistics)."""
        if self.training:
            raise NotImplementedError("the backbone runs the eval path only; call .eval()")
        outs = self._plans.get(self, x.device, self.precision).backbone(x)
        if self.attention_module:
            outs[0] = self.attention_module(outs[0])
        return outs


class BACKBONE(nn.Module):
    """The reference's alternative custom backbone is not used by the model
    (out of scope); kept as a named placeholder so
    ``from dll.models import BACKBONE`` still resolves."""

    def __init__(self, config: BackboneConfig):
        super().__init__()
        raise NotImplementedError("BACKBONE (custom MobileNetV3) is outside the accelerated "
                                  "path; MultiPersonKeypointModel uses MobileNetV3Wrapper")
