"""Restatement of the torchvision pieces the reference imports (torchvision is
absent from this image; version unpinned in the reference's setup.py:13).

Used ONLY by tests/golden/make_golden.py to import the reference's own
``dll.models`` code in this container.  Restated from torchvision's published
algorithms:
  * models.mobilenet_v3_small -- MobileNetV3 'small' inverted-residual table,
    BN eps 1e-3, hardswish / hardsigmoid SE, residual iff stride 1 and in==out
    (module structure reproduces torchvision's state-dict names);
  * models.feature_extraction.create_feature_extractor -- returns the outputs
    of the named ``features.N`` nodes;
  * ops.roi_align -- the scalar-loop restatement in oracle.kpd_oracle.
``weights=`` is ignored (the ImageNet download is unavailable offline).
"""
from __future__ import annotations

import sys
import types

import torch
import torch.nn as nn

from oracle import kpd_oracle as O


class Conv2dNormActivation(nn.Sequential):
    def __init__(self, cin, cout, k=3, stride=1, groups=1, act=nn.Hardswish):
        layers = [nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
                  nn.BatchNorm2d(cout, eps=0.001, momentum=0.01)]
        if act is not None:
            layers.append(act(inplace=True))
        super().__init__(*layers)


class SqueezeExcitation(nn.Module):
    def __init__(self, c, sq):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(c, sq, 1)
        self.fc2 = nn.Conv2d(sq, c, 1)
        self.activation = nn.ReLU()
        self.scale_activation = nn.Hardsigmoid()

    def forward(self, x):
        s = self.scale_activation(self.fc2(self.activation(self.fc1(self.avgpool(x)))))
        return s * x


class InvertedResidual(nn.Module):
    def __init__(self, cin, k, exp, cout, se, act, stride):
        super().__init__()
        A = nn.ReLU if act == "RE" else nn.Hardswish
        self.use_res_connect = stride == 1 and cin == cout
        layers = []
        if exp != cin:
            layers.append(Conv2dNormActivation(cin, exp, 1, act=A))
        layers.append(Conv2dNormActivation(exp, exp, k, stride, groups=exp, act=A))
        if se:
            layers.append(SqueezeExcitation(exp, O.make_divisible(exp // 4, 8)))
        layers.append(Conv2dNormActivation(exp, cout, 1, act=None))
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        r = self.block(x)
        if self.use_res_connect:
            r += x
        return r


class MobileNetV3(nn.Module):
    def __init__(self):
        super().__init__()
        mods = [Conv2dNormActivation(3, 16, 3, 2, act=nn.Hardswish)]
        for row in O.MBV3_SMALL_BNECK:
            mods.append(InvertedResidual(*row))
        mods.append(Conv2dNormActivation(96, 576, 1, act=nn.Hardswish))
        self.features = nn.Sequential(*mods)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Linear(576, 1024), nn.Hardswish(inplace=True),
                                        nn.Dropout(0.2, inplace=True), nn.Linear(1024, 1000))


def mobilenet_v3_small(weights=None, **kw):
    return MobileNetV3()


class _Weights:
    DEFAULT = "IMAGENET1K_V1 (not downloaded)"


class _FeatureExtractor(nn.Module):
    def __init__(self, model, return_nodes):
        super().__init__()
        self.features = model.features
        self.return_nodes = {int(k.split(".")[1]): v for k, v in return_nodes.items()}

    def forward(self, x):
        out = {}
        for i, layer in enumerate(self.features):
            x = layer(x)
            if i in self.return_nodes:
                out[self.return_nodes[i]] = x
        return out


def create_feature_extractor(model, return_nodes):
    return _FeatureExtractor(model, return_nodes)


def roi_align(input, boxes, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=False):
    assert spatial_scale == 1.0 and sampling_ratio == -1 and not aligned
    out = []
    for r in boxes:
        b = int(r[0])
        out.append(O.roi_align_loop(input[b], float(r[1]), float(r[2]), float(r[3]), float(r[4]), output_size[0]))
    return torch.stack(out)


def install() -> None:
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    fe = types.ModuleType("torchvision.models.feature_extraction")
    ops = types.ModuleType("torchvision.ops")
    models.mobilenet_v3_small = mobilenet_v3_small
    models.MobileNet_V3_Small_Weights = _Weights
    fe.create_feature_extractor = create_feature_extractor
    ops.roi_align = roi_align
    tv.models, tv.ops = models, ops
    models.feature_extraction = fe
    sys.modules.update({"torchvision": tv, "torchvision.models": models,
                        "torchvision.models.feature_extraction": fe, "torchvision.ops": ops})
