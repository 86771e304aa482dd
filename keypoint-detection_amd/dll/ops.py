"""Training-side operator (the backward of K6): the
HeatmapHead's 3x3 convolution -- nn.Conv2d(C, O, 3, padding=1), reference
dll/models/heatmap_head.py:31-45,55-66 -- as an autograd Function whose
forward and backward both run native (libkpd: kpd_conv3x3_forward /
kpd_conv3x3_backward: fp32-accurate split f16 hi / lo MFMA products with fp32
accumulation for the forward and dgrad at 56 x 56 with 64 | 256 channels and
for every wgrad, exact fp32 products on the generic fallback; deterministic
sums).  The
reference gets these gradients from autograd in Trainer.train
(dll/training/trainer.py:263,272).

    from dll.ops import conv3x3
    y = conv3x3(x, conv.weight, conv.bias)     # == F.conv2d(x, w, b, padding=1)
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native


class Conv3x3Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        return _native.conv3x3_forward(x, weight, bias).to(x.dtype)   # computed in fp32, returned like F.conv2d

    @staticmethod
    def backward(ctx, grad_y: torch.Tensor):
        x, weight = ctx.saved_tensors
        nx, nw, nb = ctx.needs_input_grad
        gx, gw, gb = _native.conv3x3_backward(x, weight, grad_y, need_x=nx, need_w=nw, need_b=ctx.has_bias and nb)
        if gw is not None:
            gw = gw.to(weight.dtype)
        if gx is not None:
            gx = gx.to(x.dtype)
        if gb is not None:
            gb = gb.to(ctx.bias_dtype)
        return gx, gw, gb


def conv3x3(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """F.conv2d(x, weight, bias, padding=1) with a native forward and backward."""
    return Conv3x3Function.apply(x, weight, bias)
