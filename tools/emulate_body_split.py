#!/usr/bin/env python3
"""CPU emulation: what does running the MobileNet body's 1x1 convs (features
4..12) as f16 hi/lo x3 MFMA products do to the channel-attention scores and
the top-64 order, compared with the fp32 path the reference runs?

Three paths over the oracle (oracle/kpd_oracle.py, golden-pinned):
  fp64  : everything in double (the "truth")
  fp32  : the reference's precision
  split : fp32, except the 1x1 convs of features.4..12 whose operands are
          split x*2^e = hi + lo (f16) with a per-image (activations) /
          per-layer (weights) power-of-two scale, products hi.hi + hi.lo +
          lo.hi accumulated in fp32 (the hmconv / fpn0x numerics)
Prints per-path max |score - fp64| and top-64 order mismatches vs fp64 and
vs fp32, and the smallest adjacent score gap.

    python tools/emulate_body_split.py [--images 64]
"""
import argparse
import math
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keypoint-detection_amd")]

from oracle import kpd_oracle as O  # noqa: E402

_orig_conv2d = F.conv2d
STATE = {"split": False, "layer": None}


def _exp_for(amax):
    # x * 2^e with max |x * 2^e| in [2^14, 2^15): hi keeps 11 bits, lo 11 more
    if amax <= 0:
        return 0
    return 14 - math.floor(math.log2(amax))


def _split(t, e):
    s = t * (2.0 ** e)
    hi = s.half().float()
    lo = (s - hi).half().float()
    return hi, lo


def split_conv1x1(x, w, b=None):
    """x [N,C,H,W] fp32, w [O,C,1,1]: per-image activation exponent, per-layer
    weight exponent, three f16 products summed in fp32."""
    N, C, H, W = x.shape
    O_ = w.shape[0]
    wm = w.view(O_, C)
    ew = _exp_for(float(wm.abs().max()))
    wh, wl = _split(wm, ew)
    out = torch.empty(N, O_, H, W)
    for n in range(N):
        xn = x[n].reshape(C, H * W)
        ex = _exp_for(float(xn.abs().max()))
        xh, xl = _split(xn, ex)
        acc = wl @ xh + wh @ xh + wh @ xl        # fp32 sums of exact products
        out[n] = (acc * 2.0 ** (-(ex + ew))).view(O_, H, W)
    if b is not None:
        out = out + b.view(1, -1, 1, 1)
    return out


def conv2d_hook(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    if STATE["split"] and w.dim() == 4 and w.shape[2] == 1 and w.shape[3] == 1 and groups == 1 \
            and x.dtype == torch.float32 and STATE.get("active"):
        return split_conv1x1(x, w, b)
    return _orig_conv2d(x, w, b, stride, padding, dilation, groups)


def body_taps(x, sd, split):
    """mbv3_small_taps with the split hook active on features.4..12 only."""
    STATE["split"] = split
    F.conv2d = conv2d_hook
    try:
        taps = []
        f = "backbone.body.features."
        x = _orig_conv2d(x, sd[f + "0.0.weight"], None, 2, 1)
        x = F.hardswish(O._bn(x, sd, f + "0.1", O.BN_EPS_BODY))
        taps.append(x)
        for i, (cin, k, exp, cout, se, act, s) in enumerate(O.MBV3_SMALL_BNECK, start=1):
            STATE["active"] = i >= 4
            p = f"{f}{i}.block."
            inp = x
            j = 0
            if exp != cin:
                x = F.conv2d(x, sd[f"{p}{j}.0.weight"])
                x = O._act(O._bn(x, sd, f"{p}{j}.1", O.BN_EPS_BODY), act)
                j += 1
            x = _orig_conv2d(x, sd[f"{p}{j}.0.weight"], None, s, (k - 1) // 2, 1, exp)
            x = O._act(O._bn(x, sd, f"{p}{j}.1", O.BN_EPS_BODY), act)
            j += 1
            if se:
                sc = F.adaptive_avg_pool2d(x, 1)
                sc = F.relu(_orig_conv2d(sc, sd[f"{p}{j}.fc1.weight"], sd[f"{p}{j}.fc1.bias"]))
                sc = F.hardsigmoid(_orig_conv2d(sc, sd[f"{p}{j}.fc2.weight"], sd[f"{p}{j}.fc2.bias"]))
                x = sc * x
                j += 1
            x = F.conv2d(x, sd[f"{p}{j}.0.weight"])
            x = O._bn(x, sd, f"{p}{j}.1", O.BN_EPS_BODY)
            if s == 1 and cin == cout:
                x = x + inp
            if i in O.MBV3_TAPS:
                taps.append(x)
        STATE["active"] = True
        x = F.conv2d(x, sd[f + "12.0.weight"])
        x = F.hardswish(O._bn(x, sd, f + "12.1", O.BN_EPS_BODY))
        taps.append(x)
        return taps
    finally:
        F.conv2d = _orig_conv2d
        STATE["split"] = False
        STATE["active"] = False


def scores_of(x, sd, split):
    taps = body_taps(x, sd, split)
    f0 = O.fpn_level(O.fpn_laterals(taps, sd)[0], sd, 0)
    return O.channel_scores(f0, sd), taps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=16)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=192)
    a = ap.parse_args()
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_images, synthetic_state_dict
    torch.set_num_threads(8)
    sd = synthetic_state_dict(MultiPersonKeypointModel(ModelConfig(), TrainingConfig()).state_dict(), seed=0)
    img = synthetic_images(a.images, 3, a.height, a.width, seed=1234)
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    with torch.no_grad():
        s64, t64 = scores_of(img.double(), sd64, False)
        s32, t32 = scores_of(img, sd, False)
        ssp, tsp = scores_of(img, sd, True)
    k64 = torch.topk(s64, 64, dim=1).indices
    for name, s, t in (("fp32", s32, t32), ("split", ssp, tsp)):
        d = (s.double() - s64).abs().max().item()
        kk = torch.topk(s, 64, dim=1).indices
        mism = int((kk != k64).any(dim=1).sum())
        tap_err = [float(((a_.double() - b_).abs().max() / b_.abs().max())) for a_, b_ in zip(t, t64)]
        print(f"{name:6s} max|score-fp64| {d:.3e}  top64 order mismatches vs fp64: {mism}/{a.images}  "
              f"tap rel err {['%.1e' % e for e in tap_err]}")
    k32 = torch.topk(s32, 64, dim=1).indices
    ksp = torch.topk(ssp, 64, dim=1).indices
    print("split vs fp32 top64 order mismatches:", int((ksp != k32).any(dim=1).sum()))
    srt = torch.sort(s64, dim=1, descending=True).values
    gaps = (srt[:, :64] - srt[:, 1:65]).abs()
    print(f"smallest adjacent gap among the top 65: {gaps.min().item():.3e}")


if __name__ == "__main__":
    main()
