#!/usr/bin/env python3
"""Timing of the K6 backward: the HeatmapHead 3x3 conv's
forward, dgrad, wgrad (+ bias grad) through dll.ops.conv3x3's native kernels
(kpd_conv3x3_forward / kpd_conv3x3_backward, csrc/conv3_grad.hip) at the
heatmap conv 2 shape -- N ROIs x 256 -> 256 channels, 56x56 (reference
heatmap_head.py:55-66; the gradients autograd computes in Trainer.train,
trainer.py:263,272).  One JSON line:

  per pass: mean ms (HIP events, after warm-ups), algorithmic TFLOP/s
  (2 * N * HW * O * 9C per pass) and its fraction of the dense MFMA peak of
  the dtype the pass issues on: forward / dgrad at 56 x 56 with 64 | 256 -> 256
  channels run split (3 f16 products per MAC on v_mfma_f32_16x16x32_f16 over
  the 57 x 57 bordered layout; 2.5 PF/s, the issued rate beside it), the
  others fp32 (v_mfma_f32_16x16x4_f32; 157.3 TF/s); beside it the same
  passes through torch's own conv (F.conv2d + autograd on this GPU, MIOpen),
  and max |d| of the native gradients vs torch fp64 on a slice.

    python tools/bench_conv3_grad.py [--rois 64] [--iters 20]
"""
import argparse
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "keypoint-detection_amd"))

PEAK_FP32 = 157.3
PEAK_F16 = 2500.0


def timed(fn, iters, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rois", type=int, default=64)
    ap.add_argument("--cin", type=int, default=256)
    ap.add_argument("--cout", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from dll import _native
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    N, C, O, H, W = a.rois, a.cin, a.cout, 56, 56
    x = torch.randn(N, C, H, W, generator=g).to(dev)
    w = (torch.randn(O, C, 3, 3, generator=g) * (1.0 / (9 * C) ** 0.5)).to(dev)
    b = torch.randn(O, generator=g).to(dev)
    gy = torch.randn(N, O, H, W, generator=g).to(dev)
    flop = 2.0 * N * H * W * O * 9 * C

    res = {"shape": {"rois": N, "cin": C, "cout": O, "h": H, "w": W}, "flop_per_pass": flop,
           "peak_tflops": {"fp32": PEAK_FP32, "f16": PEAK_F16}, "peak_note": "dense MFMA peaks, MI355X_MICROARCH.md"}
    nat = {
        "forward": lambda: _native.conv3x3_forward(x, w, b),
        "dgrad": lambda: _native.conv3x3_backward(x, w, gy, need_x=True, need_w=False, need_b=False),
        "wgrad": lambda: _native.conv3x3_backward(x, w, gy, need_x=False, need_w=True, need_b=False),
        "bias_grad": lambda: _native.conv3x3_backward(x, w, gy, need_x=False, need_w=False, need_b=True),
    }
    import os
    generic = bool(os.environ.get("KPD_K6_GENERIC")) and bool(os.environ.get("KPD_DIAG_LIB"))
    split = {"forward": H == W == 56 and C in (64, 256) and O == 256,
             "dgrad": H == W == 56 and O in (64, 256) and C == 256}
    for k, fn in nat.items():
        ms = timed(fn, a.iters)
        e = {"ms": round(ms, 4)}
        if k != "bias_grad":
            tf = flop / (ms * 1e-3) / 1e12
            if split.get(k) and not generic:
                e.update(tflops=round(tf, 2), path="split_f16x3", frac=round(tf / PEAK_F16, 4),
                         issued_tflops=round(3 * tf * 57 * 57 / (56 * 56), 2),
                         issued_frac=round(3 * tf * 57 * 57 / (56 * 56) / PEAK_F16, 4))
            else:
                e.update(tflops=round(tf, 2), path="fp32", frac=round(tf / PEAK_FP32, 4))
        res[f"native_{k}"] = e
    res["native_forward_plus_backward_ms"] = round(sum(res[f"native_{k}"]["ms"] for k in nat), 4)
    # torch's own conv on this GPU (MIOpen) for the same passes
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)

    def t_fwd():
        with torch.no_grad():
            return F.conv2d(x, w, b, padding=1)

    def t_bwd():
        y = F.conv2d(xr, wr, br, padding=1)
        return torch.autograd.grad(y, (xr, wr, br), gy)
    ms_f = timed(t_fwd, a.iters)
    ms_fb = timed(t_bwd, a.iters)
    res["torch_forward"] = {"ms": round(ms_f, 4), "tflops": round(flop / (ms_f * 1e-3) / 1e12, 2)}
    res["torch_forward_plus_backward"] = {"ms": round(ms_fb, 4),
                                          "tflops": round(3 * flop / (ms_fb * 1e-3) / 1e12, 2)}
    # numerics on a slice vs fp64 autograd
    n2 = min(N, 2)
    x64, w64, b64 = x[:n2].double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    y64 = F.conv2d(x64, w64, b64, padding=1)
    gx64, gw64, gb64 = torch.autograd.grad(y64, (x64, w64, b64), gy[:n2].double())
    y = _native.conv3x3_forward(x[:n2], w, b)
    gx, gw, gb = _native.conv3x3_backward(x[:n2], w, gy[:n2], need_x=True, need_w=True, need_b=True)
    y64, gx64, gw64, gb64 = (t.detach() for t in (y64, gx64, gw64, gb64))
    res["max_abs_d_vs_fp64"] = {"y": float((y.double() - y64).abs().max()), "gx": float((gx.double() - gx64).abs().max()),
                                "gw": float((gw.double() - gw64).abs().max()), "gb": float((gb.double() - gb64).abs().max()),
                                "images": n2}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
