#!/usr/bin/env python3
"""CPU numerics probe: heatmap conv 2 (256 -> 256, 3x3,
56x56) as Winograd F(2x2, 3x3) on the split operands, against the direct
split conv the GPU runs, both against an fp64 reference -- then carried
through conv 3 + final 1x1 + sigmoid + soft-argmax to the heatmap / keypoint
tolerances (5e-5 / 1e-5).

Split emulation (both schemes): operand x * 2^a -> hi = f16(x), lo =
f16(x - hi); weights likewise; products lo.hi + hi.hi + hi.lo are exact in
fp32 and summed here in fp64 then rounded to fp32 (the MFMA sums in fp32:
this emulation is slightly MORE accurate than the hardware for both schemes).
Winograd: V = B^T d B (fp32), U = G g G^T (fp64 at pack time, then split),
M = sum_c U V (split products), Y = A^T M A (fp32).

    python tests/winograd_probe.py [--rois 4]      (analysis script, not collected by pytest)
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keypoint-detection_amd")]


def split(x, bound):
    """x (fp32 array) scaled by 2^a (a from the bound, as split_exp_of) -> hi, lo as float64 of f16 values, scale."""
    u = bound * 1.0078125
    e = np.frexp(u)[1] if u > 0 else -100
    a = min(max(14 - int(e), -100), 100)
    xs = (x.astype(np.float32) * np.float32(2.0 ** a)).astype(np.float32)
    hi = xs.astype(np.float16)
    lo = (xs - hi.astype(np.float32)).astype(np.float16)
    return hi.astype(np.float64), lo.astype(np.float64), 2.0 ** a


def split_matmul(a_hi, a_lo, b_hi, b_lo):
    """lo.hi + hi.hi + hi.lo, summed in fp64, rounded to fp32 (per output)."""
    return (a_lo @ b_hi + a_hi @ b_hi + a_hi @ b_lo).astype(np.float32)


def direct_split(x, w, b):
    """x [C][H][W] fp32, w [O][C][3][3]: the direct 3x3 (padding 1) with split products."""
    C, H, W = x.shape
    xp = np.zeros((C, H + 2, W + 2), np.float32)
    xp[:, 1:-1, 1:-1] = x
    cols = np.stack([xp[:, dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)], 1)   # C,9,H,W
    A = cols.reshape(C * 9, H * W).T                                  # HW x 9C
    Bm = w.reshape(w.shape[0], C * 9).T                                # 9C x O
    ah, al, sa = split(A, np.abs(x).max())
    bh, bl, sb = split(Bm, np.abs(w).max())
    y = split_matmul(ah, al, bh, bl) / np.float32(sa * sb)
    return (y + b).T.reshape(-1, H, W).astype(np.float32)


BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64)
G = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64)
AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64)


def winograd_split(x, w, b):
    C, H, W = x.shape
    O = w.shape[0]
    th, tw = H // 2, W // 2
    xp = np.zeros((C, H + 2, W + 2), np.float32)
    xp[:, 1:-1, 1:-1] = x
    # input tiles d [C][th][tw][4][4] -> V = B^T d B in fp32
    d = np.stack([np.stack([xp[:, 2 * i:2 * i + 4, 2 * j:2 * j + 4] for j in range(tw)], 1) for i in range(th)], 1)
    V = np.einsum("ab,ctsbd,ed->ctsae", BT.astype(np.float32), d, BT.astype(np.float32)).astype(np.float32)
    U = np.einsum("ab,ocbd,ed->ocae", G, w.astype(np.float64), G)          # [O][C][4][4] fp64
    Vt = V.transpose(3, 4, 1, 2, 0).reshape(16, th * tw, C)                  # [xi][tiles][C]
    Ut = U.transpose(2, 3, 1, 0).reshape(16, C, O)                          # [xi][C][O]
    vh, vl, sv = split(Vt, np.abs(Vt).max())
    uh, ul, su = split(Ut.astype(np.float32), np.abs(Ut).max())
    M = np.stack([split_matmul(vh[k], vl[k], uh[k], ul[k]) for k in range(16)]) / np.float32(sv * su)
    M = M.reshape(4, 4, th, tw, O).astype(np.float32)
    Y = np.einsum("ab,bdtso,ed->otase", AT.astype(np.float32), M, AT.astype(np.float32)).astype(np.float32)
    return (Y.reshape(O, H, W) + b[:, None, None]).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rois", type=int, default=4)
    a = ap.parse_args()
    from oracle import kpd_oracle as O
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict
    sd = synthetic_state_dict(MultiPersonKeypointModel(ModelConfig(), TrainingConfig()).state_dict(), seed=0)
    img = synthetic_images(a.rois, 3, 256, 192, seed=1234)
    boxes = synthetic_boxes(a.rois, 1, seed=1235)
    ref = O.forward(sd, {"image": img, "bboxes": boxes}, return_debug=True)
    feats, _ = O.select_top_k(ref["_feat0"], sd)
    H = "heatmap_head."

    def fold(conv, bn):
        g, bb, m, v = (sd[f"{H}{bn}.{k}"].double() for k in ("weight", "bias", "running_mean", "running_var"))
        s = g / torch.sqrt(v + 1e-5)
        return (sd[f"{H}{conv}.weight"].double() * s[:, None, None, None]).numpy(), \
            ((sd[f"{H}{conv}.bias"].double() - m) * s + bb).numpy()
    w1, b1 = fold("deconv_layers.0", "deconv_layers.1")
    w2, b2 = fold("deconv_layers.4", "deconv_layers.5")
    w3, b3 = fold("final_layer.0", "final_layer.1")
    wf = sd[H + "final_layer.3.weight"].double().numpy()[:, :, 0, 0]
    bf = sd[H + "final_layer.3.bias"].double().numpy()

    def tail(h2):   # conv 3 + BN + ReLU, final 1x1, sigmoid, soft-argmax (fp64)
        t = torch.from_numpy(np.maximum(h2, 0)).double()[None]
        h3 = F.relu(F.conv2d(t, torch.from_numpy(w3), torch.from_numpy(b3), padding=1))
        hm = torch.sigmoid(torch.einsum("kc,nchw->nkhw", torch.from_numpy(wf), h3) + torch.from_numpy(bf)[None, :, None, None])
        p = torch.softmax(hm.flatten(2), -1).view_as(hm)
        xs = torch.arange(56, dtype=torch.float64) / 55
        kx = (p.sum(2) * xs).sum(-1)
        ky = (p.sum(3) * xs).sum(-1)
        return hm[0].numpy(), torch.stack([kx, ky], -1)[0].numpy()

    rows = []
    for r in range(a.rois):
        roi = O.extract_roi_features(feats[r:r + 1], boxes[r, 0])
        # the attention-weighted input of conv 1 (heatmap_head.py:94-102, as oracle.heatmap_head)
        cw = torch.sigmoid(O._fc2(roi.mean(dim=(2, 3)), sd, H + "channel_attention.")
                           + O._fc2(roi.amax(dim=(2, 3)), sd, H + "channel_attention."))
        x = roi * cw[:, :, None, None]
        sa = torch.cat([x.mean(dim=1, keepdim=True), x.amax(dim=1, keepdim=True)], dim=1)
        x = x * torch.sigmoid(F.conv2d(sa, sd[H + "spatial_attention.conv.weight"],
                                       sd[H + "spatial_attention.conv.bias"], 1, 3))
        x1 = x[0].double().numpy()
        h1 = np.maximum(F.conv2d(torch.from_numpy(x1)[None], torch.from_numpy(w1), torch.from_numpy(b1), padding=1)[0]
                        .numpy(), 0).astype(np.float32)
        y64 = F.conv2d(torch.from_numpy(h1.astype(np.float64))[None], torch.from_numpy(w2), torch.from_numpy(b2),
                       padding=1)[0].numpy()
        yd = direct_split(h1, w2, b2)
        yw = winograd_split(h1, w2, b2)
        hm64, k64 = tail(y64)
        hmd, kd = tail(yd.astype(np.float64))
        hmw, kw = tail(yw.astype(np.float64))
        sc = np.abs(y64).max()
        rows.append((np.abs(yd - y64).max() / sc, np.abs(yw - y64).max() / sc, np.abs(hmd - hm64).max(),
                     np.abs(hmw - hm64).max(), np.abs(kd - k64).max(), np.abs(kw - k64).max()))
        print("roi %d: conv2 max rel err direct %.2e winograd %.2e | heatmap %.2e / %.2e | kpt %.2e / %.2e" %
              ((r,) + rows[-1]), flush=True)
    m = np.array(rows).max(0)
    print("max over ROIs: conv2 rel err direct %.2e winograd %.2e; heatmap %.2e / %.2e (tol 5e-5); "
          "keypoints %.2e / %.2e (tol 1e-5)" % tuple(m))


if __name__ == "__main__":
    main()
