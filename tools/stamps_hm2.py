#!/usr/bin/env python3
"""Phase stamps of the split hmconv tiles (hmconv_kernel, KPD_STAMPS, diagnostic
build): per workgroup the prologue (chunk 0 window + first weights landed), the
K loop and the epilogue (stores drained).  GPU only:

    KPD_DIAG_LIB=1 KPD_STAMPS=1 python3 tools/stamps_hm2.py [names] [split|mixed] [--dual B P]

names: comma list of stamp buffers (default stamps_hm2): stamps_hm1/2/3 (the
heatmap convs; C2 model, 64 images x 1 box), stamps_kh1/2/3 (the KEYPOINT_HEAD
convs: [ResidualBlock 1 | visibility] + downsample, ResidualBlock 2 +
downsample, the regression 3x3) -- those need --dual B P (dual-head model, B
images x P given boxes; stamp buffer space bounds B*P to ~400)."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "keypoint-detection_amd")]
os.environ.setdefault("KPD_STAMPS", "1")


def report(plan, name, prec):
    st = plan.debug_buffer(name).view(torch.int64).cpu().numpy().reshape(-1, 8)
    st = st[st[:, 0] != 0]
    t = st[:, [0, 1, 2, 3]].astype(np.float64) * 0.01
    t -= t[:, 0].min()
    start, end = t[:, 0], t[:, 3]
    ph = np.diff(t, axis=1)
    print(f"{name} {prec}: wgs={len(st)} span={end.max():.1f}us KT={st[0, 5]} starts p10/p50/p90 {np.percentile(start, 10):.1f}/"
          f"{np.median(start):.1f}/{np.percentile(start, 90):.1f}")
    print("phases med (prologue, K loop, epilogue) = " + " ".join(f"{v:.2f}" for v in np.median(ph, axis=0))
          + f"  K loop per step {np.median(ph[:, 1]) / st[0, 5]:.3f}us  wg med {np.median(end - start):.2f}")
    if (st[:, 7] > st[:, 6]).all():   # shader-clock stamps around the K loop (hmconv)
        ghz = (st[:, 7] - st[:, 6]).astype(np.float64) / np.maximum(ph[:, 1] * 1e3, 1e-9)
        print(f"K-loop shader clock GHz p10/p50/p90 {np.percentile(ghz, 10):.3f}/{np.median(ghz):.3f}/{np.percentile(ghz, 90):.3f}")


def main():
    from dll.configs import KeypointHeadConfig, ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict
    dev = torch.device("cuda:0")
    args = [a for a in sys.argv[1:]]
    dual = None
    if "--dual" in args:
        i = args.index("--dual")
        dual = (int(args[i + 1]), int(args[i + 2]))
        del args[i:i + 3]
    names = (args[0] if args else "stamps_hm2").split(",")
    prec = args[1] if len(args) > 1 else "split"
    if dual:
        m = MultiPersonKeypointModel(ModelConfig(keypoint_head=KeypointHeadConfig(height=56, width=56)),
                                     TrainingConfig(), precision=prec, dual_head=True, streams=1)
        B, P = dual
    else:
        m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision=prec, streams=1)
        B, P = 64, 1
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
    m = m.to(dev).eval()
    batch = {"image": synthetic_images(B, 3, 256, 192, seed=1234).to(dev),
             "bboxes": synthetic_boxes(B, P, seed=1235).to(dev)}
    plan = m.native_plan(dev)
    with torch.no_grad():
        for _ in range(4):
            m(batch)
    torch.cuda.synchronize()
    for name in names:
        report(plan, name, prec)


if __name__ == "__main__":
    main()
