#!/usr/bin/env python3
"""Phase timeline of cbody_kernel (KPD_STAMPS): per workgroup (= image) the
s_memrealtime stamps (100 MHz) written at the kernel's phase boundaries --
start, then per block (features.5..11): XS built, rounds done, SE done,
project done, and the end of features.12.  Prints the median duration of each
phase over the images and the launch span.  GPU only.
    KPD_STAMPS=1 python3 tools/stamps_cbody.py
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "keypoint-detection_amd")]
os.environ.setdefault("KPD_STAMPS", "1")


def main():
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict
    dev = torch.device("cuda:0")
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision="split", streams=1)
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
    m = m.to(dev).eval()
    B = int(os.environ.get("PROBE_BATCH", "64"))
    batch = {"image": synthetic_images(B, 3, 256, 192, seed=1234).to(dev),
             "bboxes": synthetic_boxes(B, 1, seed=1235).to(dev)}
    plan = m.native_plan(dev)
    with torch.no_grad():
        for _ in range(6):
            m(batch)
    torch.cuda.synchronize()
    buf = plan.debug_buffer("stamps_cbody")
    st = buf.view(torch.int64).cpu().numpy().reshape(B, 128)
    rounds = st[:, 64:]
    st = st[:, :64]
    used = [c for c in range(64) if (st[:, c] != 0).all()]
    t = st[:, used].astype(np.float64) * 0.01   # us
    t0 = t[:, 0].min()
    t -= t0
    ph = np.diff(t, axis=1)
    names = ["load X + xs"]
    for i in range(5, 12):
        names += [f"f{i} rounds", f"f{i} se", f"f{i} proj", f"f{i} tap+xs"]
    names[-1] = "f12"
    ru = [c for c in range(64) if (rounds[:, c] != 0).all()]
    rt = rounds[:, ru].astype(np.float64) * 0.01 - t0
    print("round stamps (expand done, depthwise done), median us from kernel start:")
    print("  " + " ".join(f"{v:.1f}" for v in np.median(rt, axis=0)))
    print(f"workgroups {B}: start p50 {np.median(t[:, 0]):.1f} max {t[:, 0].max():.1f} us; "
          f"end p50 {np.median(t[:, -1]):.1f} max {t[:, -1].max():.1f} us")
    for j in range(ph.shape[1]):
        nm = names[j] if j < len(names) else f"phase {j}"
        print(f"  {nm:12s} med {np.median(ph[:, j]):7.2f} max {ph[:, j].max():7.2f} us")


if __name__ == "__main__":
    main()
