#!/usr/bin/env python3
"""Phase stamps of fpn0x_kernel (KPD_STAMPS): per workgroup the prologue
(first K-tile landed), the K loop, the statistics exchange and the stores
(drained), grouped by K-tile count (position classes with 1, 2 or 4 lateral-1
tap groups).  GPU only:  KPD_STAMPS=1 python3 tools/stamps_fpn0x.py"""
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
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision=sys.argv[1] if len(sys.argv) > 1 else "split", streams=1)
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
    m = m.to(dev).eval()
    B = 64
    batch = {"image": synthetic_images(B, 3, 256, 192, seed=1234).to(dev),
             "bboxes": synthetic_boxes(B, 1, seed=1235).to(dev)}
    plan = m.native_plan(dev)
    with torch.no_grad():
        for _ in range(4):
            m(batch)
    torch.cuda.synchronize()
    st = plan.debug_buffer("stamps_fpn0x").view(torch.int64).cpu().numpy().reshape(-1, 8)
    kt = st[:, 5]
    cyc = st[:, 4].astype(np.float64)                            # K loop in shader cycles
    t = st[:, [0, 1, 2, 6, 7, 3]].astype(np.float64) * 0.01      # us
    t -= t[:, 0].min()
    start, end = t[:, 0], t[:, 5]
    print(f"wgs={len(st)} span={end.max():.1f}us  starts p10/p50/p90 = {np.percentile(start, 10):.1f}/"
          f"{np.median(start):.1f}/{np.percentile(start, 90):.1f}")
    for k in sorted(set(kt.tolist())):
        sel = kt == k
        ph = np.diff(t[sel], axis=1)
        print(f"KT={k:2d} n={sel.sum():5d}  wg med={np.median(end[sel] - start[sel]):6.2f}us  phases med "
              f"(prologue, K loop, next-tile setup+issue, epilogue math+exchange, stats store) = " + " ".join(f"{v:5.2f}" for v in np.median(ph, axis=0))
              + f"  K-loop per K-tile {np.median(ph[:, 1]) / k:.3f}us  clock {np.median(cyc[sel] / (ph[:, 1] * 1e3)):.3f} GHz")
    # concurrency
    ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    print("max alive", int(np.cumsum(ev[:, 1]).max()))


if __name__ == "__main__":
    main()
