#!/usr/bin/env python3
"""Per-workgroup phase timelines of the SE-block kernels (KPD_STAMPS).

Runs single-stream forwards at the bench shape with the diagnostic stamps on
and prints, per launch: workgroups, launch span, the workgroups alive at once
(max / median), and the median duration of each phase of a workgroup.  The
stamps are s_memrealtime ticks (100 MHz, 10 ns).  GPU only.
    KPD_STAMPS=1 python3 tools/stamps_probe.py
    KPD_STAMPS=1 PROBE_PERSONS=5 python3 tools/stamps_probe.py   (dual head: roi_kh_kernel)
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
    # PROBE_PERSONS > 1: the dual-head model in split precision (roi_kh_kernel's stamps)
    P = int(os.environ.get("PROBE_PERSONS", "1"))
    dual = P > 1
    prec = "split" if dual else "mixed"
    if dual:
        from dll.configs import KeypointHeadConfig
        m = MultiPersonKeypointModel(ModelConfig(keypoint_head=KeypointHeadConfig(height=56, width=56)),
                                     TrainingConfig(), precision=prec, dual_head=True, streams=1)
    else:
        m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision=prec, streams=1)
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
    m = m.to(dev).eval()
    B = int(os.environ.get("PROBE_BATCH", "64"))
    batch = {"image": synthetic_images(B, 3, 256, 192, seed=1234).to(dev),
             "bboxes": synthetic_boxes(B, P, seed=1235).to(dev)}
    plan = m.native_plan(dev)
    with torch.no_grad():
        for _ in range(4):
            m(batch)
    torch.cuda.synchronize()
    names = [f"stamps_{k}_{i}" for i in range(11) for k in ("exdw", "seproj")] + ["stamps_latchain_0", "stamps_fir23_0"] + [f"stamps_fir_{i}" for i in range(11)] + ["stamps_roi_0", "stamps_roikh_0"]
    for name in names:
        try:
            buf = plan.debug_buffer(name)
        except Exception:
            continue
        st = buf.view(torch.int64).cpu().numpy().reshape(-1, 8)
        st = st[(st != 0).any(axis=1)]   # rows of workgroups this launch did not have (sized for the largest grid)
        if len(st) == 0:
            continue
        used = [c for c in range(8) if (st[:, c] != 0).all()]
        t = st[:, used].astype(np.float64) * 10.0 / 1000.0   # us
        t0 = t[:, 0].min()
        t -= t0
        start, end = t[:, 0], t[:, -1]
        ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
        ev = ev[np.argsort(ev[:, 0], kind="stable")]
        alive = np.cumsum(ev[:, 1])
        ph = np.diff(t, axis=1)
        print(f"{name:18s} wgs={len(st):5d} span={end.max():7.1f}us alive max={int(alive.max()):5d} "
              f"wg dur med={np.median(end - start):6.1f} max={np.max(end - start):6.1f} "
              f"start p50={np.median(start):6.1f} p90={np.percentile(start, 90):6.1f} | phases med "
              + " ".join(f"{v:5.1f}" for v in np.median(ph, axis=0)))


if __name__ == "__main__":
    main()
