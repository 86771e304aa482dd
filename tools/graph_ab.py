#!/usr/bin/env python3
"""Eager vs hipGraph-replayed forwards (kpd_plan_set_graphs) at the bench
shape, no stage timing: images/s of each, alternated.  GPU only."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "keypoint-detection_amd")]


def main():
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision="split", streams=1)
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
    m = m.to(dev).eval()
    batch = {"image": synthetic_images(B, 3, 256, 192, seed=1234).to(dev),
             "bboxes": synthetic_boxes(B, 1, seed=1235).to(dev)}
    plan = m.native_plan(dev)
    with torch.no_grad():
        for _ in range(30):
            m(batch)
        for rep in range(3):
            for g in (False, True):
                plan.set_graphs(g)
                for _ in range(3):
                    m(batch)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(40):
                    m(batch)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / 40
                print(f"B={B} graphs={int(g)} {dt * 1e3:.4f} ms/forward {B / dt:.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
