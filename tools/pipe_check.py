#!/usr/bin/env python3
"""Bit-identity of a multi-stream forward (KPD_PIPE / KPD_PIPE_PRI as set in
the environment) against the single-stream forward, C2 shape.
    KPD_PIPE=3 python tools/pipe_check.py [streams]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keypoint-detection_amd")]
from dll.configs import ModelConfig, TrainingConfig  # noqa: E402
from dll.models import MultiPersonKeypointModel  # noqa: E402
from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = torch.device("cuda", 0)
m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision="split")
m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
m = m.to(dev).eval()
img = synthetic_images(64, 3, 256, 192, seed=1234, device=dev)
boxes = synthetic_boxes(64, 1, seed=1235, device=dev)
with torch.no_grad():
    m.streams = 1
    a = m({"image": img, "bboxes": boxes})
    a = {k: v.clone() for k, v in a.items() if torch.is_tensor(v)}
    m.streams = S
    for _ in range(3):
        b = m({"image": img, "bboxes": boxes})
        for k in a:
            assert torch.equal(a[k], b[k]), k
print("pipe_check ok", S)
