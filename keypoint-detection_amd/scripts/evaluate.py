#!/usr/bin/env python3
"""Real-data PCK / ADE evaluation on a YOLO-pose split, end to end on the
device: decode (host) -> ITransform + target heatmaps (kpd_preprocess,
kpd_target_heatmaps) -> collate -> MultiPersonKeypointModel with the
ground-truth boxes (kpd_forward) -> ADE / PCK (kpd_keypoint_metrics).

The metrics are the reference's validation metrics
(dll/training/trainer.py:384-429), averaged over batches as its
validate_epoch does (:305-395); the loss terms are not computed (training is
out of scope).

    python scripts/evaluate.py --config configs/default_config.yaml \
        --model best_model.pth --dataset-dir data/ --split val --batch-size 32
"""
from __future__ import annotations

import argparse
import json
import sys
from collections import defaultdict
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))

from dll.data import create_optimized_dataloader  # noqa: E402
from dll.utils import calculate_validation_metrics  # noqa: E402
from predict import load_config, load_model, setup_logging  # noqa: E402


def evaluate(model, loader, pck_thresholds):
    sums, n = defaultdict(float), 0
    with torch.no_grad():
        for batch in loader:
            out = model({"image": batch["image"], "bboxes": batch["bboxes"]})
            for k, v in calculate_validation_metrics(out, batch, pck_thresholds).items():
                sums[k] += v
            n += 1
    return {k: v / max(n, 1) for k, v in sums.items()}, n


def main(argv=None):
    ap = argparse.ArgumentParser(description="Evaluate keypoint PCK / ADE on a dataset split")
    ap.add_argument("--config", required=True)
    ap.add_argument("--model", required=True, help="checkpoint path, or 'synthetic'")
    ap.add_argument("--dataset-dir", required=True)
    ap.add_argument("--split", default="val")
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--precision", default="split", choices=["split", "fp32", "mixed"])
    args = ap.parse_args(argv)
    setup_logging()
    cfg = load_config(args.config)
    device = torch.device(args.device)
    bcfg = cfg["model"]["backbone"]
    thresholds = cfg.get("training", {}).get("pck_thresholds", [0.002, 0.05, 0.2])
    loader = create_optimized_dataloader(args.dataset_dir, batch_size=args.batch_size, split=args.split,
                                         img_size=bcfg["input_size"], grayscale=bcfg.get("in_channels", 3) == 1,
                                         device=device)
    model = load_model(args.model, cfg, device, args.precision)
    metrics, n = evaluate(model, loader, thresholds)
    print(json.dumps({"split": args.split, "batches": n, **metrics}))
    return metrics


if __name__ == "__main__":
    main()
