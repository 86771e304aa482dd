#!/usr/bin/env python3
"""Golden vectors for the data-side rows, produced by
the REFERENCE's own code in this container:

* `generate_target_heatmap` (dll/models/heatmap_head.py:163-224);
* `Trainer._calculate_validation_metrics` (dll/training/trainer.py:384-429),
  called unbound on a stub carrying `config.pck_thresholds`;
* `OptimizedKeypointsDataset` label parsing / person filtering / target
  generation / sample dict (dll/data/dataloader.py:220-427) and
  `efficient_collate_fn` (:432-560), called on an instance made with
  `object.__new__` (no directory scan, no image decode).

dataloader.py imports cv2 and torchvision.transforms at module level; neither
is installed.  The methods exercised here never touch them, so empty
import-only placeholder modules are registered whose every attribute access
raises -- no OpenCV or torchvision behaviour is imitated.  The reference's
package __init__ files are skipped (namespace packages), bytecode is off.

    python -B tests/golden/make_data_golden.py   -> tests/golden/data.npz
"""
from __future__ import annotations

import sys
import tempfile
import types
from pathlib import Path

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import tv_shim  # noqa: E402
from data_cases import LABEL_CASES, COLLATE_BATCHES, heatmap_cases, metric_cases  # noqa: E402

OUT = ROOT / "tests" / "golden" / "data.npz"


class _ImportOnly(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        raise RuntimeError(f"{self.__name__}.{name} is not available in this container")


def import_reference():
    tv_shim.install()
    for name in ("cv2", "torchvision.transforms", "torchvision.transforms.functional"):
        sys.modules[name] = _ImportOnly(name)
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
    for sub in ("", ".models", ".data", ".utils", ".training"):
        m = types.ModuleType("dll" + sub)
        m.__path__ = [str(REF / "dll" / sub.strip(".")) if sub else str(REF / "dll")]
        sys.modules["dll" + sub] = m
    from dll.models.heatmap_head import generate_target_heatmap
    from dll.training.trainer import Trainer
    from dll.data import dataloader as dl
    return generate_target_heatmap, Trainer, dl


def main():
    gen, Trainer, dl = import_reference()
    data = {}
    # --- target heatmaps
    for i, (kp, size, sigma) in enumerate(heatmap_cases()):
        data[f"hm_kp{i}"] = kp.numpy()
        data[f"hm_meta{i}"] = np.array([size[0], size[1], sigma], np.float64)
        data[f"hm_out{i}"] = gen(kp.clone(), size, sigma).numpy()
    data["hm_n"] = np.array(len(heatmap_cases()), np.int32)
    # --- validation metrics
    thresholds = [0.002, 0.05, 0.2]
    stub = types.SimpleNamespace(config=types.SimpleNamespace(pck_thresholds=thresholds))
    stub._get_default_metrics = types.MethodType(Trainer._get_default_metrics, stub)
    for i, (pred, gt, vis) in enumerate(metric_cases()):
        m = Trainer._calculate_validation_metrics(stub, {"keypoints": pred}, {"keypoints": gt, "visibilities": vis})
        data[f"met_pred{i}"], data[f"met_gt{i}"], data[f"met_vis{i}"] = pred.numpy(), gt.numpy(), vis.numpy()
        data[f"met_out{i}"] = np.array([m["avg_ADE"]] + [m[f"pck_{t}"] for t in thresholds], np.float64)
    data["met_n"] = np.array(len(metric_cases()), np.int32)
    # --- label parsing, filtering, targets, sample dicts, collate
    ds = object.__new__(dl.OptimizedKeypointsDataset)
    ds.num_keypoints, ds.max_persons, ds.heatmap_size = 17, 10, (56, 56)
    ds.enable_caching, ds._annotation_cache = False, None
    samples = {}
    with tempfile.TemporaryDirectory() as td:
        for name, text in LABEL_CASES.items():
            p = Path(td) / f"{name}.txt"
            p.write_text(text)
            ann = ds._parse_label_file_vectorized(p)
            data[f"lab_{name}_parsed_kp"] = ann.keypoints.numpy()
            data[f"lab_{name}_parsed_vis"] = ann.visibilities.numpy()
            data[f"lab_{name}_parsed_cls"] = ann.classes.numpy()
            data[f"lab_{name}_parsed_box"] = ann.bboxes[0].numpy()
            ann = ds._filter_valid_persons(ann)
            if ann.num_persons > ds.max_persons:
                ann = ann.truncate(ds.max_persons)
            heat = ds._generate_training_targets(ann)
            image = torch.full((1, 8, 8), float(len(samples)))      # stands in for the transformed image
            s = ds._create_sample_dict(image, ann, heat, Path(f"{name}.jpg"), (640, 480))
            samples[name] = s
            data[f"lab_{name}_kp"] = s["keypoints"].numpy()
            data[f"lab_{name}_vis"] = s["visibilities"].numpy()
            data[f"lab_{name}_box"] = s["bboxes"].numpy()
            data[f"lab_{name}_heat"] = s["heatmaps"].numpy()
            data[f"lab_{name}_np"] = np.array(s["num_persons"], np.int64)
    for bi, names in enumerate(COLLATE_BATCHES):
        out = dl.efficient_collate_fn([samples[n] for n in names])
        for k in ("image", "heatmaps", "visibilities", "num_persons", "keypoints"):
            data[f"col{bi}_{k}"] = out[k].numpy()
        data[f"col{bi}_bboxes"] = out["bboxes"][0].numpy()
        data[f"col{bi}_paths"] = np.array(out["img_path"])
    data["col_n"] = np.array(len(COLLATE_BATCHES), np.int32)
    np.savez_compressed(OUT, **data)
    print("wrote", OUT, len(data), "arrays")


if __name__ == "__main__":
    main()
