"""Data-side rows: YOLO-pose label parsing, person
filtering, sample dicts and collate against goldens made by the reference's
own methods (tests/golden/make_data_golden.py); target heatmaps and the
validation metrics on the device against the reference's outputs.

Tolerances: parsing / filtering / collate bit-exact; target heatmaps within
4e-9 absolute (the peak value is ~0.018, one fp32 ulp there is 1.9e-9: the
kernel table's exp and sum may round differently from torch's CPU kernels);
ADE / PCK within 1e-6 relative (double accumulation vs torch fp32).
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
from data_cases import COLLATE_BATCHES, LABEL_CASES, heatmap_cases, metric_cases  # noqa: E402

gpu = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(golden_dir / "data.npz", allow_pickle=False)


def _bare_dataset(device="cpu"):
    from dll.data.dataloader import OptimizedKeypointsDataset
    ds = object.__new__(OptimizedKeypointsDataset)
    ds.num_keypoints, ds.max_persons, ds.heatmap_size = 17, 10, (56, 56)
    ds.enable_caching, ds._annotation_cache = False, None
    ds.device = torch.device(device)
    return ds


def _write_dataset(root: Path, names, size=(96, 128)):
    from PIL import Image
    rng = np.random.default_rng(1)
    (root / "val" / "images").mkdir(parents=True)
    (root / "val" / "labels").mkdir(parents=True)
    for n in names:
        img = rng.integers(0, 256, (*size, 3), dtype=np.uint8)
        Image.fromarray(img).save(root / "val" / "images" / f"{n}.png")
        (root / "val" / "labels" / f"{n}.txt").write_text(LABEL_CASES[n])


def test_label_parsing_and_filtering_match_reference(tmp_path, g):
    ds = _bare_dataset()
    for name, text in LABEL_CASES.items():
        p = tmp_path / f"{name}.txt"
        p.write_text(text)
        ann = ds._parse_label_file_vectorized(p)
        assert np.array_equal(ann.keypoints.numpy(), g[f"lab_{name}_parsed_kp"]), name
        assert np.array_equal(ann.visibilities.numpy(), g[f"lab_{name}_parsed_vis"]), name
        assert np.array_equal(ann.classes.numpy(), g[f"lab_{name}_parsed_cls"]), name
        assert np.array_equal(ann.bboxes[0].numpy(), g[f"lab_{name}_parsed_box"]), name
        ann = ds._filter_valid_persons(ann)
        if ann.num_persons > ds.max_persons:
            ann = ann.truncate(ds.max_persons)
        assert ann.num_persons == int(g[f"lab_{name}_np"]), name
        assert np.array_equal(ann.keypoints.numpy(), g[f"lab_{name}_kp"]), name
        assert np.array_equal(ann.visibilities.numpy(), g[f"lab_{name}_vis"]), name
        assert np.array_equal(ann.bboxes[0].numpy(), g[f"lab_{name}_box"]), name


def _golden_sample(g, name, idx):
    return {"image": torch.full((1, 8, 8), float(idx)), "heatmaps": torch.from_numpy(g[f"lab_{name}_heat"]),
            "visibilities": torch.from_numpy(g[f"lab_{name}_vis"]), "bboxes": torch.from_numpy(g[f"lab_{name}_box"]),
            "keypoints": torch.from_numpy(g[f"lab_{name}_kp"]), "num_persons": int(g[f"lab_{name}_np"]),
            "img_path": f"{name}.jpg", "orig_size": (640, 480)}


def test_collate_matches_reference(g):
    from dll.data import efficient_collate_fn
    order = {n: i for i, n in enumerate(LABEL_CASES)}
    for bi, names in enumerate(COLLATE_BATCHES):
        out = efficient_collate_fn([_golden_sample(g, n, order[n]) for n in names])
        for k in ("image", "heatmaps", "visibilities", "num_persons", "keypoints"):
            assert np.array_equal(out[k].numpy(), g[f"col{bi}_{k}"]), (bi, k)
        assert np.array_equal(out["bboxes"][0].numpy(), g[f"col{bi}_bboxes"])
        assert out["img_path"] == list(g[f"col{bi}_paths"])


def test_collate_all_empty_branch():
    from dll.data import efficient_collate_fn
    s = {"image": torch.zeros(1, 4, 4), "num_persons": 0, "img_path": "a", "orig_size": (4, 4)}
    out = efficient_collate_fn([s, dict(s, img_path="b")])
    assert out["heatmaps"].shape == (2, 1, 17, 56, 56) and out["bboxes"][0].shape == (2, 1, 4)
    assert out["num_persons"].dtype == torch.long and out["img_path"] == ["a", "b"]


def test_dataset_files_and_adaptive_sampler(tmp_path):
    from dll.data import AdaptiveBatchSampler, OptimizedKeypointsDataset
    from dll.data.dataloader import KeypointDatasetError
    names = ["two", "one", "many", "empty", "blank"]
    _write_dataset(tmp_path, names)
    (tmp_path / "val" / "images" / "orphan.png").write_bytes(
        (tmp_path / "val" / "images" / "one.png").read_bytes())      # no label: skipped
    ds = OptimizedKeypointsDataset(str(tmp_path), split="val", img_size=64, grayscale=True, device="cpu")
    assert [p.stem for p in ds.img_files] == sorted(names)
    assert ds._load_and_process_image(ds.img_files[0]).orig_size == (128, 96)
    sampler = AdaptiveBatchSampler(ds, batch_size=2, max_persons_per_batch=50)
    batches = list(sampler)
    assert sorted(i for b in batches for i in b) == list(range(len(names))) and all(len(b) <= 2 for b in batches)
    with pytest.raises(KeypointDatasetError):
        OptimizedKeypointsDataset(str(tmp_path), split="train", device="cpu")


def test_default_metrics_shape_mismatch_needs_no_device():
    from dll.utils import calculate_validation_metrics
    pred, gt, vis = metric_cases()[1]
    assert calculate_validation_metrics({"keypoints": pred}, {"keypoints": gt, "visibilities": vis}) == \
        {"avg_ADE": 0.0, "pck_0.002": 0.0, "pck_0.05": 0.0, "pck_0.2": 0.0}


@gpu
def test_gpu_target_heatmaps_vs_reference(g):
    from dll.models.heatmap_head import generate_target_heatmap
    for i, (kp, size, sigma) in enumerate(heatmap_cases()):
        assert np.array_equal(kp.numpy(), g[f"hm_kp{i}"])
        out = generate_target_heatmap(kp.to(DEV), size, sigma).cpu().numpy()
        want = g[f"hm_out{i}"]
        assert out.shape == want.shape, i
        assert np.abs(out - want).max() <= 4e-9, (i, np.abs(out - want).max())
        assert np.array_equal(out == 0, want == 0), i                  # identical support


@gpu
def test_gpu_metrics_vs_reference(g):
    from dll.utils import calculate_validation_metrics
    for i, (pred, gt, vis) in enumerate(metric_cases()):
        m = calculate_validation_metrics({"keypoints": pred.to(DEV)},
                                         {"keypoints": gt.to(DEV), "visibilities": vis.to(DEV)})
        got = np.array([m["avg_ADE"], m["pck_0.002"], m["pck_0.05"], m["pck_0.2"]])
        np.testing.assert_allclose(got, g[f"met_out{i}"], rtol=1e-6, atol=1e-7)


@gpu
def test_gpu_dataset_and_loader_end_to_end(tmp_path, g):
    """Images decoded from disk, ITransform + targets on the device, collate;
    then the model on the collated batch and the metrics."""
    from dll.configs import BackboneConfig, ModelConfig, TrainingConfig
    from dll.data import create_optimized_dataloader
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_state_dict
    from dll.utils import calculate_validation_metrics
    from oracle import preprocess_oracle as O
    from PIL import Image
    names = ["two", "one", "ragged", "invisible"]
    _write_dataset(tmp_path, names)
    dl = create_optimized_dataloader(str(tmp_path), batch_size=4, num_workers=2, split="val", img_size=64,
                                     grayscale=True, device=DEV)
    ds = dl.dataset
    for i, n in enumerate(sorted(names)):
        s = ds[i]
        assert s["image"].is_cuda and s["heatmaps"].is_cuda and s["image"].shape == (1, 64, 64)
        img = np.asarray(Image.open(ds.img_files[i]).convert("L"))
        assert np.array_equal(s["image"].cpu().numpy(), O.itransform_gray(img, 64, 1.5))
        assert np.array_equal(s["keypoints"].numpy(), g[f"lab_{n}_kp"])
        assert np.abs(s["heatmaps"].cpu().numpy() - g[f"lab_{n}_heat"]).max() <= 4e-9
    batch = next(iter(dl))
    assert batch["image"].shape == (4, 1, 64, 64) and batch["bboxes"][0].shape == (4, 1, 4)
    m = MultiPersonKeypointModel(ModelConfig(backbone=BackboneConfig(in_channels=1, input_size=64)), TrainingConfig())
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m({"image": batch["image"], "bboxes": batch["bboxes"]})
    met = calculate_validation_metrics(out, batch)
    assert set(met) == {"avg_ADE", "pck_0.002", "pck_0.05", "pck_0.2"}
    assert 0.0 < met["avg_ADE"] < 1.5 and 0.0 <= met["pck_0.2"] <= 1.0


@gpu
def test_gpu_evaluate_cli(tmp_path, capsys):
    """scripts/evaluate.py on a small YOLO-pose split (grayscale 224 config)."""
    import json
    from conftest import PKG
    sys.path.insert(0, str(PKG / "scripts"))
    import evaluate
    _write_dataset(tmp_path, ["two", "one", "ragged"], size=(120, 90))
    m = evaluate.main(["--config", str(PKG / "configs" / "default_config.yaml"), "--model", "synthetic",
                       "--dataset-dir", str(tmp_path), "--split", "val", "--batch-size", "2"])
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["batches"] == 2 and set(m) == {"avg_ADE", "pck_0.002", "pck_0.05", "pck_0.2"}
