"""Pin the CPU oracle against golden vectors produced by the reference's own
code (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import kpd_oracle as O


def _np(p):
    return np.load(p, allow_pickle=False)


def test_weights_fingerprint(golden_dir, model_sd):
    from dll.models.synthetic import weights_checksum
    g = _np(golden_dir / "weights_fingerprint.npz")
    assert sorted(model_sd.keys()) == list(g["keys"])   # product state-dict names == reference names
    assert weights_checksum(model_sd) == pytest.approx(float(g["checksum"]), rel=1e-12)


def test_forward_main(golden_dir, model_sd):
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    g = _np(golden_dir / "forward_main.npz")
    img = synthetic_images(2, 3, 256, 192, seed=1234)
    assert float(img.double().sum()) == pytest.approx(float(g["image_sum"]), rel=1e-12)
    boxes = torch.from_numpy(g["boxes"])
    out = O.forward(model_sd, {"image": img, "bboxes": boxes}, return_debug=True)
    f = out["_feat0"]
    np.testing.assert_allclose(f.mean(dim=(2, 3)).numpy(), g["feat0_chan_mean"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(f.amax(dim=(2, 3)).numpy(), g["feat0_chan_max"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(f[:, :, 60:64, 40:44].numpy(), g["feat0_slice"], rtol=1e-5, atol=1e-5)
    assert (out["_topk"].numpy() == g["topk"]).all()
    np.testing.assert_allclose(out["keypoints"].numpy(), g["keypoints"], atol=1e-5)
    assert (out["visibilities"].numpy() == g["visibilities"]).all()
    hm = out["heatmap"]
    np.testing.assert_allclose(hm.double().sum(dim=(3, 4)).numpy(), g["heatmap_sum"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(hm.amax(dim=(3, 4)).numpy(), g["heatmap_max"], atol=1e-5)
    np.testing.assert_allclose(hm[0, 0].numpy(), g["heatmap_b0p0"], atol=1e-5)


def test_forward_dummy_and_empty(golden_dir, model_sd):
    from dll.models.synthetic import synthetic_images
    img = synthetic_images(2, 3, 256, 192, seed=1234)
    g = _np(golden_dir / "forward_dummy.npz")
    out = O.forward(model_sd, {"image": img, "bboxes": torch.from_numpy(g["boxes"])})
    np.testing.assert_allclose(out["keypoints"].numpy(), g["keypoints"], atol=1e-5)
    assert (out["visibilities"].numpy() == g["visibilities"]).all()
    np.testing.assert_allclose(out["heatmap"].double().sum(dim=(3, 4)).numpy(), g["heatmap_sum"], rtol=1e-5,
                               atol=1e-3)
    e = _np(golden_dir / "forward_empty.npz")
    out = O.forward(model_sd, {"image": img, "bboxes": torch.zeros(2, 0, 4)})
    assert tuple(out["keypoints"].shape) == tuple(e["kshape"])
    assert tuple(out["visibilities"].shape) == tuple(e["vshape"])
    assert tuple(out["heatmap"].shape) == tuple(e["hshape"])


def test_forward_gray_list(golden_dir, model_sd_gray):
    from dll.models.synthetic import synthetic_images
    g = _np(golden_dir / "forward_gray_list.npz")
    img = synthetic_images(1, 1, 224, 224, seed=99)
    out = O.forward(model_sd_gray, {"image": img, "bboxes": [torch.from_numpy(g["boxes"])]})
    np.testing.assert_allclose(out["keypoints"].numpy(), g["keypoints"], atol=1e-5)
    assert (out["visibilities"].numpy() == g["visibilities"]).all()
    np.testing.assert_allclose(out["heatmap"].double().sum(dim=(3, 4)).numpy(), g["heatmap_sum"], rtol=1e-5,
                               atol=1e-3)


def test_nms_and_iou(golden_dir):
    g = _np(golden_dir / "nms.npz")
    i = 0
    while f"c{i}_boxes" in g:
        mo = int(g[f"c{i}_max_out"])
        keep = O.nms(torch.from_numpy(g[f"c{i}_boxes"]), torch.from_numpy(g[f"c{i}_scores"]),
                     float(g[f"c{i}_thr"]), None if mo < 0 else mo)
        assert keep.tolist() == g[f"c{i}_keep"].tolist(), f"case {i}"
        i += 1
    assert i == 5
    b = _np(golden_dir / "box_iou.npz")
    iou = O.box_iou_cxcywh(torch.from_numpy(b["b1"]), torch.from_numpy(b["b2"]))
    np.testing.assert_array_equal(iou.numpy(), b["iou"])


def test_heatmap_head_and_decoders(golden_dir, model_sd):
    g = _np(golden_dir / "heatmap_head.npz")
    x = torch.from_numpy(g["x"].astype(np.float32))
    hm = O.heatmap_head(x, model_sd)
    np.testing.assert_allclose(hm.double().sum(dim=(2, 3)).numpy(), g["heat_sum"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(hm[:, :, 20:24, 30:34].numpy(), g["heat_slice"], atol=1e-5)
    hm_ref = hm
    kp, vis = O.decode_heatmap(hm_ref)
    np.testing.assert_allclose(kp.numpy(), g["model_kpts"], atol=1e-5)
    assert (vis.numpy() == g["model_vis"]).all()


def test_keypoint_head(golden_dir):
    from dll.configs import KeypointHeadConfig
    from dll.models.keypoint_head import KEYPOINT_HEAD
    from dll.models.synthetic import synthetic_state_dict, weights_checksum
    g = _np(golden_dir / "keypoint_head.npz")
    kh = KEYPOINT_HEAD(KeypointHeadConfig(height=56, width=56))
    sd = synthetic_state_dict(kh.state_dict(), seed=3)
    assert weights_checksum(sd) == pytest.approx(float(g["checksum"]), rel=1e-12)
    x = torch.randn(2, 128, 56, 56, generator=torch.Generator().manual_seed(11))
    kp, vis = O.keypoint_head(x, {"kh." + k: v for k, v in sd.items()}, "kh.")
    np.testing.assert_allclose(kp.numpy(), g["keypoints"], atol=2e-6)
    np.testing.assert_allclose(vis.numpy(), g["visibility"], atol=2e-6)


def test_roi_align_vectorized_matches_loop():
    g = torch.Generator().manual_seed(3)
    feat = torch.randn(8, 20, 16, generator=g)
    for box in [(1.3, 2.2, 9.7, 17.9), (0.0, 0.0, 16.0, 20.0), (15.5, 19.5, 16.0, 20.0), (3.0, 3.0, 3.2, 3.1),
                (0.0, 0.0, 0.0, 0.0)]:
        a = O.roi_align_one(feat, *[torch.tensor(v) for v in box], out=7)
        b = O.roi_align_loop(feat, *box, out=7)
        np.testing.assert_allclose(a.numpy(), b.numpy(), atol=2e-6)
