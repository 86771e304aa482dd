"""HIP path vs the oracle / reference goldens, through the C ABI (libkpd.so).

Tolerances (stated per BASELINE.md / SURVEY §8(d)):
  precision="fp32" and "split" (fp32-accurate f16x3 products):
                     max|dkpt| <= 1e-5, heatmaps atol 5e-5, top-k indices and
                     visibility classes identical.
  precision="mixed": max|dkpt| <= 1e-3, heatmaps atol 3e-2, top-k identical
                     (backbone stays fp32), visibility flips reported and
                     bounded (<= 2% of keypoints).
"""
import numpy as np
import pytest
import torch

from oracle import kpd_oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _np(p):
    return np.load(p, allow_pickle=False)


def _model(sd, precision="fp32", in_channels=3, full_level0=False):
    from dll.configs import BackboneConfig, ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    m = MultiPersonKeypointModel(ModelConfig(backbone=BackboneConfig(in_channels=in_channels)), TrainingConfig(),
                                 precision=precision)
    m.load_state_dict(sd)
    m.full_level0 = full_level0    # tests reading the "feat0" debug copy store the whole map
    return m.to(DEV).eval()


def _nchw_feat(plan, B, Hf, Wf):
    f = plan.debug_buffer("feat0").view(B, Hf, Wf, 128)
    return f.permute(0, 3, 1, 2).cpu()


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_forward_main_vs_golden(golden_dir, model_sd, precision):
    from dll.models.synthetic import synthetic_images
    g = _np(golden_dir / "forward_main.npz")
    m = _model(model_sd, precision, full_level0=True)
    img = synthetic_images(2, 3, 256, 192, seed=1234, device=DEV)
    boxes = torch.from_numpy(g["boxes"]).to(DEV)
    with torch.no_grad():
        out = m({"image": img, "bboxes": boxes})
    torch.cuda.synchronize()
    plan = m.native_plan(DEV)
    f = _nchw_feat(plan, 2, 128, 96)
    np.testing.assert_allclose(f.mean(dim=(2, 3)).numpy(), g["feat0_chan_mean"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(f.amax(dim=(2, 3)).numpy(), g["feat0_chan_max"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(f[:, :, 60:64, 40:44].numpy(), g["feat0_slice"], rtol=1e-4, atol=1e-4)
    scores = plan.debug_buffer("scores").view(2, 128).cpu()
    np.testing.assert_allclose(scores.numpy(), g["scores"], atol=1e-6)
    topk = torch.topk(scores, 64, dim=1).indices
    assert (topk.numpy() == g["topk"]).all()
    kp = out["keypoints"].cpu().numpy()
    vis = out["visibilities"].cpu().numpy()
    hm = out["heatmap"].cpu()
    assert kp.shape == g["keypoints"].shape and vis.shape == g["visibilities"].shape
    if precision != "mixed":
        np.testing.assert_allclose(kp, g["keypoints"], atol=1e-5)
        assert (vis == g["visibilities"]).all()
        np.testing.assert_allclose(hm[0, 0].numpy(), g["heatmap_b0p0"], atol=5e-5)
        np.testing.assert_allclose(hm.amax(dim=(3, 4)).numpy(), g["heatmap_max"], atol=5e-5)
    else:
        np.testing.assert_allclose(kp, g["keypoints"], atol=1e-3)
        flips = int((vis != g["visibilities"]).any(axis=-1).sum())
        assert flips <= 0.02 * vis[..., 0].size
        np.testing.assert_allclose(hm[0, 0].numpy(), g["heatmap_b0p0"], atol=3e-2)
    # compacted + padded slot of the zero box (image 1, slot 2) is all zero
    assert not out["keypoints"][1, 2].any() and not out["visibilities"][1, 2].any()


@pytest.mark.parametrize("precision", ["split", "mixed"])
def test_level0_footprint_stores(model_sd, precision):
    """With caller boxes FPN level 0 is stored only where the ROI aligns read
    it (fpn0x_kernel footprint rectangles): every output equals the
    full-map forward's bit for bit -- boxes at the borders, tiny and
    full-image boxes, zero boxes mid-list, an image with no valid box and one
    past the box list -- and the default forward has no "feat0" debug copy."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    img = synthetic_images(5, 3, 256, 192, seed=71, device=DEV)
    boxes = synthetic_boxes(4, 3, seed=72, device=DEV)
    boxes[0, 1] = torch.tensor([0.02, 0.98, 0.05, 0.03])      # corner, sub-pixel
    boxes[1, 0] = torch.tensor([0.5, 0.5, 1.0, 1.0])          # whole image
    boxes[1, 2] = 0.0                                          # zero box mid-list
    boxes[2] = 0.0                                             # no valid box: dummy person
    boxes[3, 2] = torch.tensor([0.99, 0.5, 0.4, 0.2])         # right border
    outs = []
    for full in (True, False):
        m = _model(model_sd, precision, full_level0=full)
        with torch.no_grad():
            outs.append(m({"image": img, "bboxes": [boxes]}))
        if not full:
            with pytest.raises(ValueError):
                m.native_plan(DEV).debug_buffer("feat0")
    a, b = outs
    for k in ("keypoints", "visibilities", "heatmap"):
        assert torch.equal(a[k], b[k]), k


def test_forward_dummy_empty(golden_dir, model_sd):
    from dll.models.synthetic import synthetic_images
    m = _model(model_sd)
    img = synthetic_images(2, 3, 256, 192, seed=1234, device=DEV)
    g = _np(golden_dir / "forward_dummy.npz")
    with torch.no_grad():
        out = m({"image": img, "bboxes": torch.from_numpy(g["boxes"]).to(DEV)})
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), g["keypoints"], atol=1e-5)
    assert (out["visibilities"].cpu().numpy() == g["visibilities"]).all()
    np.testing.assert_allclose(out["heatmap"].double().sum(dim=(3, 4)).cpu().numpy(), g["heatmap_sum"],
                               rtol=1e-4, atol=2e-2)
    e = _np(golden_dir / "forward_empty.npz")
    with torch.no_grad():
        out = m({"image": img, "bboxes": torch.zeros(2, 0, 4, device=DEV)})
    assert tuple(out["visibilities"].shape) == tuple(e["vshape"])
    assert tuple(out["keypoints"].shape) == tuple(e["kshape"])
    with torch.no_grad():
        out = m({"image": img, "bboxes": None})
    assert tuple(out["heatmap"].shape) == tuple(e["hshape"])


def test_forward_gray_list(golden_dir, model_sd_gray):
    from dll.models.synthetic import synthetic_images
    g = _np(golden_dir / "forward_gray_list.npz")
    m = _model(model_sd_gray, in_channels=1)
    img = synthetic_images(1, 1, 224, 224, seed=99, device=DEV)
    with torch.no_grad():
        out = m({"image": img, "bboxes": [torch.from_numpy(g["boxes"]).to(DEV)]})
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), g["keypoints"], atol=1e-5)
    assert (out["visibilities"].cpu().numpy() == g["visibilities"]).all()
    scores = m.native_plan(DEV).debug_buffer("scores").view(1, 128).cpu()
    np.testing.assert_allclose(scores.numpy(), g["scores"], atol=1e-6)


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_odd_size_vs_oracle(model_sd, precision):
    """H/2*W/2 not a multiple of the conv M-tile -> separate channel-stats path
    and a partial last M-tile (zero-filled by the buffer range check); boxes
    touching the border and degenerate (sub-pixel) boxes."""
    from dll.models.synthetic import synthetic_images
    img = synthetic_images(2, 3, 200, 152, seed=5)
    boxes = torch.tensor([[[0.5, 0.5, 0.9, 0.95], [0.02, 0.03, 0.1, 0.1], [0.98, 0.97, 0.3, 0.4]],
                          [[0.3, 0.6, 0.001, 0.002], [0.5, 0.5, 1.0, 1.0], [0.7, 0.2, 0.4, 0.3]]])
    ref = O.forward(model_sd, {"image": img, "bboxes": boxes}, return_debug=True)
    m = _model(model_sd, precision, full_level0=True)
    with torch.no_grad():
        out = m({"image": img.to(DEV), "bboxes": boxes.to(DEV)})
    plan = m.native_plan(DEV)
    f = _nchw_feat(plan, 2, 100, 76)
    np.testing.assert_allclose(f.numpy(), ref["_feat0"].numpy(), rtol=1e-5, atol=1e-5)
    if precision != "mixed":
        np.testing.assert_allclose(out["keypoints"].cpu().numpy(), ref["keypoints"].numpy(), atol=1e-5)
        assert torch.equal(out["visibilities"].cpu(), ref["visibilities"])
        np.testing.assert_allclose(out["heatmap"].cpu().numpy(), ref["heatmap"].numpy(), atol=5e-5)
    else:
        np.testing.assert_allclose(out["keypoints"].cpu().numpy(), ref["keypoints"].numpy(), atol=1e-3)
        np.testing.assert_allclose(out["heatmap"].cpu().numpy(), ref["heatmap"].numpy(), atol=3e-2)


@pytest.mark.parametrize("precision", ["split"])
def test_large_map_lateral_fallback(model_sd, precision):
    """480x384: lateral 3 is 15 x 12 = 180 pixels, more than the fused lateral
    chain takes (lateral_chain_ok: <= 128), so the split path runs the
    per-level lateral convs and split_rows for lateral 1 and the stem tap (the
    max-based scale, not the chain's bound)."""
    from dll.models.synthetic import synthetic_images
    img = synthetic_images(1, 3, 480, 384, seed=9)
    boxes = torch.tensor([[[0.45, 0.55, 0.4, 0.7]]])
    ref = O.forward(model_sd, {"image": img, "bboxes": boxes}, return_debug=True)
    m = _model(model_sd, precision, full_level0=True)
    with torch.no_grad():
        out = m({"image": img.to(DEV), "bboxes": boxes.to(DEV)})
    plan = m.native_plan(DEV)
    f = _nchw_feat(plan, 1, 240, 192)
    np.testing.assert_allclose(f.numpy(), ref["_feat0"].numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), ref["keypoints"].numpy(), atol=1e-5)
    assert torch.equal(out["visibilities"].cpu(), ref["visibilities"])
    np.testing.assert_allclose(out["heatmap"].cpu().numpy(), ref["heatmap"].numpy(), atol=5e-5)


def test_roi_features_vs_oracle(model_sd):
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    img = synthetic_images(2, 3, 256, 192, seed=21)
    boxes = synthetic_boxes(2, 2, seed=22)
    m = _model(model_sd, full_level0=True)
    with torch.no_grad():
        m({"image": img.to(DEV), "bboxes": boxes.to(DEV)})
    plan = m.native_plan(DEV)
    roi = plan.debug_buffer("roi").view(4, 56, 56, 64).permute(0, 3, 1, 2).cpu()
    feat = _nchw_feat(plan, 2, 128, 96)
    feats, _ = O.select_top_k(feat, model_sd)   # same features -> isolates roi_align + gather
    for r in range(4):
        b, p = divmod(r, 2)
        want = O.extract_roi_features(feats[b:b + 1], boxes[b, p])[0]
        np.testing.assert_allclose(roi[r].numpy(), want.numpy(), atol=2e-5)


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_batch_independence(model_sd, precision):
    """Images are independent: a batch equals its images run one at a time,
    bit for bit in every precision (the split FPN scale is per image)."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    img = synthetic_images(6, 3, 256, 192, seed=31, device=DEV)
    img[3] *= 4.0                            # one image with a larger dynamic range
    boxes = synthetic_boxes(6, 2, seed=32, device=DEV)
    m = _model(model_sd, precision)
    with torch.no_grad():
        full = m({"image": img, "bboxes": boxes})
        for i in (0, 3, 5):
            one = m({"image": img[i:i + 1], "bboxes": boxes[i:i + 1]})
            assert torch.equal(one["keypoints"][0], full["keypoints"][i])
            assert torch.equal(one["heatmap"][0], full["heatmap"][i])
    assert torch.isfinite(full["heatmap"]).all()
    ref = O.forward(model_sd, {"image": img[3:4].cpu(), "bboxes": boxes[3:4].cpu()})
    tol_k, tol_h = (1e-5, 5e-5) if precision != "mixed" else (1e-3, 3e-2)
    np.testing.assert_allclose(full["keypoints"][3:4].cpu().numpy(), ref["keypoints"].numpy(), atol=tol_k)
    np.testing.assert_allclose(full["heatmap"][3:4].cpu().numpy(), ref["heatmap"].numpy(), atol=tol_h)


@pytest.mark.parametrize("precision", ["split", "mixed"])
def test_bench_batch_properties(model_sd, precision):
    """BASELINE C2 shape (B=64, 256x192, 1 box), the bench's precisions:
    size-independent properties + every image against the oracle."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    img = synthetic_images(64, 3, 256, 192, seed=1234)
    boxes = synthetic_boxes(64, 1, seed=1235)
    m = _model(model_sd, precision)
    with torch.no_grad():
        out = m({"image": img.to(DEV), "bboxes": boxes.to(DEV)})
    kp = out["keypoints"].cpu()
    vis = out["visibilities"].cpu()
    assert kp.shape == (64, 1, 1, 17, 2) and ((kp >= 0) & (kp <= 1)).all()
    assert torch.equal(vis.sum(-1), torch.ones(64, 1, 1, 17))
    # every image of the bench batch against the oracle (the CPU restatement
    # takes ~1 s for 64 images); mixed tolerances as in the module docstring
    ref = O.forward(model_sd, {"image": img, "bboxes": boxes}, return_debug=True)
    if precision == "mixed":
        np.testing.assert_allclose(kp.numpy(), ref["keypoints"].numpy(), atol=1e-3)
        flips = int((vis != ref["visibilities"]).any(dim=-1).sum())
        assert flips <= 0.02 * 64 * 17
    else:
        np.testing.assert_allclose(kp.numpy(), ref["keypoints"].numpy(), atol=1e-5)
        assert torch.equal(vis, ref["visibilities"])
        np.testing.assert_allclose(out["heatmap"].cpu().numpy(), ref["heatmap"].numpy(), atol=5e-5)
    topk = m.native_plan(DEV).debug_buffer("scores").view(64, 128).cpu().topk(64, dim=1).indices
    assert torch.equal(topk, ref["_topk"])


def test_nms_gpu_vs_golden(golden_dir):
    from dll.configs import PersonDetectionConfig
    from dll.models import PERSON_HEAD
    ph = PERSON_HEAD(PersonDetectionConfig())
    g = _np(golden_dir / "nms.npz")
    i = 0
    while f"c{i}_boxes" in g:
        mo = int(g[f"c{i}_max_out"])
        sc = g[f"c{i}_scores"]
        keep = ph.non_max_suppression(torch.from_numpy(g[f"c{i}_boxes"]).to(DEV), torch.from_numpy(sc).to(DEV),
                                      float(g[f"c{i}_thr"]), None if mo < 0 else mo).tolist()
        ref = g[f"c{i}_keep"].tolist()
        if keep != ref:
            # torch's CPU sort(descending) is unstable, so the reference's order
            # among exactly tied scores is unspecified; ours is lower-index-first.
            # Accept only a permutation among equal scores.
            assert [sc[k] for k in keep] == [sc[k] for k in ref], f"case {i}"
            assert sorted(keep) == sorted(ref), f"case {i}"
        i += 1


def test_nms_prefix_paths():
    """nms_reg_kernel's prefix fast path (the top ~1024 candidates by score)
    and its two ways out: a prefix that runs dry before max_output (a dense
    cluster of 2,000 overlapping boxes on top: fallback to the full pass),
    ties at the prefix threshold beyond the list (3,000 equal scores), and
    max_output = 0 (keep everything).  Oracle: the reference's greedy NMS
    restated (oracle.kpd_oracle.nms); tied scores may keep a different index
    of equal score (torch's CPU sort is unstable), so those cases compare the
    kept scores and boxes."""
    from dll import _native
    g = torch.Generator().manual_seed(7)
    n = 5000
    boxes = torch.rand(n, 4, generator=g) * torch.tensor([1.0, 1.0, 0.2, 0.2]) + torch.tensor([0.0, 0.0, 0.02, 0.02])
    scores = torch.randperm(n, generator=g).float() / n * 0.5 + 0.3       # distinct scores
    cl = torch.arange(2000)
    boxes[cl] = torch.tensor([0.5, 0.5, 0.3, 0.3]) + 1e-3 * torch.rand(2000, 4, generator=g)
    scores[cl] = 0.9 + 0.05 * torch.arange(2000, 0, -1).float() / 2000   # the cluster ranks first
    for mo, thr in ((5, 0.3), (40, 0.3), (0, 0.5)):
        got = _native.nms(boxes.to(DEV), scores.to(DEV), thr, mo).cpu()
        ref = O.nms(boxes, scores, thr, mo if mo > 0 else None)
        assert torch.equal(got, ref), (mo, thr)
    tied = scores.clone()
    tied[2000:2500] = 0.8 + 0.1 * torch.arange(500, 0, -1).float() / 500   # 500 distinct on top
    tied[2500:5000] = 0.75                                                # then 2,500 ties
    tied[cl] = 0.2 + 0.05 * torch.arange(2000, 0, -1).float() / 2000     # the cluster last
    got = _native.nms(boxes.to(DEV), tied.to(DEV), 0.3, 5).cpu()           # kept within the 500
    assert torch.equal(got, O.nms(boxes, tied, 0.3, 5))
    got = _native.nms(boxes.to(DEV), tied.to(DEV), 0.3, 600).cpu()         # runs into the ties
    ref = O.nms(boxes, tied, 0.3, 600)
    assert got.numel() == ref.numel()
    assert torch.equal(tied[got], tied[ref])
    # ties beyond the LDS list when the prefix holds every alive candidate
    # (ADVICE r4): all 3,000 scores equal -> the list re-compacts to the keys
    # above tau (none) and must fall back to the full pass, not stop empty
    b3 = boxes[:3000].contiguous()
    eq = torch.full((3000,), 0.6)
    for mo in (5, 0):
        got = _native.nms(b3.to(DEV), eq.to(DEV), 0.3, mo).cpu()
        ref = O.nms(b3, eq, 0.3, mo if mo > 0 else None, stable=True)
        assert got.numel() > 0 and torch.equal(got, ref), mo
    # 500 distinct scores above 2,600 ties at the lowest score: the kept boxes
    # must run on into the ties
    b4 = boxes[:3100].contiguous()
    s4 = torch.full((3100,), 0.4)
    s4[:500] = 0.5 + 0.4 * torch.randperm(500, generator=g).float() / 500
    got = _native.nms(b4.to(DEV), s4.to(DEV), 0.3, 600).cpu()
    ref = O.nms(b4, s4, 0.3, 600, stable=True)
    assert torch.equal(got, ref)
    assert (s4[got] == 0.4).any()
    # the tie order is implementation-defined (the reference sorts with an
    # unstable sort): whatever order the kernel picks, its kept set must be a
    # valid greedy-NMS result
    _assert_greedy_nms(b3, eq, 0.3, _native.nms(b3.to(DEV), eq.to(DEV), 0.3, 0).cpu(), complete=True)
    _assert_greedy_nms(b4, s4, 0.3, got, complete=False)
    _assert_greedy_nms(boxes, tied, 0.3, _native.nms(boxes.to(DEV), tied.to(DEV), 0.3, 0).cpu(), complete=True)


def _assert_greedy_nms(boxes, scores, thr, keep, complete):
    """keep is a greedy NMS result under SOME order of tied scores: scores
    non-increasing along keep, no kept pair above the IoU threshold, and every
    box not kept that ranks above the last kept score (every box when the run
    was not cut by max_output) overlaps a kept box scored at or above it."""
    ks = scores[keep]
    assert bool((ks[1:] <= ks[:-1]).all())
    iou = O.box_iou_cxcywh(boxes[keep], boxes[keep])
    iou.fill_diagonal_(0)
    assert float(iou.max()) <= thr
    dropped = torch.ones(len(boxes), dtype=torch.bool)
    dropped[keep] = False
    if not complete:
        dropped &= scores > ks[-1]
    idx = dropped.nonzero().flatten()
    if idx.numel():
        cover = (O.box_iou_cxcywh(boxes[idx], boxes[keep]) > thr) & (ks[None, :] >= scores[idx][:, None])
        assert bool(cover.any(dim=1).all())


def _dual_model(precision="fp32"):
    from dll.configs import KeypointHeadConfig, ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_state_dict
    m = MultiPersonKeypointModel(ModelConfig(keypoint_head=KeypointHeadConfig(height=56, width=56)),
                                 TrainingConfig(), precision=precision, dual_head=True)
    sd = synthetic_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    return m.to(DEV).eval(), sd


def test_dual_head_vs_oracle():
    """KEYPOINT_HEAD on 128-channel ROI features (§8 a11): native vs the oracle
    restatement (itself pinned to the reference module's goldens)."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    m, sd = _dual_model()
    img = synthetic_images(2, 3, 256, 192, seed=41)
    boxes = synthetic_boxes(2, 3, seed=42)
    boxes[1, 0] = 0.0
    with torch.no_grad():
        out = m({"image": img.to(DEV), "bboxes": boxes.to(DEV)})
    ref = O.forward(sd, {"image": img, "bboxes": boxes}, dual_head=True)
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), ref["keypoints"].numpy(), atol=1e-5)
    np.testing.assert_allclose(out["kh_keypoints"].cpu().numpy(), ref["kh_keypoints"].numpy(), atol=1e-5)
    np.testing.assert_allclose(out["kh_visibilities"].cpu().numpy(), ref["kh_visibilities"].numpy(), atol=1e-5)


def _check_detections(got_boxes, got_scores, ref_boxes, ref_scores, what):
    """Detected boxes / scores vs the oracle: identical keep sets (the same
    number of kept persons per image, in the same slots), scores to 1e-5,
    boxes to 1e-4."""
    kept_got = (got_scores > 0).sum(dim=1)
    kept_ref = (ref_scores > 0).sum(dim=1)
    assert torch.equal(kept_got, kept_ref), f"{what}: kept counts {kept_got.tolist()} vs {kept_ref.tolist()}"
    np.testing.assert_allclose(got_scores.numpy(), ref_scores.numpy(), atol=1e-5, err_msg=what)
    np.testing.assert_allclose(got_boxes.numpy(), ref_boxes.numpy(), atol=1e-4, err_msg=what)


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_person_detector_glue_vs_oracle(precision):
    """No 'bboxes' -> build-defined detector glue (§8 a10): pooled 1x1 heads,
    anchor decode, threshold, NMS (max 5).  At BASELINE C3's size (B = 256,
    256x192, one stream: the debug copy of FPN level 0 needs a single pass;
    test_c4_rank_shard_bit_identical covers the detector at two streams) in
    every precision, with a dynamic-range
    outlier in the batch.  Nine images are checked twice against the oracle:
    on the GPU's own FPN level 0 (isolates the glue) and on the oracle's FPN
    level 0 computed from the image (the whole detector path, so a split-mode
    level-0 error that moved a threshold or NMS decision fails here), then
    the keypoint stage on the detected boxes."""
    from dll.models.synthetic import synthetic_images
    m, sd = _dual_model(precision)
    B = 256
    img = synthetic_images(B, 3, 256, 192, seed=51, device=DEV)
    img[17] *= 4.0                             # dynamic-range outlier (x25 saturates the
    #                                            class sigmoids into exact ties, whose NMS
    #                                            order the reference's unstable sort leaves open)
    with torch.no_grad():
        out = m(img)                           # plain tensor input: the reference's detector branch
    sel = [0, 1, 17, 63, 64, 127, 128, 200, 255]
    feat = m.native_plan(DEV).debug_buffer("feat0").view(B, 128, 96, 128)[sel].permute(0, 3, 1, 2).cpu()
    got = torch.stack([out["boxes"][i].cpu() for i in sel])
    got_s = out["box_scores"][sel].cpu()
    assert got.shape == (len(sel), 5, 4)
    assert (got_s > 0).any(), "no person detected in the checked images"
    ref_boxes, ref_scores = O.person_detect(feat, sd, 256, 192, 0.3, 0.3, 5)
    _check_detections(got, got_s, ref_boxes, ref_scores, "glue on the GPU's level 0")
    img_c = img[sel].cpu()
    feat_o = O.backbone_level0(img_c, sd)
    ob, os_ = O.person_detect(feat_o, sd, 256, 192, 0.3, 0.3, 5)
    _check_detections(got, got_s, ob, os_, "detector on the oracle's level 0")
    ref = O.forward(sd, {"image": img_c, "bboxes": got}, dual_head=True)
    tol = 1e-5 if precision != "mixed" else 1e-3
    np.testing.assert_allclose(out["keypoints"][sel].cpu().numpy(), ref["keypoints"].numpy(), atol=tol)
    if precision != "mixed":
        assert torch.equal(out["visibilities"][sel].cpu(), ref["visibilities"])
    np.testing.assert_allclose(out["kh_keypoints"][sel].cpu().numpy(), ref["kh_keypoints"].numpy(), atol=tol)


def test_person_detector_unfused_chain_vs_oracle():
    """Level-0 rows too wide for the fused kernel's LDS (over 262 columns) take
    the unfused detector front end (adaptive_pool56_kernel -> 1x1 heads ->
    person_decode_kernel, the chain the fused person_detect_kernel replaces at
    the BASELINE sizes; both pool column sums, then rows): 256 x 576 images
    (level 0: 288 columns), checked against the oracle's glue on the GPU's
    own FPN level 0."""
    from dll.models.synthetic import synthetic_images
    m, sd = _dual_model("split")
    m.full_level0 = True
    B, H, W = 4, 256, 576
    img = synthetic_images(B, 3, H, W, seed=53, device=DEV)
    with torch.no_grad():
        out = m(img)
    feat = m.native_plan(DEV).debug_buffer("feat0").view(B, H // 2, W // 2, 128).permute(0, 3, 1, 2).cpu()
    got = torch.stack([out["boxes"][i].cpu() for i in range(B)])
    got_s = out["box_scores"].cpu()
    assert got.shape == (B, 5, 4)
    assert (got_s > 0).any(), "no person detected"
    ref_boxes, ref_scores = O.person_detect(feat, sd, H, W, 0.3, 0.3, 5)
    _check_detections(got, got_s, ref_boxes, ref_scores, "unfused glue on the GPU's level 0")


def _predict_module():
    import sys
    from conftest import PKG
    if str(PKG / "scripts") not in sys.path:
        sys.path.insert(0, str(PKG / "scripts"))
    import predict
    return predict, PKG


def _cli_image(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 255, (240, 180, 3), dtype=np.uint8)).save(tmp_path / "img.png")
    return tmp_path / "img.png"


@pytest.mark.parametrize("size", [None, "256x192"])
def test_predict_cli(tmp_path, capsys, size):
    """scripts/predict.py end to end at its default precision (split): YAML
    config (grayscale 224, or 256x192 as in BASELINE C1), synthetic weights, a
    PNG and a YOLO label; printout format of the reference.  The printed
    person-0 keypoints are checked against the oracle's forward on the same
    preprocessed image and boxes."""
    predict, PKG = _predict_module()
    png = _cli_image(tmp_path)
    (tmp_path / "img.txt").write_text("0 0.5 0.5 0.4 0.8\n0 0.3 0.4 0.2 0.3\n")
    args = ["--config", str(PKG / "configs" / "default_config.yaml"), "--model", "synthetic",
            "--input", str(png), "--gt", str(tmp_path / "img.txt"), "--output", str(tmp_path / "out")]
    if size:
        args += ["--size", size]
    res = predict.main(args)
    txt = capsys.readouterr().out
    assert "Keypoints shape: (2, 17, 2)" in txt
    assert " 1. nose" in txt and "17. right_ankle" in txt
    model = res["model"]
    assert model.precision == "split"
    H, W = (256, 192) if size else (224, 224)
    transform = predict.make_transform(1, (H, W), DEV)
    from PIL import Image
    x = transform(Image.open(png).convert("RGB")).unsqueeze(0).cpu()
    sd = {k: v.cpu() for k, v in model.state_dict().items()}
    boxes = torch.tensor([[[0.5, 0.5, 0.4, 0.8], [0.3, 0.4, 0.2, 0.3]]])
    ref = O.forward(sd, {"image": x, "bboxes": boxes})
    out = res["results"][0][1]
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), ref["keypoints"].numpy(), atol=1e-5)
    assert torch.equal(out["visibilities"].cpu(), ref["visibilities"])
    k0 = ref["keypoints"][0, 0, 0]
    assert f" 1. {'nose':<15} ({float(k0[0, 0]):.3f}, {float(k0[0, 1]):.3f})" in txt


def test_predict_cli_detector(tmp_path, capsys, caplog):
    """predict.py without --gt: the reference passes
    bboxes=None and prints zeros (scripts/predict.py:99); here the person
    detector supplies the boxes by default.  The detected boxes equal the
    oracle's detector on the same FPN level 0, the printout shows person 0's
    keypoints, and --reference-zeros restores the reference's all-zero output."""
    import logging
    predict, PKG = _predict_module()
    png = _cli_image(tmp_path)
    base = ["--config", str(PKG / "configs" / "default_config.yaml"), "--model", "synthetic",
            "--input", str(png), "--output", str(tmp_path / "out"), "--size", "256x192"]
    with caplog.at_level(logging.INFO):
        res = predict.main(base)
    txt = capsys.readouterr().out
    assert "boxes from person detector" in caplog.text
    model = res["model"]
    out = res["results"][0][1]
    assert out["keypoints"].shape == (1, 5, 1, 17, 2)
    assert "Keypoints shape: (5, 17, 2)" in txt
    feat = model.native_plan(DEV).debug_buffer("feat0").view(1, 128, 96, 128).permute(0, 3, 1, 2).cpu()
    sd = {k: v.cpu() for k, v in model.state_dict().items()}
    ref_boxes, ref_scores = O.person_detect(feat, sd, 256, 192, 0.3, 0.3, 5)
    _check_detections(torch.stack([b.cpu() for b in out["boxes"]]), out["box_scores"].cpu(), ref_boxes, ref_scores,
                      "predict.py detector")
    kept = int((ref_scores > 0).sum())
    if kept:
        k0 = out["keypoints"][0, 0, 0].cpu()
        assert k0.abs().sum() > 0
        assert f" 1. {'nose':<15} ({float(k0[0, 0]):.3f}, {float(k0[0, 1]):.3f})" in txt
    caplog.clear()
    with caplog.at_level(logging.INFO):
        res = predict.main(base + ["--reference-zeros"])
    txt = capsys.readouterr().out
    assert "reference zeros" in caplog.text
    out = res["results"][0][1]
    assert not out["keypoints"].any() and out["keypoints"].shape == (1, 1, 17, 2)
    assert " 1. nose            (0.000, 0.000)" in txt


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_sub_batch_streams_match(model_sd, precision):
    """kpd_forward splits B >= 32 over sub-batch streams: same outputs as one
    stream, bit for bit in every precision (the split FPN scale is per image)."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    img = synthetic_images(48, 3, 256, 192, seed=41, device=DEV)
    boxes = synthetic_boxes(48, 2, seed=42, device=DEV)
    boxes[5, 1] = 0.0                       # a zero box inside the second sub-batch
    outs = []
    for streams in (1, 3):
        m = _model(model_sd, precision)
        m.streams = streams
        with torch.no_grad():
            outs.append(m({"image": img, "bboxes": boxes}))
    a, b = outs
    assert torch.equal(a["keypoints"], b["keypoints"]) and torch.equal(a["heatmap"], b["heatmap"])
    assert torch.equal(a["visibilities"], b["visibilities"])


@pytest.mark.parametrize("streams", [1, 2])
def test_graph_replay_matches_eager(model_sd, streams):
    """kpd_plan_set_graphs: the same call signature runs eagerly, is captured,
    then replays one hipGraph per call -- outputs bit-identical to the eager
    forward at every call, also with new inputs copied into the same buffers
    and with sub-batch streams inside the graph."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    m = _model(model_sd, "split")
    m.streams = streams
    B, P = 32, 2
    img = synthetic_images(B, 3, 256, 192, seed=81, device=DEV)
    boxes = synthetic_boxes(B, P, seed=82, device=DEV)
    with torch.no_grad():
        ref = m({"image": img, "bboxes": boxes})           # eager: the plan is built here
    plan = m.native_plan(DEV)
    kpts = torch.empty(B, P, 1, 17, 2, device=DEV)         # the model's output layouts
    vis = torch.empty(B, P, 1, 17, 3, device=DEV)
    heat = torch.empty(B, P, 17, 56, 56, device=DEV)
    plan.set_graphs(True)
    try:
        for it in range(4):                                 # eager, capture + launch, replay, replay
            kpts.fill_(-1.0)
            heat.fill_(-1.0)
            plan.forward(img, boxes, kpts, vis, heat)
            torch.cuda.synchronize()
            assert torch.equal(kpts, ref["keypoints"]), it
            assert torch.equal(heat, ref["heatmap"]), it
            assert torch.equal(vis, ref["visibilities"]), it
        # new data in the same buffers: the replay computes it
        img2 = synthetic_images(B, 3, 256, 192, seed=83, device=DEV)
        with torch.no_grad():
            ref2 = m({"image": img2, "bboxes": boxes})      # eager (other output buffers)
        img.copy_(img2)
        plan.forward(img, boxes, kpts, vis, heat)
        torch.cuda.synchronize()
        assert torch.equal(kpts, ref2["keypoints"]) and torch.equal(heat, ref2["heatmap"])
        # a larger batch re-carves the workspace: the captured graphs are
        # stale (their kernels hold the old workspace addresses) and the
        # original signature must run eagerly / be captured again
        big = synthetic_images(2 * B, 3, 256, 192, seed=84, device=DEV)
        with torch.no_grad():
            out_big = m({"image": big, "bboxes": torch.cat([boxes, boxes])})
            half = m({"image": big[B:], "bboxes": boxes})
        assert torch.equal(out_big["keypoints"][B:], half["keypoints"])
        for it in range(3):
            kpts.fill_(-1.0)
            heat.fill_(-1.0)
            plan.forward(img, boxes, kpts, vis, heat)
            torch.cuda.synchronize()
            assert torch.equal(kpts, ref2["keypoints"]) and torch.equal(heat, ref2["heatmap"]), it
            assert torch.equal(vis, ref2["visibilities"]), it
    finally:
        plan.set_graphs(False)


def test_graph_capture_failure_recovers(model_sd):
    """An abandoned capture (kpd_plan_set_graphs mode 2 forces it) runs the
    call eagerly with the plan's workspace state restored: the captured
    forward had marked the split-scale slots clean and may have re-carved,
    but none of its work ran.  Outputs stay bit-identical to eager through the
    failed capture, a re-carve, the next (successful) capture and replays."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    m = _model(model_sd, "split")
    B, P = 16, 2
    img = synthetic_images(B, 3, 256, 192, seed=91, device=DEV)
    boxes = synthetic_boxes(B, P, seed=92, device=DEV)
    with torch.no_grad():
        ref = m({"image": img, "bboxes": boxes})
    plan = m.native_plan(DEV)
    kpts = torch.empty(B, P, 1, 17, 2, device=DEV)
    vis = torch.empty(B, P, 1, 17, 3, device=DEV)
    heat = torch.empty(B, P, 17, 56, 56, device=DEV)
    try:
        for it, mode in enumerate((True, "abandon", None, None, "grow", None, None, None)):
            if mode == "abandon":
                plan.set_graphs(True, abandon_next_capture=True)
            if mode == "grow":   # a larger batch re-carves the workspace (stale graphs, fresh zero borders)
                big = synthetic_images(2 * B, 3, 256, 192, seed=93, device=DEV)
                with torch.no_grad():
                    m({"image": big, "bboxes": torch.cat([boxes, boxes])})
                plan.set_graphs(True, abandon_next_capture=True)
            elif mode is True:
                plan.set_graphs(True)
            kpts.fill_(-1.0)
            heat.fill_(-1.0)
            vis.fill_(-1.0)
            plan.forward(img, boxes, kpts, vis, heat)
            torch.cuda.synchronize()
            assert torch.equal(kpts, ref["keypoints"]), it
            assert torch.equal(heat, ref["heatmap"]), it
            assert torch.equal(vis, ref["visibilities"]), it
    finally:
        plan.set_graphs(False)


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_c5_shape_dual_head_vs_oracle(precision):
    """BASELINE config C5's shape at a CPU-checkable batch: 384x288 input
    (FPN0 map 192x144 -> 108 M-tiles per image), 5 boxes per image with zero
    padding slots, heatmap head + KEYPOINT_HEAD."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    m, sd = _dual_model(precision)
    img = synthetic_images(2, 3, 384, 288, seed=51)
    boxes = synthetic_boxes(2, 5, seed=52)
    boxes[0, 3:] = 0.0                     # two padding slots in image 0
    with torch.no_grad():
        out = m({"image": img.to(DEV), "bboxes": boxes.to(DEV)})
    ref = O.forward(sd, {"image": img, "bboxes": boxes}, dual_head=True)
    tol_k, tol_h = (1e-5, 5e-5) if precision != "mixed" else (1e-3, 3e-2)
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), ref["keypoints"].numpy(), atol=tol_k)
    np.testing.assert_allclose(out["heatmap"].cpu().numpy(), ref["heatmap"].numpy(), atol=tol_h)
    if precision != "mixed":
        assert torch.equal(out["visibilities"].cpu(), ref["visibilities"])
    else:   # bf16 heads: visibility class flips bounded as in the module docstring
        flips = (out["visibilities"].cpu() != ref["visibilities"]).any(-1).float().mean().item()
        assert flips <= 0.02
    np.testing.assert_allclose(out["kh_keypoints"].cpu().numpy(), ref["kh_keypoints"].numpy(), atol=tol_k)
    np.testing.assert_allclose(out["kh_visibilities"].cpu().numpy(), ref["kh_visibilities"].numpy(), atol=tol_k)


@pytest.mark.parametrize("precision", ["fp32", "split", "mixed"])
def test_c4_rank_shard_bit_identical(precision):
    """BASELINE C4's per-rank workload on one GPU: rank 3's shard of a
    2048-image batch (shard_range(2048, 8, 3) = 256 images, 256x192), person
    detector + NMS + dual head.  Every image's outputs are bit-identical when
    the same images run as other shards / batch sizes (an 8-rank
    sharded run equals the 1-rank run per image)."""
    from dll.distributed import shard_range
    from dll.models.synthetic import synthetic_images
    a0, b0 = shard_range(2048, 8, 3)
    assert (a0, b0) == (768, 1024)
    m, sd = _dual_model(precision)
    m.streams = 2
    img = synthetic_images(b0 - a0, 3, 256, 192, seed=70 + a0, device=DEV)
    img[17] *= 25.0                           # dynamic-range outlier inside the shard
    with torch.no_grad():
        full = m(img)
        parts = [m(img[a:b]) for a, b in ((0, 37), (37, 38), (38, 160), (160, 256))]
    keys = ("keypoints", "visibilities", "heatmap", "kh_keypoints", "kh_visibilities", "box_scores")
    for k in keys:
        got = torch.cat([p[k] for p in parts], dim=0)
        assert torch.equal(got, full[k]), k
    assert torch.equal(torch.stack([b for p in parts for b in p["boxes"]]), torch.stack(full["boxes"]))
    assert full["keypoints"].shape == (256, 5, 1, 17, 2)
    # images against the oracle on the detected boxes: the first three, both
    # sides of every split boundary and the last one
    sel = [0, 1, 2, 36, 37, 38, 159, 160, 255]
    ref = O.forward(sd, {"image": img[sel].cpu(), "bboxes": torch.stack([full["boxes"][i] for i in sel]).cpu()},
                    dual_head=True)
    tol = 1e-5 if precision != "mixed" else 1e-3
    np.testing.assert_allclose(full["keypoints"][sel].cpu().numpy(), ref["keypoints"].numpy(), atol=tol)
    np.testing.assert_allclose(full["kh_keypoints"][sel].cpu().numpy(), ref["kh_keypoints"].numpy(), atol=tol)


def test_saturated_heatmaps_finite(model_sd):
    """An image scaled x40 drives heatmap logits far into the sigmoid's
    saturation (e^-v overflows): every precision returns finite heatmaps in
    [0, 1] and finite keypoints (the fused mixed-precision sigmoid once gave
    NaN there).  The channel scores saturate too, so top-k ties make the
    oracle comparison ill-posed here; only the invariants are checked."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    img = synthetic_images(2, 3, 256, 192, seed=31, device=DEV) * 40.0
    boxes = synthetic_boxes(2, 2, seed=32, device=DEV)
    for precision in ("fp32", "split", "mixed"):
        m = _model(model_sd, precision)
        with torch.no_grad():
            out = m({"image": img, "bboxes": boxes})
        h = out["heatmap"]
        assert torch.isfinite(h).all() and (h >= 0).all() and (h <= 1).all(), precision
        assert torch.isfinite(out["keypoints"]).all(), precision


@pytest.mark.parametrize("precision", ["split"])
def test_c5_full_rank_share(precision):
    """BASELINE C5's per-GPU share at full size: 256 images (2048 / 8) of
    384x288, 5 given boxes per image, heatmap head + KEYPOINT_HEAD (1,280
    ROIs).  Bit-identity of every output across two different shard splits,
    finite heatmaps in [0, 1], and 5 images against the oracle -- among them
    an image with padding slots (zero boxes mid-list and at the end) and the
    dynamic-range outlier."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    m, sd = _dual_model(precision)
    m.streams = 2
    B = 256
    img = synthetic_images(B, 3, 384, 288, seed=61, device=DEV)
    img[100] *= 4.0                            # larger dynamic range (scores stay untied)
    boxes = synthetic_boxes(B, 5, seed=62, device=DEV)
    boxes[7, 1] = 0.0                          # zero box mid-list: compacted, slot 4 padded
    boxes[7, 3] = 0.0
    boxes[200, 2:] = 0.0                       # trailing padding slots
    with torch.no_grad():
        full = m({"image": img, "bboxes": boxes})
        parts = [m({"image": img[a:b], "bboxes": boxes[a:b]}) for a, b in ((0, 100), (100, 101), (101, 256))]
    keys = ("keypoints", "visibilities", "heatmap", "kh_keypoints", "kh_visibilities")
    for k in keys:
        assert torch.equal(torch.cat([p[k] for p in parts], dim=0), full[k]), k
    h = full["heatmap"]
    assert h.shape == (B, 5, 17, 56, 56)
    assert torch.isfinite(h).all() and (h >= 0).all() and (h <= 1).all()
    assert not full["keypoints"][7, 3:].any() and not h[7, 3:].any()
    assert not full["keypoints"][200, 2:].any()
    sel = [0, 7, 100, 200, 255]
    ref = O.forward(sd, {"image": img[sel].cpu(), "bboxes": boxes[sel].cpu()}, dual_head=True)
    np.testing.assert_allclose(full["keypoints"][sel].cpu().numpy(), ref["keypoints"].numpy(), atol=1e-5)
    np.testing.assert_allclose(h[sel].cpu().numpy(), ref["heatmap"].numpy(), atol=5e-5)
    assert torch.equal(full["visibilities"][sel].cpu(), ref["visibilities"])
    np.testing.assert_allclose(full["kh_keypoints"][sel].cpu().numpy(), ref["kh_keypoints"].numpy(), atol=1e-5)
    np.testing.assert_allclose(full["kh_visibilities"][sel].cpu().numpy(), ref["kh_visibilities"].numpy(),
                               atol=1e-5)
