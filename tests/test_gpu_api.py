"""The dll.models API surface beyond MultiPersonKeypointModel.forward, on the
device: submodule forwards (HeatmapHead and its attention modules,
KEYPOINT_HEAD, MobileNetV3Wrapper, ChannelAttention, PERSON_HEAD), the
heatmap decoders, the model's helper methods and module functions, and the
INTEGRATION.md ctypes stub executed verbatim.

Goldens come from the reference's own code (tests/golden/make_golden.py:
heatmap_head.npz, keypoint_head.npz, decoders.npz); the oracle pins what no
golden holds (all four FPN levels).  Tolerances: decoders 1e-6 (argmax /
visibility classes exact), submodule outputs as the forward's fp32 bar
(1e-5 keypoints, 5e-5 heatmaps) in fp32 and split precision.
"""
import ctypes
import re

import numpy as np
import pytest
import torch

from oracle import kpd_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _np(p):
    return np.load(p, allow_pickle=False)


def _model(sd, precision="split"):
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision=precision)
    m.load_state_dict(sd)
    return m.to(DEV).eval()


@pytest.fixture(scope="module")
def dec(golden_dir):
    import sys
    sys.path.insert(0, str(golden_dir))
    import decoder_cases
    return _np(golden_dir / "decoders.npz"), decoder_cases.inputs()


def test_decoders_vs_golden(dec):
    from dll.models import decode_heatmaps, decode_heatmaps_soft_argmax, decode_heatmaps_subpixel
    g, c = dec
    h = c["h"].to(DEV)
    k, s = decode_heatmaps(h)
    assert np.array_equal(k.cpu().numpy(), g["argmax_kpts"]) and np.array_equal(s.cpu().numpy(), g["argmax_scores"])
    for w in (3, 5):
        k, s = decode_heatmaps_subpixel(h, window_size=w)
        np.testing.assert_allclose(k.cpu().numpy(), g[f"sub{w}_kpts"], atol=1e-6)
        np.testing.assert_allclose(s.cpu().numpy(), g[f"sub{w}_scores"], atol=0)
    for i, t in enumerate(g["sa_temps"]):
        k, s = decode_heatmaps_soft_argmax(h, temperature=float(t))
        np.testing.assert_allclose(k.cpu().numpy(), g[f"sa{i}_kpts"], atol=1e-6)
        assert np.array_equal(s.cpu().numpy(), g[f"sa{i}_scores"])
    k, s = decode_heatmaps(h[2])                      # [K, H, W] input keeps the reference's shapes
    assert k.shape == g["argmax3d_kpts"].shape and np.array_equal(k.cpu().numpy(), g["argmax3d_kpts"])
    k, s = decode_heatmaps_subpixel(h[2])
    assert k.shape == g["sub3d_kpts"].shape
    np.testing.assert_allclose(k.cpu().numpy(), g["sub3d_kpts"], atol=1e-6)
    hr = c["hr"].to(DEV)                              # non-square maps
    assert np.array_equal(decode_heatmaps(hr)[0].cpu().numpy(), g["hr_argmax_kpts"])
    np.testing.assert_allclose(decode_heatmaps_subpixel(hr)[0].cpu().numpy(), g["hr_sub_kpts"], atol=1e-6)
    np.testing.assert_allclose(decode_heatmaps_soft_argmax(hr)[0].cpu().numpy(), g["hr_sa_kpts"], atol=1e-6)
    # window_size 0 (reference :327 pad = 0 // 2): the 1x1 window at the maximum
    # = the argmax where the maximum is positive, zeros where its mass is 0
    k0, s0 = decode_heatmaps_subpixel(h, window_size=0)
    ka, sa = decode_heatmaps(h)
    pos = (sa > 0).unsqueeze(-1)
    torch.testing.assert_close(k0, torch.where(pos, ka, torch.zeros_like(ka)), atol=1e-6, rtol=0)
    assert torch.equal(s0, torch.where(sa > 0, sa, torch.zeros_like(sa)))


def test_model_helpers_vs_golden(dec, model_sd):
    from dll.models import select_top_k_channels
    g, c = dec
    m = _model(model_sd)
    h = c["h"].to(DEV)
    k, v = m.decode_heatmap(h)
    np.testing.assert_allclose(k.cpu().numpy(), g["model_kpts"], atol=1e-6)
    assert np.array_equal(v.cpu().numpy(), g["model_vis"])
    np.testing.assert_allclose(m._soft_argmax(h).cpu().numpy(), g["model_sa"], atol=1e-6)
    feats = c["feats"].to(DEV)
    np.testing.assert_allclose(m.channel_attention(feats).cpu().numpy(), g["ca_scores"], atol=1e-6)
    sel = select_top_k_channels(feats, m.channel_attention, k=64)
    topk = m.channel_attention.native_select(feats)[1].cpu().numpy()
    assert np.array_equal(topk, g["ca_topk"])
    np.testing.assert_allclose(sel.double().sum(dim=(2, 3)).cpu().numpy(), g["selected_sum"], rtol=1e-6)
    roi = m.extract_roi_features(feats[:1], c["boxes"][1].to(DEV))
    assert tuple(roi.shape) == tuple(g["roi_feat_shape"])
    np.testing.assert_allclose(roi[0, :8, 20:28, 10:18].cpu().numpy(), g["roi_feat_slice"], atol=1e-6)
    np.testing.assert_allclose(roi.double().sum(dim=(2, 3)).cpu().numpy(), g["roi_feat_sum"], rtol=1e-5)
    kp = c["kp"].to(DEV)
    got = torch.stack([m.convert_to_original_coords(kp.clone(), b) for b in c["boxes"].to(DEV)])
    np.testing.assert_allclose(got.cpu().numpy(), g["kp_orig"], atol=1e-7)


@pytest.mark.parametrize("precision", ["fp32", "split"])
def test_heatmap_head_forward_vs_golden(golden_dir, model_sd, precision):
    """HeatmapHead.forward standalone on the golden's ROI features
    (heatmap_head.npz), attention weights vs a plain fp32 torch restatement,
    and the attention modules' own forwards."""
    g = _np(golden_dir / "heatmap_head.npz")
    m = _model(model_sd, precision)
    x = torch.from_numpy(g["x"].astype(np.float32)).to(DEV)
    heat, (cw, sw) = m.heatmap_head(x)
    assert heat.shape == (1, 17, 56, 56) and cw.shape == (1, 64, 1, 1) and sw.shape == (1, 1, 56, 56)
    np.testing.assert_allclose(heat[:, :, 20:24, 30:34].cpu().numpy(), g["heat_slice"], atol=5e-5)
    np.testing.assert_allclose(heat.double().sum(dim=(2, 3)).cpu().numpy(), g["heat_sum"], rtol=1e-4)
    k, v = m.decode_heatmap(heat)
    np.testing.assert_allclose(k.cpu().numpy(), g["model_kpts"], atol=1e-5)
    assert np.array_equal(v.cpu().numpy(), g["model_vis"])
    # attention weights: sigmoid(fc(avg) + fc(max)) and sigmoid(conv7x7([mean, max]))
    xc = x.double().cpu()
    p = "heatmap_head."
    sd = {k2: t.double() for k2, t in model_sd.items() if k2.startswith(p)}

    def fc(t):
        t = torch.relu(t @ sd[p + "channel_attention.fc.0.weight"].T + sd[p + "channel_attention.fc.0.bias"])
        return t @ sd[p + "channel_attention.fc.2.weight"].T + sd[p + "channel_attention.fc.2.bias"]
    cw_ref = torch.sigmoid(fc(xc.mean(dim=(2, 3))) + fc(xc.amax(dim=(2, 3))))
    np.testing.assert_allclose(cw.view(1, 64).cpu().double().numpy(), cw_ref.numpy(), atol=1e-6)
    xa = xc * cw_ref.view(1, 64, 1, 1)
    a = torch.cat([xa.mean(dim=1, keepdim=True), xa.amax(dim=1, keepdim=True)], dim=1)
    sw_ref = torch.sigmoid(torch.nn.functional.conv2d(a, sd[p + "spatial_attention.conv.weight"],
                                                      sd[p + "spatial_attention.conv.bias"], padding=3))
    np.testing.assert_allclose(sw.cpu().double().numpy(), sw_ref.numpy(), atol=1e-6)
    # the attention modules' own forwards
    cw2 = m.heatmap_head.channel_attention(x)
    np.testing.assert_allclose(cw2.cpu().numpy(), cw.cpu().numpy(), atol=0)
    sw2 = m.heatmap_head.spatial_attention(xa.float().to(DEV))
    np.testing.assert_allclose(sw2.cpu().double().numpy(), sw_ref.numpy(), atol=1e-6)
    # batch of ROIs vs the oracle's head
    xb = torch.rand(3, 64, 56, 56, generator=torch.Generator().manual_seed(4))
    hb, _ = m.heatmap_head(xb.to(DEV))
    np.testing.assert_allclose(hb.cpu().numpy(), O.heatmap_head(xb, model_sd).numpy(), atol=5e-5)


def test_visibility_threshold_exact_float(model_sd):
    """keypoint_model.py:268-280 compares conf.item() (a Python double) with
    0.3 / 0.7: a confidence of exactly float32(0.7) = 0.69999998... is class 1
    (occluded), float32(0.3) = 0.30000001... is class 1 too.  Maxima chosen so
    torch's sigmoid lands on those floats exactly."""
    m = _model(model_sd)
    planes, want = [], []
    for target in (0.7, 0.3):
        t32 = torch.tensor(target, dtype=torch.float32)
        bits0 = int(torch.logit(t32.double()).float().view(torch.int32))
        found = None
        for d in sorted(range(-64, 65), key=abs):     # the float32 values a few ulps around the logit
            x = torch.tensor(bits0 + d, dtype=torch.int32).view(torch.float32)
            if torch.sigmoid(x) == t32:
                found = x
                break
        assert found is not None
        hp = torch.full((56, 56), -3.0)
        hp[20, 30] = found
        planes.append(hp)
        c = float(torch.sigmoid(found))        # the reference's conf.item()
        want.append(0 if c < 0.3 else (1 if c < 0.7 else 2))
    h = torch.stack(planes).view(1, 2, 56, 56).to(DEV)
    _, v = m.decode_heatmap(h)
    got = v.view(2, 3).argmax(dim=-1).tolist()
    assert got == want == [1, 1]


def test_heatmap_head_split_signed_inputs(model_sd):
    """Stand-alone HeatmapHead in split precision on inputs of either sign: the
    hi/lo operand scale must come from max |x| (the model's ROI features are
    post-ReLU, a caller's need not be).  ROI 0 randn, ROI 1 all negative,
    ROI 2 with a negative tail 50x its positive maximum."""
    g = torch.Generator().manual_seed(21)
    x = torch.randn(3, 64, 56, 56, generator=g)
    x[1] = -x[1].abs() - 0.1
    x[2] = torch.rand(64, 56, 56, generator=g) * 0.1
    x[2, 5, 10:20, 10:20] = -5.0
    m = _model(model_sd, "split")
    h, _ = m.heatmap_head(x.to(DEV))
    assert torch.isfinite(h).all()
    np.testing.assert_allclose(h.cpu().numpy(), O.heatmap_head(x, model_sd).numpy(), atol=5e-5)


@pytest.mark.parametrize("precision", ["fp32", "split"])
def test_keypoint_head_forward_vs_golden(golden_dir, precision):
    from dll.configs import KeypointHeadConfig
    from dll.models import KEYPOINT_HEAD
    from dll.models.synthetic import synthetic_state_dict, weights_checksum
    g = _np(golden_dir / "keypoint_head.npz")
    kh = KEYPOINT_HEAD(KeypointHeadConfig(height=56, width=56))
    ksd = synthetic_state_dict(kh.state_dict(), seed=3)
    assert abs(weights_checksum(ksd) - float(g["checksum"])) < 1e-6
    kh.load_state_dict(ksd)
    kh.precision = precision
    kh = kh.to(DEV).eval()
    xk = torch.randn(2, 128, 56, 56, generator=torch.Generator().manual_seed(11))
    kp, vis = kh(xk.to(DEV))
    np.testing.assert_allclose(kp.cpu().numpy(), g["keypoints"], atol=1e-5)
    np.testing.assert_allclose(vis.cpu().numpy(), g["visibility"], atol=1e-5)


@pytest.mark.parametrize("precision", ["fp32", "split"])
def test_backbone_forward_four_levels(model_sd, precision):
    """MobileNetV3Wrapper.forward returns the four FPN levels (the model's
    forward computes only level 0)."""
    from dll.models.synthetic import synthetic_images
    m = _model(model_sd, precision)
    img = synthetic_images(2, 3, 256, 192, seed=12)
    outs = m.backbone(img.to(DEV))
    taps = O.mbv3_small_taps(img, model_sd)
    lats = O.fpn_laterals(taps, model_sd)
    for i, o in enumerate(outs):
        ref = O.fpn_level(lats[i], model_sd, i)
        assert o.shape == ref.shape
        np.testing.assert_allclose(o.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("hw", [(256, 192), (200, 152)])
def test_backbone_body_and_fpn_submodules(model_sd, hw):
    """backbone.body(x) returns the feature extractor's OrderedDict of the four
    taps and backbone.fpn(taps) the four levels (reference backbone.py:29-39,
    253-264), each native on its own; the FPN also on taps the caller made
    (the oracle's), and with a level size that is not a 2x multiple of the
    next (nearest indexing as F.interpolate)."""
    from dll.models.synthetic import synthetic_images
    m = _model(model_sd)
    H, W = hw
    img = synthetic_images(2, 3, H, W, seed=21)
    taps = m.backbone.body(img.to(DEV))
    assert list(taps.keys()) == ["feat0", "feat1", "feat2", "feat3"]
    ref_taps = O.mbv3_small_taps(img, model_sd)
    for t, r in zip(taps.values(), ref_taps):
        assert t.shape == r.shape
        np.testing.assert_allclose(t.cpu().numpy(), r.numpy(), rtol=1e-4, atol=1e-4)
    outs = m.backbone.fpn(list(taps.values()))
    own = m.backbone.fpn([r.to(DEV) for r in ref_taps])
    lats = O.fpn_laterals(ref_taps, model_sd)
    for i in range(4):
        ref = O.fpn_level(lats[i], model_sd, i)
        assert outs[i].shape == ref.shape
        np.testing.assert_allclose(outs[i].cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(own[i].cpu().numpy(), ref.numpy(), rtol=1e-5, atol=2e-5)
    # odd level sizes: level 1 at 13 x 9 upsampled from 6 x 5 (not 2x)
    g = torch.Generator().manual_seed(5)
    odd = [torch.rand(1, c, h, w, generator=g) for c, (h, w) in zip((16, 24, 48, 576),
                                                                     ((52, 36), (13, 9), (6, 5), (3, 2)))]
    got = m.backbone.fpn([o.to(DEV) for o in odd])
    lats = O.fpn_laterals(odd, model_sd)
    for i in range(4):
        np.testing.assert_allclose(got[i].cpu().numpy(), O.fpn_level(lats[i], model_sd, i).numpy(), rtol=1e-5,
                                   atol=2e-5)
    with pytest.raises(ValueError):
        m.backbone.fpn(list(taps.values())[:3])


def test_person_head_forward(model_sd):
    from dll.models import MultiPersonKeypointModel  # noqa: F401
    m = _model(model_sd)
    feats = [torch.rand(2, 128, s, s, generator=torch.Generator().manual_seed(s)) for s in (56, 28, 14, 7)]
    out = m.person_detector([f.to(DEV) for f in feats])
    w = model_sd["person_detector.box_heads.3.weight"]
    b = model_sd["person_detector.box_heads.3.bias"]
    ref = torch.nn.functional.conv2d(feats[3].double(), w.double(), b.double())
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), atol=1e-5)


def test_integration_stub_runs_verbatim(model_sd, monkeypatch):
    """The ctypes binding shown in INTEGRATION.md (the block that starts with
    '# kpd ctypes stub'), executed as written against libkpd.so: its
    kpd_forward must return the drop-in model's outputs."""
    from conftest import ROOT
    from dll import _native
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    text = (ROOT / "INTEGRATION.md").read_text()
    code = re.search(r"```python\n(# kpd ctypes stub\n.*?)```", text, re.S).group(1)
    monkeypatch.setenv("KPD_LIB", str(_native.lib_path()))
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    img = synthetic_images(2, 3, 256, 192, seed=3).to(DEV)
    boxes = synthetic_boxes(2, 2, seed=4).to(DEV)
    boxes[1, 1] = 0.0
    plan = ns["kpd_plan_from_state_dict"](model_sd)
    try:
        out = ns["kpd_forward"](plan, img, boxes)
        torch.cuda.synchronize()
    finally:
        ns["_kpd"].kpd_plan_destroy(plan)
    m = _model(model_sd, "split")
    with torch.no_grad():
        ref = m({"image": img, "bboxes": boxes})
    for k in ("keypoints", "visibilities", "heatmap"):
        assert torch.equal(out[k], ref[k]), k
