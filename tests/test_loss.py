"""Training loss row: AdaptiveHeatmapLoss
(reference dll/losses/keypoint_loss.py:202-280) against goldens made by the
reference's own module (tests/golden/make_loss_golden.py), and the device
kernel (kpd_adaptive_heatmap_loss) against those goldens and the CPU oracle.

Tolerances: the threshold (an order statistic + torch's fp32 lerp) bit-exact;
the loss within 2e-6 relative (the device sums in double, torch in fp32
blocks); d loss / d pred within 1e-5 relative + 1e-6 of max|grad| absolute
(fused analytic derivative vs autograd's chain of rounded ops: where mse is
tiny, 1 - exp(-mse) cancels, so one ulp of exp moves the focal factor by
a large relative amount on values that are ~0 anyway).
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
from loss_cases import CASES, make_inputs  # noqa: E402

gpu = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def lg(golden_dir):
    return np.load(golden_dir / "losses.npz", allow_pickle=False)


def _case(i):
    name, B, K, H, W, kind, with_tw, kw = CASES[i]
    pred, gt, tw = make_inputs(B, K, H, W, kind, with_tw, seed=100 + i)
    return name, pred, gt, tw, kw


def _kw(kw):
    return dict(keypoint_weight=kw.get("keypoint_weight", 50.0), background_weight=kw.get("background_weight", 1.0),
                adaptive=kw.get("adaptive_threshold", True), focal_alpha=kw.get("focal_alpha", 2.0))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_oracle_vs_reference_golden(lg, i):
    from oracle import loss_oracle as LO
    name, pred, gt, tw, kw = _case(i)
    assert float(pred.double().sum() + gt.double().sum()) == pytest.approx(float(lg[f"{name}/in_sum"]), rel=1e-12)
    p = pred.clone().requires_grad_(True)
    loss = LO.adaptive_heatmap_loss(p, gt, tw, **_kw(kw))
    loss.backward()
    assert float(LO.adaptive_threshold(gt, kw.get("adaptive_threshold", True))) == float(lg[f"{name}/thr"])
    assert float(loss.detach()) == pytest.approx(float(lg[f"{name}/loss"]), rel=1e-6)
    np.testing.assert_allclose(p.grad.numpy(), lg[f"{name}/grad"], rtol=1e-6, atol=1e-12)


def test_loss_module_rejects_cpu():
    from dll.losses import AdaptiveHeatmapLoss
    x = torch.rand(1, 2, 4, 4)
    with pytest.raises((ValueError, RuntimeError)):
        AdaptiveHeatmapLoss()(x, x)


@gpu
@pytest.mark.parametrize("i", range(len(CASES)))
def test_gpu_loss_vs_reference_golden(lg, i):
    from dll.losses import AdaptiveHeatmapLoss
    name, pred, gt, tw, kw = _case(i)
    crit = AdaptiveHeatmapLoss(**kw)
    p = pred.to(DEV).requires_grad_(True)
    g = gt.to(DEV)
    loss = crit(p, g, tw.to(DEV) if tw is not None else None)
    loss.backward()
    torch.cuda.synchronize()
    assert float(crit._compute_adaptive_threshold(g)) == float(lg[f"{name}/thr"])
    assert float(loss.detach()) == pytest.approx(float(lg[f"{name}/loss"]), rel=2e-6)
    want = lg[f"{name}/grad"]
    np.testing.assert_allclose(p.grad.cpu().numpy(), want, rtol=1e-5, atol=1e-6 * float(np.abs(want).max()))


@gpu
def test_gpu_loss_at_training_size_vs_oracle():
    """A training-batch shape (16 x 17 x 64 x 48, 836k values): threshold
    bit-exact, loss and gradient within tolerance of the oracle; deterministic
    across calls."""
    from oracle import loss_oracle as LO
    from dll import _native
    g0 = torch.Generator().manual_seed(7)
    B, K, H, W = 16, 17, 64, 48
    ys = torch.arange(H, dtype=torch.float32).view(1, 1, H, 1)
    xs = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W)
    cy, cx = torch.rand(B, K, 1, 1, generator=g0) * H, torch.rand(B, K, 1, 1, generator=g0) * W
    gt = torch.exp(-((ys - cy) ** 2 + (xs - cx) ** 2) / 8.0)
    gt[0, 0] = 0.17   # a flat plane: many ties
    pred = (gt + 0.1 * torch.randn(B, K, H, W, generator=g0)).clamp(0, 1)
    tw = (torch.rand(B, K, generator=g0) > 0.2).float()
    p = pred.clone().requires_grad_(True)
    ref = LO.adaptive_heatmap_loss(p, gt, tw)
    ref.backward()
    l1, g1, t1 = _native.adaptive_heatmap_loss(pred.to(DEV), gt.to(DEV), tw.to(DEV), 50.0, 1.0, True, 2.0, True)
    l2, g2, t2 = _native.adaptive_heatmap_loss(pred.to(DEV), gt.to(DEV), tw.to(DEV), 50.0, 1.0, True, 2.0, True)
    torch.cuda.synchronize()
    assert float(t1) == float(LO.adaptive_threshold(gt))
    assert float(l1) == pytest.approx(float(ref.detach()), rel=2e-6)
    np.testing.assert_allclose(g1.cpu().numpy(), p.grad.numpy(), rtol=1e-5, atol=1e-6 * float(p.grad.abs().max()))
    assert torch.equal(l1, l2) and torch.equal(g1, g2) and torch.equal(t1, t2)


@gpu
def test_gpu_quantile_select_exact():
    """The radix select: torch.quantile(x, 0.9) bit-exact with duplicates and
    sizes whose rank is fractional or integral (values inside (0.05, 0.3), so
    the clamp does not hide the interpolated quantile)."""
    from dll import _native
    from oracle import loss_oracle as LO
    g0 = torch.Generator().manual_seed(11)
    for n in (11, 101, 1000, 4097, 65537):
        x = 0.05 + 0.25 * torch.rand(n, generator=g0)
        x[: n // 3] = x[n // 2]                       # duplicates
        x = x.view(1, 1, 1, n)
        _, _, thr = _native.adaptive_heatmap_loss(x.to(DEV), x.to(DEV), None, 50.0, 1.0, True, 0.0, False)
        want = torch.clamp(torch.quantile(x.flatten(), 0.9), 0.05, 0.3)
        assert float(thr) == float(want) == float(LO.adaptive_threshold(x)), n


# ---------------------------------------------------------------------------
# KeypointLoss (ImprovedKeypointLoss) and the eval forward with targets
# (reference keypoint_model.py:208-209, 509-584; keypoint_loss.py:28-393),
# against goldens of the reference's own _compute_loss_and_metrics over a
# 13-call sequence (tests/golden/make_kploss_golden.py): the balancer adapts
# its weights at call 10.  Tolerances: components 2e-6 (heatmap: device
# double sums vs torch fp32; coordinate / visibility: the same torch ops on
# another device), weights and total 1e-5.
# ---------------------------------------------------------------------------
from kploss_cases import SEQ, checksum, make_call  # noqa: E402


@pytest.fixture(scope="module")
def kg(golden_dir):
    return np.load(golden_dir / "kploss.npz", allow_pickle=False)


def _glue_inputs(outputs, batch):
    """The person-axis reductions of _compute_loss_and_metrics (reference :513-568)."""
    pv = outputs["visibilities"].squeeze(2).max(dim=1)[0]
    gv = batch["visibilities"].max(dim=1)[0]
    return outputs["keypoints"].squeeze(2), batch["keypoints"], pv, gv


def test_kploss_small_terms_and_balancer_vs_reference_golden(kg):
    """CPU: the coordinate and visibility terms and the balancer's weight
    sequence (fed the golden components) reproduce the reference's."""
    from dll.losses import DynamicLossBalancer, SpatialCoordinateLoss
    from dll.configs import TrainingConfig
    tc = TrainingConfig()
    bal = DynamicLossBalancer({"heatmap": tc.lambda_keypoint, "coordinate": 5.0, "visibility": tc.lambda_visibility})
    coord = SpatialCoordinateLoss()
    for i in range(len(SEQ)):
        outputs, batch = make_call(i)
        assert checksum(outputs, batch) == pytest.approx(float(kg[f"{i}/in_sum"]), rel=1e-12)
        pk, gk, pv, gv = _glue_inputs(outputs, batch)
        assert float(coord(pk, gk, gv)) == pytest.approx(float(kg[f"{i}/coordinate_loss"]), rel=2e-6)
        ce = torch.nn.functional.cross_entropy(pv.reshape(-1, 3), gv.reshape(-1).long())
        assert float(ce) == pytest.approx(float(kg[f"{i}/visibility_loss"]), rel=2e-6)
        w = bal.update_weights({k: float(kg[f"{i}/{k}_loss"]) for k in ("heatmap", "coordinate", "visibility")})
        np.testing.assert_allclose([w["heatmap"], w["coordinate"], w["visibility"]], kg[f"{i}/weights"], rtol=1e-12)


def test_kploss_bad_shape_raises_like_reference():
    """[B,P,K] terms against the [B,K] mask: P must be 1 or B (reference :186-187)."""
    from dll.losses import SpatialCoordinateLoss
    g = torch.Generator().manual_seed(0)
    pk, gk = torch.rand(2, 3, 17, 2, generator=g), torch.rand(2, 3, 17, 2, generator=g)
    with pytest.raises(RuntimeError):
        SpatialCoordinateLoss()(pk, gk, torch.ones(2, 17))


def _loss_model(sd):
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    cfg = ModelConfig()
    cfg.heatmap_head.heatmap_size = (56, 56)
    m = MultiPersonKeypointModel(cfg, TrainingConfig())
    m.load_state_dict(sd)
    return m.to(DEV).eval()


@gpu
def test_kploss_sequence_vs_reference_golden(kg, model_sd):
    """_compute_loss_and_metrics with the device heatmap term, call by call."""
    m = _loss_model(model_sd)
    for i in range(len(SEQ)):
        outputs, batch = make_call(i)
        o = {k: v.to(DEV) for k, v in outputs.items()}
        b = {k: v.to(DEV) for k, v in batch.items()}
        res = m._compute_loss_and_metrics(o, b)
        for k in ("heatmap_loss", "coordinate_loss", "visibility_loss"):
            assert res[k] == pytest.approx(float(kg[f"{i}/{k}"]), rel=2e-6), (i, k)
        assert res["keypoint_loss"] == res["heatmap_loss"]
        w = res["loss_weights"]
        np.testing.assert_allclose([w["heatmap"], w["coordinate"], w["visibility"]], kg[f"{i}/weights"], rtol=1e-5)
        assert float(res["loss"]) == pytest.approx(float(kg[f"{i}/loss"]), rel=1e-5)
        assert res["loss_metrics"].total_loss == pytest.approx(float(res["loss"]), rel=1e-6)


@gpu
def test_eval_forward_with_targets(model_sd):
    """model(batch) with 'keypoints' / 'visibilities' / 'heatmaps' (the
    trainer's validation call, trainer.py:331-334) returns the eval outputs
    plus the loss of those outputs; without 'heatmaps' the zero targets of
    heatmap_size are used."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    m, ref = _loss_model(model_sd), _loss_model(model_sd)
    img = synthetic_images(2, 3, 256, 192, seed=31).to(DEV)
    boxes = synthetic_boxes(2, 1, seed=32).to(DEV)
    g = torch.Generator().manual_seed(33)
    tg = {"keypoints": torch.rand(2, 1, 17, 2, generator=g).to(DEV),
          "visibilities": torch.randint(0, 3, (2, 1, 17), generator=g).to(DEV),
          "heatmaps": torch.rand(2, 1, 17, 56, 56, generator=g).to(DEV)}
    out = m({"image": img, "bboxes": boxes, **tg})
    plain = ref({"image": img, "bboxes": boxes})
    for k in ("heatmap", "keypoints", "visibilities"):
        assert torch.equal(out[k], plain[k])
    exp = ref._compute_loss_and_metrics(dict(plain), {"image": img, **tg})
    assert float(out["loss"]) == float(exp["loss"])
    for k in ("heatmap_loss", "coordinate_loss", "visibility_loss", "total_loss"):
        assert out[k] == exp[k]
    tg.pop("heatmaps")
    out2 = m({"image": img, "bboxes": boxes, **tg})
    assert out2["heatmap_loss"] > 0 and np.isfinite(float(out2["loss"]))
