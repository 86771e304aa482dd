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
