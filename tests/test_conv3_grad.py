"""The heatmap head's 3x3 convolution forward and backward (SURVEY §8(f)
rank 4, the backward of K6; kpd_conv3x3_forward / kpd_conv3x3_backward)
against torch autograd in float64 on the CPU.  Tolerance: 1e-5 of the
output's magnitude (fp32 sums of up to N*H*W = 6,272 products, exact
products on both sides)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _ref(x, w, b, gy):
    x64, w64, b64 = (t.detach().double().cpu().requires_grad_(True) for t in (x, w, b))
    y = F.conv2d(x64, w64, b64, padding=1)
    y.backward(gy.double().cpu())
    return y.detach(), x64.grad, w64.grad, b64.grad


def _close(got, want, rel=1e-5):
    got = got.detach().double().cpu()
    scale = want.abs().max().item() + 1e-30
    err = (got - want).abs().max().item()
    assert err <= rel * scale, f"max|d| {err:.3e} > {rel} x {scale:.3e}"


@pytest.mark.parametrize("N,C,H,W,O", [(2, 64, 14, 14, 256), (1, 5, 9, 11, 7), (2, 256, 56, 56, 64), (1, 64, 56, 56, 256),
                                       (3, 17, 20, 13, 33)])
def test_conv3x3_forward_backward_vs_torch(N, C, H, W, O):
    from dll.ops import conv3x3
    g = torch.Generator().manual_seed(N * 1000 + C + O)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5
    b = torch.randn(O, generator=g) * 0.1
    gy = torch.randn(N, O, H, W, generator=g)
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = conv3x3(xd, wd, bd)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    yr, gxr, gwr, gbr = _ref(x, w, b, gy)
    _close(y, yr)
    _close(xd.grad, gxr)
    _close(wd.grad, gwr)
    _close(bd.grad, gbr)


def test_conv3x3_deterministic_and_partial_grads():
    """Same inputs -> bit-identical gradients; gradients requested alone equal
    the ones computed together; no bias."""
    from dll import _native
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 32, 28, 28, generator=g).to(DEV)
    w = (torch.randn(48, 32, 3, 3, generator=g) * 0.1).to(DEV)
    gy = torch.randn(2, 48, 28, 28, generator=g).to(DEV)
    a = _native.conv3x3_backward(x, w, gy)
    b = _native.conv3x3_backward(x, w, gy)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    gx, _, _ = _native.conv3x3_backward(x, w, gy, need_w=False, need_b=False)
    _, gw, _ = _native.conv3x3_backward(x, w, gy, need_x=False, need_b=False)
    assert torch.equal(gx, a[0]) and torch.equal(gw, a[1])
    y = _native.conv3x3_forward(x, w, None)
    _close(y, F.conv2d(x.double().cpu(), w.double().cpu(), None, padding=1))


def test_heatmap_head_conv_chain_grads():
    """The HeatmapHead conv chain shape (64 -> 256 -> 256 -> 64 at 56x56, BN
    folded, ReLU between): weight gradients of a loss through native convs
    equal torch autograd's.  The fp64 reference takes the ReLU masks of the
    native forward (a pre-activation within ~1e-6 of zero may fall on the
    other side of the kink in fp32; one flipped element moves a weight
    gradient by ~1e-4 of its magnitude), and the masks themselves agree with
    the fp64 forward's on all but a 1e-4 fraction of the elements."""
    from dll.ops import conv3x3
    g = torch.Generator().manual_seed(3)
    chans = [64, 256, 256, 64]
    ws = [torch.randn(chans[i + 1], chans[i], 3, 3, generator=g) * (2.0 / (9 * chans[i])) ** 0.5 for i in range(3)]
    bs = [torch.randn(chans[i + 1], generator=g) * 0.05 for i in range(3)]
    x = torch.rand(1, 64, 56, 56, generator=g)
    target = torch.rand(1, 64, 56, 56, generator=g)

    def run(conv, dev, dtype, masks):
        wp = [t.to(dev, dtype).requires_grad_(True) for t in ws]
        bp = [t.to(dev, dtype).requires_grad_(True) for t in bs]
        h = x.to(dev, dtype)
        own = []
        for i in range(3):
            pre = conv(h, wp[i], bp[i])
            own.append((pre > 0).cpu())
            h = pre * (own[i] if masks is None else masks[i]).to(dev, dtype)
        loss = ((h - target.to(dev, dtype)) ** 2).mean()
        loss.backward()
        return [p.grad for p in wp] + [p.grad for p in bp], own

    got, masks = run(conv3x3, DEV, torch.float32, None)
    want, masks64 = run(lambda h, w, b: F.conv2d(h, w, b, padding=1), "cpu", torch.float64, masks)
    for m, m64 in zip(masks, masks64):
        assert (m != m64).float().mean().item() <= 1e-4
    for u, v in zip(got, want):
        _close(u, v, rel=2e-5)
