"""Inputs of the decoder / helper goldens (decoders.npz), regenerated from
seeds by both tests/golden/make_golden.py and the tests (the fixture holds
the reference's outputs only)."""
import torch

BOXES = [[0.5, 0.5, 0.4, 0.8], [0.05, 0.9, 0.3, 0.5], [0.5, 0.5, 1.4, 0.2]]


def inputs():
    g = torch.Generator().manual_seed(77)
    h = torch.rand(3, 17, 56, 56, generator=g)
    h[0, 0] = 0.0
    h[0, 0, 10, 20] = h[0, 0, 30, 5] = 0.9            # exact tie: first index wins
    h[0, 1] = 0.0
    h[0, 1, 0, 55] = 1.0                               # corner peak: clipped window
    h[0, 2] = 0.0                                      # all zero: subpixel mass 0
    h[1] = h[1] ** 8                                   # peaky maps
    hr = torch.rand(2, 5, 24, 40, generator=g)         # non-square maps
    kp = torch.rand(1, 17, 2, generator=g)
    feats = torch.rand(2, 128, 20, 16, generator=g)
    return {"h": h, "hr": hr, "kp": kp, "feats": feats, "boxes": torch.tensor(BOXES)}
