"""Inputs for tests/golden/data.npz (shared by make_data_golden.py and the
tests, so the fixture stores outputs plus only what is cheap to re-create)."""
import numpy as np
import torch


def _person(rng, n_kp=17, vis=None, zero_xy=False):
    box = [0, *np.round(rng.uniform(0.1, 0.9, 4), 6)]
    kps = []
    for k in range(n_kp):
        x, y = (0.0, 0.0) if zero_xy else tuple(np.round(rng.uniform(0, 1, 2), 6))
        v = (2 if k % 3 else 1) if vis is None else vis
        kps += [x, y, v]
    return " ".join(str(float(v)) if i > 0 else "0" for i, v in enumerate(box + kps))


def _label_cases():
    rng = np.random.default_rng(99)
    p = lambda **kw: _person(rng, **kw)  # noqa: E731
    return {
        "two": p() + "\n" + p() + "\n",
        "one": p() + "\n",                                     # single person: bbox kept unmasked (size(0) == 1)
        "ragged": p() + "\n" + p(n_kp=5) + "\n",               # short row padded with zeros
        "short": p(n_kp=10) + "\n" + p(n_kp=10) + "\n",        # < 17 keypoints everywhere: padded
        "extra": p(n_kp=19) + "\n" + p(n_kp=19) + "\n",        # > 17 keypoints: truncated
        "blank": p() + "\n\n" + p() + "\n",                    # blank line -> zero person, filtered out
        "invisible": p(vis=0) + "\n" + p() + "\n" + p(zero_xy=True) + "\n",   # two filtered, one kept
        "none_valid": p(vis=0) + "\n",                         # nothing valid -> empty annotation
        "empty": "",                                           # empty file -> empty annotation
        "malformed": p() + "\n0 0.5 abc 0.2 0.2\n",            # parse error -> empty annotation
        "many": "".join(p() + "\n" for _ in range(12)),        # > max_persons rows
        "boxonly": "0 0.5 0.5 0.2 0.4\n0 0.3 0.3 0.1 0.1\n",   # no keypoint columns at all
    }


LABEL_CASES = _label_cases()
COLLATE_BATCHES = [["two", "one", "ragged"], ["empty", "invisible", "many", "blank"], ["malformed"]]


def heatmap_cases():
    g = torch.Generator().manual_seed(5)
    kp4 = torch.rand(2, 3, 17, 2, generator=g)
    kp4[0, 0, :6] = torch.tensor([[0.0, 0.0], [0.999, 0.999], [1.0, 0.5], [-0.01, 0.5], [0.5, 1.2], [0.05, 0.95]])
    kp3 = torch.rand(4, 17, 2, generator=g) * 1.2 - 0.1      # some outside [0, 1)
    return [(kp4, (56, 56), 3.0), (kp3, (64, 48), 2.0), (kp4[1], (56, 56), 2.5), (kp3, (30, 41), 1.0)]


def metric_cases():
    g = torch.Generator().manual_seed(6)
    B, P, K = 3, 2, 17
    gt = torch.rand(B, P, K, 2, generator=g)
    pred5 = (gt + torch.randn(B, P, K, 2, generator=g) * 0.05).unsqueeze(2)     # [B,P,1,K,2]
    vis = (torch.rand(B, P, K, generator=g) > 0.3).float() * 2
    return [
        (pred5, gt, vis),                                     # the model's output layout vs collated GT
        (pred5[:, :1], gt, vis),                              # P mismatch -> default (zero) metrics
        (pred5, gt, torch.zeros_like(vis)),                   # nothing visible -> zeros
        (pred5.squeeze(2), gt[:, 0], vis[:, 0]),              # 4-D pred vs 3-D GT: first person
    ]
