"""Goldens for AdaptiveHeatmapLoss from the REFERENCE's own module.

Runs only in the build container: loads /root/reference/dll/losses/
keypoint_loss.py by file path (no package __init__; bytecode off), evaluates
each case of loss_cases.py (loss, threshold, d loss / d pred by autograd) and
writes tests/golden/losses.npz.

    python -B tests/golden/make_loss_golden.py
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from loss_cases import CASES, make_inputs  # noqa: E402

REF = Path("/root/reference/dll/losses/keypoint_loss.py")


def main():
    spec = importlib.util.spec_from_file_location("ref_keypoint_loss", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    for i, (name, B, K, H, W, kind, with_tw, kw) in enumerate(CASES):
        pred, gt, tw = make_inputs(B, K, H, W, kind, with_tw, seed=100 + i)
        crit = mod.AdaptiveHeatmapLoss(**kw)
        p = pred.clone().requires_grad_(True)
        loss = crit(p, gt, tw)
        loss.backward()
        out[f"{name}/loss"] = np.float32(loss.item())
        out[f"{name}/thr"] = np.float32(crit._compute_adaptive_threshold(gt).item())
        out[f"{name}/grad"] = p.grad.numpy().astype(np.float32)
        out[f"{name}/in_sum"] = np.float64(pred.double().sum() + gt.double().sum())
    np.savez_compressed(HERE / "losses.npz", **out)
    print("wrote", HERE / "losses.npz", len(out), "arrays")


if __name__ == "__main__":
    main()
