"""Goldens for the eval forward with targets (reference
keypoint_model.py:208-209, 509-584: _compute_loss_and_metrics + KeypointLoss,
losses/keypoint_loss.py:28-393) from the REFERENCE's own code.

Runs only in the build container: imports the reference model module the way
make_golden.py does (namespace packages, bytecode off, tv_shim for the absent
torchvision), and calls its _compute_loss_and_metrics on a stand-in `self`
(config, num_keypoints, loss_fn = the reference KeypointLoss) over the call
sequence of kploss_cases.py.  Writes tests/golden/kploss.npz.

    python -B tests/golden/make_kploss_golden.py
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kploss_cases import SEQ, checksum, make_call  # noqa: E402
from make_golden import import_reference  # noqa: E402


def main():
    R = import_reference()
    from dll.losses import KeypointLoss
    cfg = R.cfg.ModelConfig()
    cfg.heatmap_head.heatmap_size = (56, 56)
    tcfg = R.cfg.TrainingConfig()
    me = types.SimpleNamespace(config=cfg, num_keypoints=17,
                               loss_fn=KeypointLoss(num_keypoints=17, config=tcfg, device=torch.device("cpu")))
    out = {}
    for i in range(len(SEQ)):
        outputs, batch = make_call(i)
        out[f"{i}/in_sum"] = np.float64(checksum(outputs, batch))
        res = R.Model._compute_loss_and_metrics(me, dict(outputs), batch)
        out[f"{i}/loss"] = np.float32(res["loss"].item())
        for k in ("heatmap_loss", "coordinate_loss", "visibility_loss", "total_loss"):
            out[f"{i}/{k}"] = np.float64(res[k])
        w = res["loss_weights"]
        out[f"{i}/weights"] = np.array([w["heatmap"], w["coordinate"], w["visibility"]], np.float64)
    np.savez_compressed(HERE / "kploss.npz", **out)
    print("wrote", HERE / "kploss.npz", len(out), "arrays")


if __name__ == "__main__":
    main()
