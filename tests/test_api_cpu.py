"""CPU-side API checks (no GPU): the tensor helper functions against the
reference's own outputs (decoders.npz), the inference-only guards, and the
plan key (the person-detector thresholds rebuild the plan)."""
import sys

import numpy as np
import pytest
import torch


def _model():
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    return MultiPersonKeypointModel(ModelConfig(), TrainingConfig())


def test_box_helpers_vs_golden(golden_dir):
    sys.path.insert(0, str(golden_dir))
    import decoder_cases
    from dll.models import box_center_to_corners, pad_to_length
    g = np.load(golden_dir / "decoders.npz", allow_pickle=False)
    c = decoder_cases.inputs()
    got = torch.stack([box_center_to_corners(b) for b in c["boxes"]])
    assert np.array_equal(got.numpy(), g["corners"])
    padded = pad_to_length([torch.ones(2, 3), 2 * torch.ones(2, 3)], 4)
    assert np.array_equal(torch.stack(padded).numpy(), g["padded"])
    assert pad_to_length([], 3) == [] and len(pad_to_length([torch.ones(1)] * 5, 2)) == 2
    m = _model()
    got = torch.stack([m.convert_to_original_coords(c["kp"].clone(), b) for b in c["boxes"]])
    np.testing.assert_allclose(got.numpy(), g["kp_orig"], atol=1e-7)


def test_inference_only_guards():
    m = _model()
    x = torch.zeros(1, 3, 64, 64)
    m.train()
    with torch.no_grad(), pytest.raises(NotImplementedError, match="training mode"):
        m({"image": x})
    m.eval()
    # a batch with targets takes the same device path (its loss is added after
    # the native forward): a CPU input still fails loudly, before any loss
    from dll import _native
    with pytest.raises(_native.KpdNativeError, match="HIP device"):
        m({"image": x, "bboxes": torch.zeros(1, 1, 4), "keypoints": torch.zeros(1, 1, 17, 2),
           "visibilities": torch.zeros(1, 1, 17)})
    with pytest.raises(TypeError):
        m({"image": [1, 2]})
    from dll import _native
    with pytest.raises(_native.KpdNativeError, match="HIP device"):
        m({"image": x, "bboxes": torch.zeros(1, 1, 4)})


def test_plan_key_tracks_detector_thresholds():
    m = _model()
    k0 = m._weights_key(torch.device("cpu"))
    m.config.person_head.conf_threshold = 0.55
    assert m._weights_key(torch.device("cpu")) != k0
    m.precision = "mixed"
    assert m.heatmap_head.precision == "mixed" and m.backbone.precision == "mixed"
    with pytest.raises(ValueError):
        m.precision = "fp8"


def test_integration_stub_block_parses():
    import ast
    import re
    from conftest import ROOT
    text = (ROOT / "INTEGRATION.md").read_text()
    code = re.search(r"```python\n(# kpd ctypes stub\n.*?)```", text, re.S).group(1)
    tree = ast.parse(code)
    names = {n.name for n in tree.body if isinstance(n, ast.FunctionDef)}
    assert {"kpd_plan_from_state_dict", "kpd_forward"} <= names
    # the argtypes list matches the 18 parameters of kpd_forward in include/kpd.h
    hdr = (ROOT / "include" / "kpd.h").read_text()
    sig = re.search(r"int kpd_forward\((.*?)\);", hdr, re.S).group(1)
    assert len(sig.split(",")) == 18
    at = re.search(r"_kpd\.kpd_forward\.argtypes = \[(.*?)\]", code).group(1)
    assert len(at.split(",")) == 18
