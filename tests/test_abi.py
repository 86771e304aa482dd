"""C-ABI library checks that need no GPU: the in-tree libkpd.so loads and
exports every symbol include/kpd.h declares; argument validation errors come
back as negative codes with a message."""
import ctypes
import re

import pytest
import torch

from conftest import ROOT


def _declared():
    hdr = (ROOT / "include" / "kpd.h").read_text()
    return sorted(set(re.findall(r"\b(kpd_[a-z0-9_]+)\s*\(", hdr)))


def test_header_matches_binding():
    from dll import _native
    assert _declared() == sorted(_native.EXPORTS)


def test_library_exports_every_symbol():
    from dll import _native
    lib = _native.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.kpd_version().decode().startswith("kpd")


def test_plan_argument_validation():
    from dll import _native
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.kpd_plan_create(0, 2, ctypes.byref(h)) == -1
    assert b"in_channels" in lib.kpd_last_error()
    assert lib.kpd_plan_create(0, 3, ctypes.byref(h)) == 0
    # forward before finalize -> KPD_ESTATE
    rc = lib.kpd_forward(h, None, 1, 3, 64, 64, None, 0, 0, 0, None, None, None, None, None, None, None, None)
    assert rc == -3 and b"finalized" in lib.kpd_last_error()
    assert lib.kpd_plan_set_detector(h, 1.5, 0.3) == -1
    # finalize without weights -> missing tensors listed (or no HIP device here)
    rc = lib.kpd_plan_finalize(h, 0)
    assert rc in (-2, -3)
    lib.kpd_plan_destroy(h)


def test_model_rejects_cpu_input():
    from dll import _native
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig()).eval()
    with pytest.raises(TypeError):
        m({"image": [1, 2, 3]})
    with pytest.raises(_native.KpdNativeError):
        m({"image": torch.zeros(1, 3, 64, 64), "bboxes": torch.zeros(1, 1, 4)})


def test_state_dict_roundtrip_names():
    """Reference checkpoints load by name (predict.py:47-57 filtering)."""
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig())
    sd = m.state_dict()
    assert "backbone.body.features.0.0.weight" in sd
    assert "backbone.body.features.11.block.2.fc1.weight" in sd
    assert "backbone.fpn.fpn_convs.0.1.running_var" in sd
    assert "person_detector.anchors" in sd and sd["person_detector.anchors"].shape == (28224, 4)
    assert "heatmap_head.final_layer.3.weight" in sd
    assert sum(p.numel() for p in m.parameters()) == 2516500
    m2 = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), dual_head=True)
    assert any(k.startswith("keypoint_head.") for k in m2.state_dict())


def test_anchors_match_oracle():
    from dll.configs import PersonDetectionConfig
    from dll.models import PERSON_HEAD
    from oracle import kpd_oracle as O
    ph = PERSON_HEAD(PersonDetectionConfig())
    assert torch.equal(ph.anchors, O.generate_anchors())


def test_default_build_reads_no_diagnostic_switches(monkeypatch):
    """The production libkpd.so is not a diagnostic build: the ablation /
    A/B switches (KPD_HMCONV_DBG=1 gives wrong results by design in a
    `make diag` build) and the KPD_STAMPS phase stamps are compiled out, so
    no environment variable other than KPD_GRAPH (the graph-replay default)
    is ever read -- a stray KPD_HMCONV_DBG=1 on a serving box changes nothing."""
    from dll import _native
    monkeypatch.delenv("KPD_LIB", raising=False)
    monkeypatch.delenv("KPD_DIAG_LIB", raising=False)
    path = _native.lib_path()
    assert path.name == "libkpd.so"
    lib = _native.load()
    assert lib.kpd_build_flags() & 1 == 0
    switches = set()
    for f in (ROOT / "keypoint-detection_amd" / "csrc").glob("*.hip"):
        switches |= set(re.findall(r'kpd_diag_env\("(KPD_[A-Z0-9_]+)"\)', f.read_text()))
    assert {"KPD_HMCONV_DBG", "KPD_FPN0X_DBG", "KPD_STAMPS"} <= switches
    blob = path.read_bytes()
    assert [n for n in sorted(switches) if n.encode() in blob] == []
    assert b"KPD_GRAPH" in blob
    monkeypatch.setenv("KPD_DIAG_LIB", "1")
    assert _native.lib_path().name == "libkpd_diag.so"
