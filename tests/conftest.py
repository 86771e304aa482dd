import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "keypoint-detection_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def model_sd():
    """Synthetic weights (seed 0) in the reference's state-dict naming."""
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_state_dict
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig())
    return synthetic_state_dict(m.state_dict(), seed=0)


@pytest.fixture(scope="session")
def model_sd_gray():
    from dll.configs import BackboneConfig, ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_state_dict
    m = MultiPersonKeypointModel(ModelConfig(backbone=BackboneConfig(in_channels=1)), TrainingConfig())
    return synthetic_state_dict(m.state_dict(), seed=0)
