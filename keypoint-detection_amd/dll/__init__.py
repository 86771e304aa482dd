"""MI355X-native drop-in for the reference's ``dll`` inference path.

Only the hot path (``dll.models`` + configs) is provided; the reference's
data pipeline, training loop and visualisation are out of scope.
"""
from .configs import ModelConfig, TrainingConfig
from .models import MultiPersonKeypointModel

__version__ = "1.0.0+mi355x"

__all__ = ["MultiPersonKeypointModel", "ModelConfig", "TrainingConfig"]
