from .backbone import BACKBONE, MobileNetV3Wrapper
from .heatmap_head import HeatmapHead
from .keypoint_head import KEYPOINT_HEAD
from .keypoint_model import MultiPersonKeypointModel
from .person_head import PERSON_HEAD

__all__ = ["MultiPersonKeypointModel", "BACKBONE", "PERSON_HEAD", "KEYPOINT_HEAD", "MobileNetV3Wrapper",
           "HeatmapHead"]
