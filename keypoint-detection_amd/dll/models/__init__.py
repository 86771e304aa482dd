from .backbone import BACKBONE, MobileNetV3Wrapper
from .heatmap_head import HeatmapHead, decode_heatmaps, decode_heatmaps_soft_argmax, decode_heatmaps_subpixel
from .keypoint_head import KEYPOINT_HEAD
from .keypoint_model import (MultiPersonKeypointModel, box_center_to_corners, pad_to_length,
                             select_top_k_channels)
from .person_head import PERSON_HEAD

__all__ = ["MultiPersonKeypointModel", "BACKBONE", "PERSON_HEAD", "KEYPOINT_HEAD", "MobileNetV3Wrapper",
           "HeatmapHead"]
