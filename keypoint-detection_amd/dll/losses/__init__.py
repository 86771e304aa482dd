from .keypoint_loss import AdaptiveHeatmapLoss

__all__ = ["AdaptiveHeatmapLoss"]
