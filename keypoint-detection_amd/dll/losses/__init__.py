from .keypoint_loss import (AdaptiveHeatmapLoss, DynamicLossBalancer, ImprovedKeypointLoss, KeypointLoss, LossMetrics,
                            SpatialCoordinateLoss)

__all__ = ["AdaptiveHeatmapLoss", "DynamicLossBalancer", "ImprovedKeypointLoss", "KeypointLoss", "LossMetrics",
           "SpatialCoordinateLoss"]
