"""Data drop-in for the reference's ``dll.data``: the device ITransform, the
YOLO-pose dataset and its collate (dataloader.py)."""
from .dataloader import (AdaptiveBatchSampler, OptimizedKeypointsDataset, create_adaptive_dataloader,
                         create_optimized_dataloader, efficient_collate_fn)
from .transforms import ITransform

__all__ = ["create_optimized_dataloader", "OptimizedKeypointsDataset", "ITransform", "efficient_collate_fn",
           "AdaptiveBatchSampler", "create_adaptive_dataloader"]
