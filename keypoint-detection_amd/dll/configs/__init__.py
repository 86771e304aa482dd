from .base_config import BaseConfig, DeviceConfig
from .model_config import (BackboneConfig, HeatmapHeadConfig, KeypointHeadConfig,
                           ModelConfig, PersonDetectionConfig)
from .training_config import (AugmentationConfig, LossConfig, LRSchedulerConfig,
                              OptimizerConfig, TrainingConfig)

__all__ = [
    "BaseConfig", "DeviceConfig", "ModelConfig", "BackboneConfig", "PersonDetectionConfig",
    "KeypointHeadConfig", "HeatmapHeadConfig", "TrainingConfig", "OptimizerConfig",
    "AugmentationConfig", "LossConfig", "LRSchedulerConfig",
]
