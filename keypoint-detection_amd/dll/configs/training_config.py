"""Training configuration.  Only ``pck_thresholds`` is read on the inference
hot path; the remaining fields are kept so the reference's constructor call
``TrainingConfig()`` and YAML dicts keep working (reference:
dll/configs/training_config.py:94-133).  Training itself is out of scope."""
from dataclasses import dataclass, field
from typing import List

from .base_config import BaseConfig, DeviceConfig


@dataclass
class OptimizerConfig(BaseConfig):
    name: str = "adam"
    learning_rate: float = 0.001
    weight_decay: float = 1e-4
    momentum: float = 0.9
    beta1: float = 0.9
    beta2: float = 0.999


@dataclass
class AugmentationConfig(BaseConfig):
    enabled: bool = False
    prob: float = 0.5


@dataclass
class LossConfig(BaseConfig):
    keypoint_loss_weight: float = 15.0
    visibility_loss_weight: float = 5.0


@dataclass
class LRSchedulerConfig(BaseConfig):
    factor: float = 0.1
    patience: int = 3
    min_lr: float = 1e-6
    mode: str = "min"
    threshold: float = 1e-4
    metric: str = "loss"


@dataclass
class TrainingConfig(BaseConfig):
    num_epochs: int = 50
    batch_size: int = 32
    num_workers: int = 4
    optimizer: OptimizerConfig = field(default_factory=OptimizerConfig)
    augmentation: AugmentationConfig = field(default_factory=AugmentationConfig)
    loss: LossConfig = field(default_factory=LossConfig)
    lr_scheduler: LRSchedulerConfig = field(default_factory=LRSchedulerConfig)
    device: DeviceConfig = field(default_factory=DeviceConfig)
    checkpoint_interval: int = 5
    validation_interval: int = 1
    lr_factor: float = 0.1
    patience: int = 3
    min_lr: float = 1e-6
    lambda_keypoint: float = 15.0
    lambda_visibility: float = 5.0
    l2_lambda: float = 0.0003
    default_validation_threshold: float = 0.5
    pck_thresholds: List[float] = field(default_factory=lambda: [0.002, 0.05, 0.2])
