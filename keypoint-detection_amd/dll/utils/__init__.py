"""Evaluation helpers (reference ``dll.utils.metric`` / Trainer metrics)."""
from .metric import calculate_validation_metrics, get_default_metrics

__all__ = ["calculate_validation_metrics", "get_default_metrics"]
