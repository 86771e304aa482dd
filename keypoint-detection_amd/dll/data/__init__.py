"""Preprocessing drop-in for the reference's ``dll.data.transforms``."""
from .transforms import ITransform

__all__ = ["ITransform"]
