"""Geometry types of the legacy camera-model path (``geometry/lie_rotation.py``)."""
from .lie_rotation import LieRotation

__all__ = ["LieRotation"]
