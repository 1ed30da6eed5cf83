"""Seeded synthetic-scene dataset (the replacement for the reference's
``data/camera_and_parameters_dataset.py``, whose ``_project_points`` (:153-201) does not parse)."""
from .camera_and_parameters_dataset import CameraAndParametersDataset, CameraViewsAndPoints

__all__ = ["CameraAndParametersDataset", "CameraViewsAndPoints"]
