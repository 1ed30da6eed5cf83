"""Geometry: the legacy camera-model path's ``LieRotation`` (``geometry/lie_rotation.py``) and the PyTorch
building blocks of the reference's own error closure (``closure_ops``)."""
from .closure_ops import (calibration_network_error, get_camera_relative_points, one_minus_cos_x_on_x_squared,
                          pixel_coordinates_to_homogeneous, project_points_basic_pinhole, project_points_brown_conrady,
                          projective_plane_angle_distance, ray_angle_objective, reprojection_objective,
                          rotate_vector_axis_angle, sin_x_on_x)
from .lie_rotation import LieRotation

__all__ = ["LieRotation", "calibration_network_error", "get_camera_relative_points", "one_minus_cos_x_on_x_squared",
           "pixel_coordinates_to_homogeneous", "project_points_basic_pinhole", "project_points_brown_conrady",
           "projective_plane_angle_distance", "ray_angle_objective", "reprojection_objective",
           "rotate_vector_axis_angle", "sin_x_on_x"]
