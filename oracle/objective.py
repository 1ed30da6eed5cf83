"""Multi-view BA reprojection objective (oracle restatement, test infrastructure only).

SURVEY.md section 8(a) defines the benchmark objective.  For a parameter
vector x (one row per problem) with layout

    [f, cx, cy | X_0..X_{N-1} (xyz interleaved) | t_1..t_{M-1} | w_1..w_{M-1} | k1 k2 k3 p1 p2]

(``camera_model/calibration_pinhole_camera_model.py:33-75``; the five
Brown-Conrady coefficients are appended only when distortion is enabled)

    E(x) = sum_{m,n} vis[m,n] * || pi_m(X_n) - obs[m,n] ||^2

where pi_m is:
  1. scale normalisation s = (mean|X| * N + mean|t| * M) / (N + M)
     (``calibration_pinhole_camera_model.py:97-104``; restated with keepdim so
     that it broadcasts correctly for batch > 1),
  2. p = X/s for view 0, p = R(w_m) X/s + t_m/s for views m >= 1
     (``:107-115``, Rodrigues from ``geometry/axis_angle_rotation.py:25-48``),
  3. u = f*x/z + cx, v = f*y/z + cy (``geometry/camera_projection.py:20-35``),
     optionally followed by the Brown-Conrady block of
     ``camera_model/distorted_camera_model.py:59-86`` with fx = fy = f, s = 0.

Every op is written in the same order as the reference so that fp64/fp32
values and autograd gradients round identically.
"""
from typing import NamedTuple, Optional

import torch

from .trig import sinc, versine_ratio


def num_parameters(num_views: int, num_points: int, distortion: bool = False) -> int:
    return 3 + 3 * num_points + 6 * (num_views - 1) + (5 if distortion else 0)


class Unpacked(NamedTuple):
    intrinsics: torch.Tensor  # (B,1,1,3)
    points: torch.Tensor  # (B,1,N,3)
    translations: torch.Tensor  # (B,M-1,1,3)
    rotations: torch.Tensor  # (B,M-1,1,3)
    distortion: Optional[torch.Tensor]  # (B,1,1,5) or None


def split_parameters(x: torch.Tensor, num_views: int, num_points: int, distortion: bool = False) -> Unpacked:
    """Views of x (``calibration_pinhole_camera_model.py:33-75``)."""
    expected = num_parameters(num_views, num_points, distortion)
    if x.size(-1) != expected:
        raise ValueError(f"expected {expected} parameters, got {x.size(-1)}")
    lead = x.shape[:-1]
    p_end = 3 + 3 * num_points
    t_end = p_end + 3 * (num_views - 1)
    w_end = t_end + 3 * (num_views - 1)
    return Unpacked(
        intrinsics=x[..., 0:3].reshape(lead + (1, 1, 3)),
        points=x[..., 3:p_end].reshape(lead + (1, num_points, 3)),
        translations=x[..., p_end:t_end].reshape(lead + (num_views - 1, 1, 3)),
        rotations=x[..., t_end:w_end].reshape(lead + (num_views - 1, 1, 3)),
        distortion=x[..., w_end:w_end + 5].reshape(lead + (1, 1, 5)) if distortion else None,
    )


def rodrigues(v: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """R(w) v (``geometry/axis_angle_rotation.py:25-48``)."""
    theta = torch.linalg.vector_norm(w, dim=-1, keepdim=True)
    vw = (v * w).sum(dim=-1, keepdims=True)
    wxv = torch.linalg.cross(w, v, dim=-1)
    return v * torch.cos(theta) + versine_ratio(theta) * vw * w + wxv * sinc(theta)


def view_points(points: torch.Tensor, translations: torch.Tensor, rotations: torch.Tensor) -> torch.Tensor:
    """(B,M,N,3) camera-relative points, keepdim restatement of
    ``calibration_pinhole_camera_model.py:78-117``."""
    n = points.size(-2)
    m = translations.size(-3) + 1
    point_scale = points.abs().mean(dim=(-1, -2, -3), keepdim=True)
    view_scale = translations.abs().mean(dim=(-1, -2, -3), keepdim=True)
    scale = (point_scale * n + view_scale * m) / (n + m)
    translations = translations / scale
    points = points / scale
    moved = rodrigues(points, rotations) + translations
    return torch.concatenate([points, moved], dim=-3)


def project(p: torch.Tensor, intrinsics: torch.Tensor, distortion: Optional[torch.Tensor]) -> torch.Tensor:
    """Pinhole (``geometry/camera_projection.py:20-35``) plus optional
    Brown-Conrady on the f-scaled coordinates (``distorted_camera_model.py:59-86``)."""
    f = intrinsics[..., 0:1]
    c = intrinsics[..., 1:3]
    if distortion is None:
        return f * p[..., 0:2] / p[..., 2:3] + c
    z = p[..., 2:3]
    u = f * p[..., 0:1] / z
    v = f * p[..., 1:2] / z
    k1 = distortion[..., 0:1]
    k2 = distortion[..., 1:2]
    k3 = distortion[..., 2:3]
    p1 = distortion[..., 3:4]
    p2 = distortion[..., 4:5]
    r2 = u * u + v * v
    uv = u * v
    radial = 1.0 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
    ud = u * radial + 2.0 * p1 * uv + p2 * (r2 + 2 * u * u) + c[..., 0:1]
    vd = v * radial + 2.0 * p2 * uv + p1 * (r2 + 2 * v * v) + c[..., 1:2]
    return torch.cat([ud, vd], dim=-1)


def reprojection_error(
    x: torch.Tensor,
    observations: torch.Tensor,
    visibility: torch.Tensor,
    num_views: int,
    num_points: int,
    distortion: bool = False,
) -> torch.Tensor:
    """E(x), shape x.shape[:-1].  observations (..., M, N, 2), visibility (..., M, N)."""
    parts = split_parameters(x, num_views, num_points, distortion)
    p = view_points(parts.points, parts.translations, parts.rotations)
    uv = project(p, parts.intrinsics, parts.distortion)
    sq = (uv - observations).square().sum(dim=-1)
    return (sq * visibility.to(sq.dtype)).sum(dim=(-1, -2))


class ReprojectionClosure:
    """Closure in the reference's ``error_function(parameters, batch_mask)`` form
    (``networks/calibration_network.py:58-67``), over the squared objective."""

    def __init__(self, observations, visibility, num_views, num_points, distortion=False):
        self.observations = observations
        self.visibility = visibility
        self.num_views = num_views
        self.num_points = num_points
        self.distortion = distortion
        self.calls = 0

    def __call__(self, x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        self.calls += 1
        return reprojection_error(
            x, self.observations[mask], self.visibility[mask], self.num_views, self.num_points, self.distortion
        )


# ---- ray-angle residual (the error CalibrationNetwork minimises) ----------------------

def homogeneous_rays(observations: torch.Tensor, intrinsics: torch.Tensor) -> torch.Tensor:
    """(u - cx, v - cy, elu(f) + 1): ``geometry/homogeneous_projection.py:21-44``."""
    focal = torch.nn.functional.elu(intrinsics[..., 0:1]) + 1.0
    centred = observations - intrinsics[..., 1:3]
    return torch.cat([centred, focal.expand(centred.shape[:-1] + (-1,))], dim=-1)


def projective_plane_angle_distance(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """2 atan2(|a^ - b^|, |a^ + b^|), norms clamped at 2^-52
    (``geometry/projective_plane_angle_distance.py:20-64``)."""
    a = a / torch.linalg.vector_norm(a, dim=-1, keepdim=True).clamp(min=2.220446049250313e-16)
    b = b / torch.linalg.vector_norm(b, dim=-1, keepdim=True).clamp(min=2.220446049250313e-16)
    total = torch.linalg.vector_norm(a + b, dim=-1)
    diff = torch.linalg.vector_norm(a - b, dim=-1)
    return 2.0 * torch.atan2(diff, total)


def ray_angle_error(
    x: torch.Tensor,
    observations: torch.Tensor,
    visibility: torch.Tensor,
    num_views: int,
    num_points: int,
) -> torch.Tensor:
    """``CalibrationNetwork.forward``'s error_function (``networks/calibration_network.py:58-67``):
    sum_{m,n} vis * angle(ray(obs), p), p from the keepdim restatement of
    ``get_camera_relative_points``."""
    parts = split_parameters(x, num_views, num_points, False)
    rays = homogeneous_rays(observations, parts.intrinsics)
    p = view_points(parts.points, parts.translations, parts.rotations)
    distance = projective_plane_angle_distance(rays, p)
    return (distance * visibility).sum(dim=(-1, -2))


class RayAngleClosure:
    """``error_function(parameters, batch_mask)`` over the ray-angle objective."""

    def __init__(self, observations, visibility, num_views, num_points):
        self.observations = observations
        self.visibility = visibility
        self.num_views = num_views
        self.num_points = num_points
        self.calls = 0

    def __call__(self, x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        self.calls += 1
        return ray_angle_error(x, self.observations[mask], self.visibility[mask], self.num_views, self.num_points)
