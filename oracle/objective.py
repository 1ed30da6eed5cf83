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
  3. u = f*x/z + cx, v = f*y/z + cy (``geometry/camera_projection.py:20-35``), or with
     distortion the reference's own distorted model (``camera_model/distorted_camera_model.py:
     24-103``: z' nudge, u = fx (x/z) + s (y/z), v = fy (y/z), radial + tangential block) on
     camera rows fx = fy = f, s = 0, zero rotation / translation -- pinned bitwise to that
     file's output (``tests/golden/distortion.npz``).

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


def project(p: torch.Tensor, intrinsics: torch.Tensor) -> torch.Tensor:
    """Pinhole (``geometry/camera_projection.py:20-35``): f * xy / z + c."""
    return intrinsics[..., 0:1] * p[..., 0:2] / p[..., 2:3] + intrinsics[..., 1:3]


# slot order of the reference's 16-parameter camera table (``spatial_maths.camera_model_parameters``,
# as listed by ``tests/camera_model/test_distorted_camera_model.py:13-30``)
CX, CY, K1, K2, K3, P1, P2, FX, SKEW, FY = range(10)


def camera_rows(x: torch.Tensor, num_views: int) -> torch.Tensor:
    """(B, P) BA parameters -> (B*M, 16) camera rows in the reference's slot order: fx = fy = f,
    skew, rotation and translation 0 (the BA objective supplies camera-relative points),
    cx, cy, k1 k2 k3 p1 p2 from x (distortion = the last 5 entries)."""
    b = x.shape[0]
    zero = x.new_zeros(b, 1)
    f, cx, cy, k = x[:, 0:1], x[:, 1:2], x[:, 2:3], x[:, -5:]
    row = torch.cat([cx, cy, k, f, zero, f] + [zero] * 6, dim=-1)
    return row[:, None, :].expand(b, num_views, 16).reshape(b * num_views, 16)


def distorted_rows(pts: torch.Tensor, rows: torch.Tensor):
    """u', v' (R, N) of points (R, N, 3) under camera rows (R, 16): the reference's
    ``_full_forward_model`` (``camera_model/distorted_camera_model.py:24-103``) at zero rotation
    and translation -- its extrinsic step is then the identity, bit for bit -- with the z' == 0
    nudge (:57), the f-scaled coordinates u = fx (x'/z') + s (y'/z'), v = fy (y'/z') (:59-62)
    and the radial / tangential block (:64-86), in the same operation order."""
    xp = pts[:, :, 0]
    yp = pts[:, :, 1]
    zp = pts[:, :, 2].clone()
    zp[zp == 0] += 1e-8
    u = rows[:, None, FX] * (xp / zp) + rows[:, None, SKEW] * (yp / zp)
    v = rows[:, None, FY] * (yp / zp)
    r2 = u * u + v * v
    uv = u * v
    radial = (1.0 + rows[:, None, K1] * r2 + rows[:, None, K2] * r2 * r2
              + rows[:, None, K3] * r2 * r2 * r2)
    ud = u * radial + 2.0 * rows[:, None, P1] * uv + rows[:, None, P2] * (r2 + 2 * u * u) + rows[:, None, CX]
    vd = v * radial + 2.0 * rows[:, None, P2] * uv + rows[:, None, P1] * (r2 + 2 * v * v) + rows[:, None, CY]
    return ud, vd


def project_distorted(p: torch.Tensor, x: torch.Tensor, num_views: int) -> torch.Tensor:
    """Brown-Conrady projection of camera-relative points p (B, M, N, 3) for BA parameters x
    (B, P): ``distorted_rows`` per view on (B*M, N) rows, as the reference model evaluates them."""
    b, _, n, _ = p.shape
    ud, vd = distorted_rows(p.reshape(b * num_views, n, 3), camera_rows(x, num_views))
    return torch.stack([ud, vd], dim=-1).reshape(b, num_views, n, 2)


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
    lead = x.shape[:-1]
    if distortion:
        uv = project_distorted(p.reshape((-1,) + p.shape[-3:]), x.reshape(-1, x.size(-1)), num_views)
        uv = uv.reshape(lead + uv.shape[-3:])
    else:
        uv = project(p, parts.intrinsics)
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
