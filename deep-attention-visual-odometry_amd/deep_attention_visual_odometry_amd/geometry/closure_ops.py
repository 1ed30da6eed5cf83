"""PyTorch building blocks of the reference's own error closure (``networks/calibration_network.py:58-67``).

``CalibrationNetwork`` hands ``BFGSSolver`` a Python closure composed of these functions, so a caller
switching to this package keeps writing it the same way; the drop-in solver then runs that closure
through its generic loop (``autograd_solvers/bfgs_solver.py``).  They are plain tensor code -- the
closure is the caller's, not the hot path (the fused kernels evaluate the same objective as
``RayAngleError``) -- written with ``torch.where`` branches so that no op synchronises with the host:
  * ``sin_x_on_x``, ``one_minus_cos_x_on_x_squared``: ``utils/func_sin_x_on_x.py:5-98`` and
    ``utils/func_one_minus_cos_x_on_x_squared.py:6-51`` -- the same series thresholds and the same
    hand-written backward formulas (differentiable again, for the create_graph mode);
  * ``rotate_vector_axis_angle``: ``geometry/axis_angle_rotation.py:25-48``;
  * ``pixel_coordinates_to_homogeneous``: ``geometry/homogeneous_projection.py:21-44`` ((u - cx, v - cy,
    elu(f) + 1));
  * ``projective_plane_angle_distance``: ``geometry/projective_plane_angle_distance.py:20-64`` (Kahan's
    2 atan2(|a^ - b^|, |a^ + b^|), norms clamped at 2^-52);
  * ``get_camera_relative_points``: ``camera_model/calibration_pinhole_camera_model.py:78-117``, with the
    scale means kept as (B, 1, 1, 1) so that it broadcasts for B > 1 (the reference's means drop those
    dimensions, which breaks any batch other than 1);
  * ``project_points_basic_pinhole``: ``geometry/camera_projection.py:20-35`` (f xy / z + c);
  * ``project_points_brown_conrady``: ``camera_model/distorted_camera_model.py:24-103`` at the BA
    objective's camera (fx = fy = f, skew 0, the extrinsics already applied): the z' == 0 nudge, the
    f-scaled coordinates and the radial / tangential block, in the reference's operation order.
``reprojection_objective`` / ``ray_angle_objective`` compose them into the objectives the fused kernels
evaluate (``ReprojectionError`` / ``RayAngleError`` on CPU tensors run these; on the GPU the kernels).
"""
import torch
from torch.nn.functional import elu

_SINC_SERIES = 0.01
_VERSINE_SERIES = 0.05
_EPS = 2.220446049250313e-16


def _reciprocal(x: torch.Tensor) -> torch.Tensor:
    return torch.where(x == 0, torch.zeros_like(x), 1.0 / x)


class _SinXonX(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        ctx.set_materialize_grads(False)
        x2 = x * x
        series = 1.0 - x2 / 6.0 + (x2 * x2) / 120 - (x2 * x2 * x2) / 5040
        return torch.where(x.abs() < _SINC_SERIES, series, torch.sin(x) / x)

    @staticmethod
    def backward(ctx, grad):
        if grad is None:
            return None
        (x,) = ctx.saved_tensors
        return grad * x * _CosOverXSquaredMinusSinOverXCubed.apply(x)[0]


class _CosOverXSquaredMinusSinOverXCubed(torch.autograd.Function):
    """cos(x)/x^2 - sin(x)/x^3 and 1/x (0 at 0), the derivative of sin(x)/x over x."""

    @staticmethod
    def forward(ctx, x):
        x2 = x * x
        series = -1.0 / 3.0 + x2 / 30.0 - (x2 * x2) / 840 + (x2 * x2 * x2) / 45360
        out = torch.where(x.abs() < _SINC_SERIES, series, torch.cos(x) / x2 - torch.sin(x) / (x * x2))
        recip = _reciprocal(x)
        ctx.save_for_backward(x, out, recip)
        ctx.set_materialize_grads(False)
        return out, recip

    @staticmethod
    def backward(ctx, grad, grad_recip):
        if grad is None and grad_recip is None:
            return None
        x, out, recip = ctx.saved_tensors
        g = 0.0
        if grad is not None:
            g = -1.0 * grad * recip * (_SinXonX.apply(x) + 3.0 * out)
        if grad_recip is not None:
            g = g - grad_recip * recip * recip
        return g


class _OneMinusCosXonXSquared(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x2 = x * x
        series = 0.5 - x2 / 24 + (x2 * x2) / 720 - (x2 * x2 * x2) / 40320
        out = torch.where(x.abs() < _VERSINE_SERIES, series, (1.0 - torch.cos(x)) / x2)
        recip = _reciprocal(x)
        ctx.save_for_backward(x, out, recip)
        ctx.set_materialize_grads(False)
        return out, recip

    @staticmethod
    def backward(ctx, grad, grad_recip):
        if grad is None:
            return None
        x, out, recip = ctx.saved_tensors
        g = grad * recip * (_SinXonX.apply(x) - 2.0 * out)
        if grad_recip is not None:
            g = g - grad_recip * recip * recip
        return g


def sin_x_on_x(x: torch.Tensor) -> torch.Tensor:
    return _SinXonX.apply(x)


def one_minus_cos_x_on_x_squared(x: torch.Tensor) -> torch.Tensor:
    return _OneMinusCosXonXSquared.apply(x)[0]


def rotate_vector_axis_angle(vector: torch.Tensor, axis_angle: torch.Tensor) -> torch.Tensor:
    """R(axis_angle) vector by Rodrigues' formula: v cos t + (1 - cos t)/t^2 (v . w) w + sin(t)/t (w x v)."""
    angle = torch.linalg.vector_norm(axis_angle, dim=-1, keepdim=True)
    dot = (vector * axis_angle).sum(dim=-1, keepdims=True)
    cross = torch.linalg.cross(axis_angle, vector, dim=-1)
    return vector * torch.cos(angle) + one_minus_cos_x_on_x_squared(angle) * dot * axis_angle \
        + cross * sin_x_on_x(angle)


def pixel_coordinates_to_homogeneous(projected_points: torch.Tensor, intrinsics: torch.Tensor) -> torch.Tensor:
    """(B..., 2) pixels and (B..., 3) intrinsics (f, cx, cy) -> (B..., 3) rays (u - cx, v - cy, elu(f) + 1)."""
    focal = elu(intrinsics[..., 0:1]) + 1.0
    centred = projected_points - intrinsics[..., 1:3]
    return torch.cat([centred, focal.expand(centred.shape[:-1] + (-1,))], dim=-1)


def projective_plane_angle_distance(a: torch.Tensor, b: torch.Tensor, keepdim: bool = False) -> torch.Tensor:
    """Angle between two sets of homogeneous 3-vectors, 2 atan2(|a^ - b^|, |a^ + b^|)."""
    a = a / torch.linalg.vector_norm(a, dim=-1, keepdim=True).clamp(min=_EPS)
    b = b / torch.linalg.vector_norm(b, dim=-1, keepdim=True).clamp(min=_EPS)
    total = torch.linalg.vector_norm(a + b, dim=-1, keepdim=keepdim)
    diff = torch.linalg.vector_norm(a - b, dim=-1, keepdim=keepdim)
    return 2.0 * torch.atan2(diff, total)


def get_camera_relative_points(world_points: torch.Tensor, camera_translations: torch.Tensor,
                               camera_rotations: torch.Tensor) -> torch.Tensor:
    """(B, 1, N, 3) points, (B, M-1, 1, 3) translations and axis-angle rotations -> (B, M, N, 3) points relative
    to each view (view 0 at the origin), all scaled by (mean|X| N + mean|t| M) / (N + M)."""
    n = world_points.size(-2)
    m = camera_translations.size(-3) + 1
    point_scale = world_points.abs().mean(dim=(-1, -2, -3), keepdim=True)
    view_scale = camera_translations.abs().mean(dim=(-1, -2, -3), keepdim=True)
    scale = (point_scale * n + view_scale * m) / (n + m)
    camera_translations = camera_translations / scale
    world_points = world_points / scale
    moved = rotate_vector_axis_angle(world_points, camera_rotations) + camera_translations
    return torch.concatenate([world_points, moved], dim=-3)


def calibration_network_error(true_projected_points: torch.Tensor, visibility_mask: torch.Tensor, num_views: int,
                              num_points: int):
    """The error closure ``CalibrationNetwork.forward`` builds (``networks/calibration_network.py:58-67``), over
    observations (B, M, N, 2) and a visibility mask (B, M, N): error_function(parameters, batch_mask) -> (b,)."""
    from ..camera_model import unpack_calibration_parameters

    def error_function(parameters: torch.Tensor, batch_mask: torch.Tensor) -> torch.Tensor:
        targets = true_projected_points[batch_mask]
        camera_parameters = unpack_calibration_parameters(parameters, num_views, num_points)
        homogeneous_points = pixel_coordinates_to_homogeneous(targets, camera_parameters.intrinsics)
        world_points = get_camera_relative_points(world_points=camera_parameters.world_points,
                                                  camera_translations=camera_parameters.camera_translations,
                                                  camera_rotations=camera_parameters.camera_rotations)
        distance = projective_plane_angle_distance(homogeneous_points, world_points)
        return (distance * visibility_mask[batch_mask]).sum(dim=(-1, -2))

    return error_function


def project_points_basic_pinhole(points: torch.Tensor, intrinsics: torch.Tensor) -> torch.Tensor:
    """(B..., 3) camera-relative points and (B..., 3) intrinsics (f, cx, cy) -> (B..., 2) pixels."""
    return intrinsics[..., 0:1] * points[..., 0:2] / points[..., 2:3] + intrinsics[..., 1:3]


def project_points_brown_conrady(points: torch.Tensor, intrinsics: torch.Tensor,
                                 coefficients: torch.Tensor) -> torch.Tensor:
    """(B..., 3) camera-relative points, (B..., 3) intrinsics (f, cx, cy) and (B..., 5) coefficients
    (k1, k2, k3, p1, p2) -> (B..., 2) distorted pixels.  The skew term s (y'/z') of the reference's model is kept
    with s = 0, so a non-finite y'/z' propagates as it does there."""
    x, y, z = points[..., 0], points[..., 1], points[..., 2]
    z = torch.where(z == 0, z + 1e-8, z)
    f, cx, cy = intrinsics[..., 0], intrinsics[..., 1], intrinsics[..., 2]
    k1, k2, k3, p1, p2 = coefficients.unbind(-1)
    u = f * (x / z) + torch.zeros_like(f) * (y / z)
    v = f * (y / z)
    r2 = u * u + v * v
    uv = u * v
    radial = 1.0 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
    ud = u * radial + 2.0 * p1 * uv + p2 * (r2 + 2 * u * u) + cx
    vd = v * radial + 2.0 * p2 * uv + p1 * (r2 + 2 * v * v) + cy
    return torch.stack([ud, vd], dim=-1)


def _unpacked_points(parameters: torch.Tensor, num_views: int, num_points: int, distortion: bool):
    from ..camera_model import unpack_calibration_parameters

    base = parameters[..., :-5] if distortion else parameters
    cam = unpack_calibration_parameters(base, num_views, num_points)
    points = get_camera_relative_points(world_points=cam.world_points, camera_translations=cam.camera_translations,
                                        camera_rotations=cam.camera_rotations)
    return cam, points


def reprojection_objective(parameters: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor,
                           num_views: int, num_points: int, distortion: bool = False) -> torch.Tensor:
    """E(x) = sum_{m,n} vis ||pi_m(X_n) - obs||^2 for (B..., P) parameters, (B..., M, N, 2) observations and
    (B..., M, N) visibility: the squared objective the fused kernels evaluate, as torch ops."""
    cam, points = _unpacked_points(parameters, num_views, num_points, distortion)
    if distortion:
        lead = parameters.shape[:-1]
        uv = project_points_brown_conrady(points, cam.intrinsics, parameters[..., -5:].reshape(lead + (1, 1, 5)))
    else:
        uv = project_points_basic_pinhole(points, cam.intrinsics)
    sq = (uv - observations).square().sum(dim=-1)
    return (sq * visibility.to(sq.dtype)).sum(dim=(-1, -2))


def ray_angle_objective(parameters: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor,
                        num_views: int, num_points: int) -> torch.Tensor:
    """sum_{m,n} vis * angle(ray(obs), p_m(X_n)): CalibrationNetwork's error (calibration_network.py:58-67)."""
    cam, points = _unpacked_points(parameters, num_views, num_points, False)
    rays = pixel_coordinates_to_homogeneous(observations, cam.intrinsics)
    return (projective_plane_angle_distance(rays, points) * visibility.to(points.dtype)).sum(dim=(-1, -2))
