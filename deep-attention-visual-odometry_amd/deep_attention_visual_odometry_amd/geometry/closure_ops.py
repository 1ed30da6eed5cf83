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
    dimensions, which breaks any batch other than 1).
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
