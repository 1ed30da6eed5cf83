"""Calibration parameter layout and the native reprojection objective.

``unpack_calibration_parameters`` mirrors
``camera_model/calibration_pinhole_camera_model.py:33-75`` (same names,
same shapes, same ValueError on a wrong P).  ``ReprojectionError`` is the
error-function object the drop-in ``BFGSSolver`` recognises and runs fully
fused on the GPU; it is also an ordinary ``error_function(parameters,
batch_mask)`` closure (``networks/calibration_network.py:58-67`` contract)
whose value and derivatives (first order, and second order for
create_graph callers: H v and the observation cross term) come from HIP
kernels, differentiable w.r.t. the parameters and the observations.
"""
from typing import NamedTuple

import torch

from .. import native_ops
from ..geometry.closure_ops import get_camera_relative_points  # noqa: F401  (reference: camera_model/__init__.py)


def num_parameters(num_views: int, num_points: int, distortion: bool = False) -> int:
    return 3 + 3 * num_points + 6 * (num_views - 1) + (5 if distortion else 0)


class CalibrationParameters(NamedTuple):
    intrinsics: torch.Tensor
    world_points: torch.Tensor
    camera_translations: torch.Tensor
    camera_rotations: torch.Tensor


def unpack_calibration_parameters(parameters: torch.Tensor, num_views: int, num_points: int) -> CalibrationParameters:
    """Views of a (B..., 3 + 3N + 6(M-1)) parameter tensor (pinhole layout)."""
    expected = 3 + 3 * num_points + 6 * (num_views - 1)
    if parameters.size(-1) != expected:
        raise ValueError(
            f"The final dimension of the input tensor must be 3 + 3 * num_points + 6 * (num_views - 1) = "
            f"{expected}, got {parameters.size(-1)}")
    lead = parameters.shape[:-1]
    p_end = 3 + 3 * num_points
    t_end = p_end + 3 * (num_views - 1)
    return CalibrationParameters(
        intrinsics=parameters[..., 0:3].reshape(lead + (1, 1, 3)),
        world_points=parameters[..., 3:p_end].reshape(lead + (1, num_points, 3)),
        camera_translations=parameters[..., p_end:t_end].reshape(lead + (num_views - 1, 1, 3)),
        camera_rotations=parameters[..., t_end:].reshape(lead + (num_views - 1, 1, 3)),
    )


class _NativeObjective(torch.autograd.Function):
    """E(x, obs) per row from the HIP objective kernel.  Its backward is itself
    differentiable (``_NativeGradient``), so ``torch.autograd.grad(..., create_graph=True)``
    -- the reference's differentiate-through-the-solve mode -- gets exact second
    derivatives from the forward-over-reverse kernel (``dava_ba_second_order``)."""

    @staticmethod
    def forward(ctx, x, observations, visibility, num_views, num_points, distortion, residual):
        need_x, need_obs = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if need_obs:  # dE/dobs comes from the second-order kernel (v = 0)
            err, grad, _, obs_grad, _ = native_ops.ba_second_order(
                x, observations, visibility, num_views, num_points, distortion, residual=residual, want_hv=False)
        else:
            err, grad, _ = native_ops.ba_evaluate(x, observations, visibility, num_views, num_points, distortion,
                                                  want_grad=need_x, residual=residual)
            obs_grad = None
        ctx.save_for_backward(x, observations, visibility)
        ctx.meta = (num_views, num_points, distortion, residual)
        ctx.first = (grad, obs_grad)
        return err

    @staticmethod
    def backward(ctx, grad_out):
        x, obs, vis = ctx.saved_tensors
        need_x, need_obs = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if torch.is_grad_enabled():  # create_graph: keep the gradient differentiable
            grad, obs_grad = _NativeGradient.apply(x, obs, vis, *ctx.meta)
        else:
            grad, obs_grad = ctx.first
        gx = grad_out.unsqueeze(-1) * grad if need_x else None
        gobs = grad_out[:, None, None, None] * obs_grad if (need_obs and obs_grad is not None) else None
        return gx, gobs, None, None, None, None, None


class _NativeGradient(torch.autograd.Function):
    """(dE/dx, dE/dobs) as a differentiable function of (x, obs): its VJP along the x-cotangent
    u is (H u, (d2E/dobs dx) u), from one forward-over-reverse launch."""

    @staticmethod
    def forward(ctx, x, observations, visibility, num_views, num_points, distortion, residual):
        _, grad, _, obs_grad, _ = native_ops.ba_second_order(
            x, observations, visibility, num_views, num_points, distortion, residual=residual, want_hv=False)
        ctx.save_for_backward(x, observations, visibility)
        ctx.meta = (num_views, num_points, distortion, residual)
        ctx.set_materialize_grads(False)
        return grad, obs_grad

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, u, u_obs):
        # u_obs: a cotangent on dE/dobs (differentiating it again): the observations carry it as a tangent in
        # the same forward-over-reverse launch (dava_ba_second_order_obs)
        if u is None and u_obs is None:
            return None, None, None, None, None, None, None
        x, obs, vis = ctx.saved_tensors
        _, _, hv, _, obs_hv = native_ops.ba_second_order(x, obs, vis, *ctx.meta[:3], direction=u,
                                                          residual=ctx.meta[3],
                                                          want_obs=ctx.needs_input_grad[1], obs_direction=u_obs)
        return (hv if ctx.needs_input_grad[0] else None, obs_hv if ctx.needs_input_grad[1] else None,
                None, None, None, None, None)


class ReprojectionError:
    """Squared multi-view reprojection error of SURVEY.md 8(a).

    E(x) = sum_{m,n} vis[m,n] || pi_m(X_n) - obs[m,n] ||^2

    observations: (B..., M, N, 2) float32, visibility: (B..., M, N) bool/0-1,
    on the same ROCm device as the parameters.  With ``distortion=True`` the
    five Brown-Conrady coefficients (k1 k2 k3 p1 p2) are appended to the
    parameter vector (``camera_model/distorted_camera_model.py:59-86``).
    """

    def __init__(self, observations: torch.Tensor, visibility: torch.Tensor, num_views: int, num_points: int,
                 distortion: bool = False):
        if observations.shape[-3:] != (num_views, num_points, 2):
            raise ValueError(f"observations must end in ({num_views}, {num_points}, 2), got {tuple(observations.shape)}")
        if visibility.shape != observations.shape[:-1]:
            raise ValueError("visibility must have shape observations.shape[:-1]")
        if num_views < 2:
            raise ValueError("num_views must be >= 2")
        # (device tensors: the kernels read float32; CPU tensors keep their dtype for the torch objective)
        self.observations = observations if observations.device.type == "cpu" else observations.to(torch.float32)
        self.visibility = visibility.to(torch.uint8)
        self.num_views = int(num_views)
        self.num_points = int(num_points)
        self.distortion = bool(distortion)

    residual = native_ops.N.DAVA_RESIDUAL_SQUARED_REPROJECTION

    @property
    def num_parameters(self) -> int:
        return num_parameters(self.num_views, self.num_points, self.distortion)

    @property
    def batch_shape(self) -> torch.Size:
        return self.observations.shape[:-3]

    def __call__(self, parameters: torch.Tensor, batch_mask: torch.Tensor) -> torch.Tensor:
        if parameters.size(-1) != self.num_parameters:
            raise ValueError(f"expected {self.num_parameters} parameters, got {parameters.size(-1)}")
        obs = self.observations[batch_mask]
        vis = self.visibility[batch_mask]
        lead = parameters.shape[:-1]
        x = parameters.reshape(-1, parameters.size(-1))
        obs = obs.reshape(-1, self.num_views, self.num_points, 2)
        vis = vis.reshape(-1, self.num_views, self.num_points)
        if x.device.type == "cpu":
            # CPU tensors: the same objective as torch ops (geometry.closure_ops), so the drop-in solves where
            # the parameters live, as the reference does (bfgs_solver.py:94-117); autograd gives its derivatives
            # to any order.  Device tensors take the HIP kernels below, never this.
            return self._torch_objective(x, obs.to(x.dtype), vis).reshape(lead)
        if x.dtype != torch.float32:
            raise TypeError("ReprojectionError evaluates in float32")
        err = _NativeObjective.apply(x, obs, vis, self.num_views, self.num_points, self.distortion, self.residual)
        return err.reshape(lead)


    def _torch_objective(self, x, obs, vis):
        from ..geometry.closure_ops import reprojection_objective

        return reprojection_objective(x, obs, vis, self.num_views, self.num_points, self.distortion)


class RayAngleError(ReprojectionError):
    """The error ``CalibrationNetwork`` minimises (``networks/calibration_network.py:58-67``):

    E(x) = sum_{m,n} vis[m,n] * angle(ray(obs[m,n]), p_m(X_n))

    with ray(u, v) = (u - cx, v - cy, elu(f) + 1)
    (``geometry/homogeneous_projection.py:21-44``), p_m(X_n) the scale-normalised
    camera-relative point (``camera_model/calibration_pinhole_camera_model.py:78-117``)
    and the angle in Kahan's form 2 atan2(|a^ - b^|, |a^ + b^|)
    (``geometry/projective_plane_angle_distance.py:20-64``).  Pinhole parameter
    layout only; the fused solver and the evaluation kernel both run it on the GPU (on CPU tensors, torch ops).
    """

    residual = native_ops.N.DAVA_RESIDUAL_RAY_ANGLE

    def __init__(self, observations: torch.Tensor, visibility: torch.Tensor, num_views: int, num_points: int):
        super().__init__(observations, visibility, num_views, num_points, distortion=False)

    def _torch_objective(self, x, obs, vis):
        from ..geometry.closure_ops import ray_angle_objective

        return ray_angle_objective(x, obs, vis, self.num_views, self.num_points)


from .pinhole_camera_model_l1 import PinholeCameraModelL1  # noqa: E402  (legacy IOptimisableFunction model)
