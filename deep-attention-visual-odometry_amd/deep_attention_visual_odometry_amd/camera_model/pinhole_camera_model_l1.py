"""``PinholeCameraModelL1`` on the GPU (reference: ``camera_model/pinhole_camera_model_l1.py``).

The legacy ``IOptimisableFunction`` consumed by ``BFGSCameraSolver`` +
``LineSearchStrongWolfeConditions`` (``solvers/``; configurations
``bfgs_solver_*_config.yaml``).  Same constructor, properties and methods as the
reference; ``get_error`` / ``get_gradient`` are one HIP launch over every
(batch, estimate) (``dava_l1_camera_evaluate``, csrc/camera_l1.hip), returning the
reference's L1 error and its HAND-WRITTEN gradient (max_gradient clipping included).
``add`` / ``masked_update`` are parameter bookkeeping with the reference's semantics;
``as_parameters_vector`` returns the (B, E, P) vector ``add`` consumes (the reference's
cannot run for its own tensor shapes, see the method).

Autograd through the model's error/gradient tensors follows the reference's
``enable_error_gradients`` / ``enable_grad_gradients`` (``:139-198``): the backward is the
HIP VJP kernel (``dava_l1_camera_vjp``: one forward-mode dual-number pass per input element,
contracted with the cotangents in-kernel).  With ``enable_error_gradients=False`` the error is
returned detached; with ``enable_grad_gradients=False`` the gradient is differentiated with the
world and camera-relative points held constant, as the reference's detaches do -- on a full
evaluation only: its partial recompute of masked estimates (``:223-270``) detaches nothing, and
neither does this one.  Gradients
into ``true_projected_points`` (r06) follow the reference's error: -scale sgn((u - t) vis) vis per pixel
coordinate, formed from the reference's own torch expressions for u, v (``_target_term``); its hand-written
gradient depends on them only through sign(), so not at all.
"""
from typing import Optional

import torch

from .. import _native as N
from .. import _ops  # noqa: F401  (registers torch.ops.dava.l1_camera_evaluate)
from ..geometry.lie_rotation import LieRotation
from ..solvers.i_optimisable_function import IOptimisableFunction
from ..utils import merge_cached_values


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


class _L1Evaluate(torch.autograd.Function):
    """error (B, E) / gradient (B, E, P) of the six parameter tensors, differentiable: the backward
    is ``dava::l1_camera_vjp`` (two launches when the gradient's points are detached and the
    error's are not)."""

    @staticmethod
    def forward(ctx, fixed, want_error, want_gradient, focal, cx, cy, trans, lie, world):
        target, vis, min_z, ratio, mg, scale, detach_points = fixed
        err, grad = torch.ops.dava.l1_camera_evaluate(focal, cx, cy, trans, lie, world, target, vis, min_z, ratio,
                                                      mg, scale, want_error, want_gradient)
        ctx.save_for_backward(focal, cx, cy, trans, lie, world)
        ctx.fixed, ctx.want = fixed, (want_error, want_gradient)
        return err, grad

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_err, g_grad):
        focal, cx, cy, trans, lie, world = ctx.saved_tensors
        target, vis, min_z, ratio, mg, scale, detach_points = ctx.fixed
        ge = _c(g_err) if (g_err is not None and ctx.want[0]) else None
        gg = _c(g_grad) if (g_grad is not None and ctx.want[1]) else None
        args = (focal, cx, cy, trans, lie, world, target, vis, min_z, ratio, mg, scale)
        if detach_points and ge is not None and gg is not None:
            vjp = torch.ops.dava.l1_camera_vjp(*args, ge, None, False) + torch.ops.dava.l1_camera_vjp(
                *args, None, gg, True)
        else:
            vjp = torch.ops.dava.l1_camera_vjp(*args, ge, gg, bool(detach_points and gg is not None))
        b, e, m = trans.shape[0], trans.shape[1], trans.shape[2]
        n2 = world.shape[2]
        d_f, d_cx, d_cy, d_t, d_l, d_w = torch.split(vjp, [1, 1, 1, 3 * m, 3 * m, 3 * n2], dim=-1)
        return (None, None, None, d_f.reshape(b, e), d_cx.reshape(b, e), d_cy.reshape(b, e), d_t.reshape(b, e, m, 3),
                d_l.reshape(b, e, m, 3), d_w.reshape(b, e, n2, 3))


class PinholeCameraModelL1(IOptimisableFunction):
    """Camera intrinsics, per-view extrinsics and world points for B x E estimates;
    true_projected_points (B, M, N, 2), visibility_mask (B, M, N)."""

    CX = 0
    CY = 1
    F = 2
    VIEW_START = 3

    def __init__(
        self,
        focal_length: torch.Tensor,
        cx: torch.Tensor,
        cy: torch.Tensor,
        translation: torch.Tensor,
        orientation: LieRotation,
        world_points: torch.Tensor,
        true_projected_points: torch.Tensor,
        visibility_mask: torch.Tensor,
        minimum_z_distance: float = 1e-3,
        maximum_pixel_ratio: float = 5.0,
        constrain: bool = False,
        max_gradient: float = -1.0,
        enable_error_gradients: bool = True,
        enable_grad_gradients: bool = True,
        _error: Optional[torch.Tensor] = None,
        _gradient: Optional[torch.Tensor] = None,
        _error_mask: Optional[torch.Tensor] = None,
        _gradient_mask: Optional[torch.Tensor] = None,
    ):
        self.minimum_z_distance = float(minimum_z_distance)
        self.maximum_pixel_ratio = 1.0 / abs(float(maximum_pixel_ratio))  # stored inverted, as the reference
        self._constrain = bool(constrain)
        self._max_gradient = float(max_gradient)
        self._num_views = true_projected_points.size(1)
        self._num_points = true_projected_points.size(2)
        self._num_estimates = focal_length.size(1)
        self._enable_error_gradients = bool(enable_error_gradients)
        self._enable_grad_gradients = bool(enable_grad_gradients)
        # the reference keeps this as an fp32 0-d tensor: its value is fp32-rounded
        self._error_scale = torch.tensor(1.0 / (self._num_views * self._num_points)).sqrt()
        self._focal_length = focal_length
        self._cx = cx
        self._cy = cy
        self._translation = translation
        self._world_points = world_points
        self._true_projected_points = true_projected_points
        self._visibility_mask = visibility_mask
        self._orientation = orientation
        self._error = _error
        self._gradient = _gradient
        self._error_mask = _error_mask
        self._gradient_mask = _gradient_mask

    # ---- IOptimisableFunction properties ----
    @property
    def batch_size(self) -> int:
        return self._true_projected_points.size(0)

    @property
    def num_estimates(self) -> int:
        return self._num_estimates

    @property
    def num_parameters(self) -> int:
        return 3 + 6 * self._num_views + 3 * self._num_points - 7

    @property
    def device(self) -> torch.device:
        return self._true_projected_points.device

    @property
    def focal_length(self) -> torch.Tensor:
        return self._focal_length

    @property
    def cx(self) -> torch.Tensor:
        return self._cx

    @property
    def cy(self) -> torch.Tensor:
        return self._cy

    # ---- evaluation (HIP) ----
    def _evaluate(self, want_error: bool, want_gradient: bool, detach_points: Optional[bool] = None):
        N.require_device_tensor(self._focal_length, "focal_length")
        inputs = (self._focal_length, self._cx, self._cy, self._translation, self._orientation.lie_vector,
                  self._world_points)
        differentiable = torch.is_grad_enabled() and any(t.requires_grad for t in inputs)
        dt = self._focal_length.dtype
        for t in inputs[1:] + (self._true_projected_points,):
            dt = torch.promote_types(dt, t.dtype)  # the dtype the reference's expressions produce
        if not dt.is_floating_point:
            dt = torch.get_default_dtype()
        if dt not in (torch.float32, torch.float64):
            raise TypeError("PinholeCameraModelL1 evaluates in float32 or float64")
        b, e, m, n = self.batch_size, self.num_estimates, self._num_views, self._num_points
        dev = self.device
        cast = lambda t: _c(t.to(device=dev, dtype=dt))  # noqa: E731  (differentiable when needed)
        focal = cast(self._focal_length).reshape(b, e)
        cx = cast(self._cx).reshape(b, e)
        cy = cast(self._cy).reshape(b, e)
        trans = cast(self._translation).reshape(b, e, m, 3)
        lie = cast(self._orientation.lie_vector).reshape(b, e, m, 3)
        world = cast(self._world_points).reshape(b, e, n - 2, 3)
        target = cast(self._true_projected_points.detach()).reshape(b, m, n, 2)
        vis = _c(self._visibility_mask.detach().to(device=dev, dtype=torch.uint8)).reshape(b, m, n)
        fixed = (target, vis, float(self.minimum_z_distance), float(self.maximum_pixel_ratio),
                 float(self._max_gradient), float(self._error_scale.item()),
                 (not self._enable_grad_gradients) if detach_points is None else bool(detach_points))
        if differentiable:
            err, grad = _L1Evaluate.apply(fixed, bool(want_error), bool(want_gradient), focal, cx, cy, trans, lie,
                                          world)
            if not self._enable_error_gradients:
                err = err.detach()  # the reference detaches u, v (:139-141)
        else:
            err, grad = torch.ops.dava.l1_camera_evaluate(focal.detach(), cx.detach(), cy.detach(), trans.detach(),
                                                          lie.detach(), world.detach(), *fixed[:6],
                                                          bool(want_error), bool(want_gradient))
        if want_error and torch.is_grad_enabled() and self._true_projected_points.requires_grad:
            err = err + self._target_term(dt)
        err = err if want_error else None
        grad = grad if want_gradient else None
        return err, grad

    def _target_term(self, dt: torch.dtype) -> torch.Tensor:
        """A zero-valued (B, E) term whose gradient w.r.t. true_projected_points is the reference error's
        (``:139-150``): d/dt sum scale |(u - t) vis| = -scale sgn((u - t) vis) vis (torch.abs backward, 0 at 0).
        u, v come from the reference's own torch expressions (``_get_u`` / ``_get_v``, ``:467-496``); the error's
        value stays the kernel's.  (The hand-written gradient depends on t only through sign(), whose derivative
        is 0, as in the reference.)"""
        t = self._true_projected_points.to(dt)
        with torch.no_grad():
            rel = self._get_camera_relative_points().to(dt)
            f = self._focal_length.to(dt).reshape(self.batch_size, self.num_estimates, 1, 1)
            u = f * rel[..., 0] / rel[..., 2] + self._cx.to(dt).reshape(f.shape)
            v = f * rel[..., 1] / rel[..., 2] + self._cy.to(dt).reshape(f.shape)
            vis = self._visibility_mask.to(dt)[:, None, :, :]
            scale = self._error_scale.to(dt)
            su = scale * torch.sign((u - t[:, None, :, :, 0]) * vis) * vis
            sv = scale * torch.sign((v - t[:, None, :, :, 1]) * vis) * vis
        term = -(su * t[:, None, :, :, 0] + sv * t[:, None, :, :, 1]).sum(dim=(-2, -1))
        return term - term.detach()

    def get_error(self) -> torch.Tensor:
        """Total L1 reprojection error per estimate, (B, E) (``:132-190``)."""
        if self._error is None or self._error_mask is not None:
            err, _ = self._evaluate(True, False)
            if self._error is not None:  # keep the still-valid values, as the reference's partial recompute
                err = torch.where(self._error_mask, self._error, err)
            self._error = err
            self._error_mask = None
        return self._error

    def get_gradient(self) -> torch.Tensor:
        """The reference's hand-written gradient per estimate, (B, E, P) (``:192-285``)."""
        if self._gradient is None or self._gradient_mask is not None:
            # the reference's partial recompute (:223-270) applies no enable_grad_gradients detach
            _, grad = self._evaluate(False, True, detach_points=False if self._gradient is not None else None)
            if self._gradient is not None:
                grad = torch.where(self._gradient_mask.unsqueeze(-1), self._gradient, grad)
            self._gradient = grad
            self._gradient_mask = None
        return self._gradient

    def as_parameters_vector(self) -> torch.Tensor:
        """(B, E, P) in the layout ``add`` consumes.  (The reference's version (``:316-339``)
        concatenates (B, E) and (B, E, M, ...) tensors and repeats ty where tz belongs, so it
        cannot run for its own tensor shapes; this returns the vector it describes.)"""
        b, e, m = self.batch_size, self.num_estimates, self._num_views
        ov = self._orientation.as_parameters_vector().reshape(b, e, m, 3)
        tr = self._translation.reshape(b, e, m, 3)
        wp = self._world_points
        return torch.cat([
            self.cx.reshape(b, e, 1), self.cy.reshape(b, e, 1), self.focal_length.reshape(b, e, 1),
            ov[..., 0], ov[..., 1], ov[..., 2], tr[..., 0], tr[..., 1], tr[..., 2],
            wp[:, :, :, 0], wp[:, :, :, 1], wp[:, :, 1:, 2],
        ], dim=-1)

    def add(self, parameters: torch.Tensor) -> "PinholeCameraModelL1":
        """A new model at the current parameters + ``parameters`` (B, E, P) (``:346-404``)."""
        m, n = self._num_views, self._num_points
        a_idx = self.VIEW_START
        b_idx, c_idx = a_idx + m, a_idx + 2 * m
        tx_idx, ty_idx, tz_idx = a_idx + 3 * m, a_idx + 4 * m, a_idx + 5 * m
        x_idx = a_idx + 6 * m
        y_idx = x_idx + n - 2
        z_idx = y_idx + n - 2
        end_idx = z_idx + n - 3
        t_params = torch.stack([parameters[:, :, tx_idx:ty_idx], parameters[:, :, ty_idx:tz_idx],
                                parameters[:, :, tz_idx:x_idx]], dim=-1)
        z_params = parameters[:, :, z_idx:end_idx]
        z_params = torch.cat([torch.zeros_like(z_params[:, :, 0:1]), z_params], dim=-1)
        point_params = torch.stack([parameters[:, :, x_idx:y_idx], parameters[:, :, y_idx:z_idx], z_params], dim=-1)
        new_orientation = self._orientation.add_lie_parameters(
            torch.stack([parameters[:, :, a_idx:b_idx], parameters[:, :, b_idx:c_idx],
                         parameters[:, :, c_idx:tx_idx]], dim=-1).unsqueeze(-2),
            constrain=self._constrain)
        new_f = self._focal_length + parameters[:, :, self.F]
        new_cx = self._cx + parameters[:, :, self.CX]
        new_cy = self._cy + parameters[:, :, self.CY]
        if self._constrain:
            new_f = new_f.clamp(min=self.maximum_pixel_ratio, max=1e3)
            new_cx = new_cx.clamp(min=-1.0, max=1.0)
            new_cy = new_cy.clamp(min=-1.0, max=1.0)
        return type(self)(
            focal_length=new_f, cx=new_cx, cy=new_cy, translation=self._translation + t_params,
            orientation=new_orientation, world_points=self._world_points + point_params,
            true_projected_points=self._true_projected_points, visibility_mask=self._visibility_mask,
            minimum_z_distance=self.minimum_z_distance, constrain=self._constrain, max_gradient=self._max_gradient,
            enable_error_gradients=self._enable_error_gradients, enable_grad_gradients=self._enable_grad_gradients)

    def masked_update(self, other: "PinholeCameraModelL1", mask: torch.Tensor) -> "PinholeCameraModelL1":
        """Take ``other``'s values where ``mask`` (B, E) is true (``:406-460``)."""
        if other._true_projected_points is not self._true_projected_points:
            raise ValueError("Can only do masked update between instances targeting the same points")
        focal = torch.where(mask, other._focal_length, self._focal_length)
        cx = torch.where(mask, other._cx, self._cx)
        cy = torch.where(mask, other._cy, self._cy)
        vector_mask = mask[:, :, None, None].tile(1, 1, self._translation.size(2), self._translation.size(3))
        orientation = self._orientation.masked_update(other._orientation, vector_mask.unsqueeze(-2))
        translation = torch.where(vector_mask, other._translation, self._translation)
        if other._world_points is self._world_points:
            world_points = self._world_points
        else:
            world_mask = mask[:, :, None, None].tile(1, 1, *self._world_points.shape[2:])
            world_points = torch.where(world_mask, other._world_points, self._world_points)
        error, error_mask = merge_cached_values(self._error, self._error_mask, other._error, other._error_mask, mask)
        gradient, gradient_mask = merge_cached_values(self._gradient, self._gradient_mask, other._gradient,
                                                       other._gradient_mask, mask)
        return type(self)(
            focal_length=focal, cx=cx, cy=cy, translation=translation, orientation=orientation,
            world_points=world_points, true_projected_points=self._true_projected_points,
            visibility_mask=self._visibility_mask, minimum_z_distance=self.minimum_z_distance,
            constrain=self._constrain, max_gradient=self._max_gradient,
            enable_error_gradients=self._enable_error_gradients, enable_grad_gradients=self._enable_grad_gradients,
            _error=error, _error_mask=error_mask, _gradient=gradient, _gradient_mask=gradient_mask)

    # ---- the reference's private views, for callers / tests that use them ----
    def _get_world_points(self) -> torch.Tensor:
        """(B, E, N, 3) with the gauge points (0,0,0), (1,0,0), (x, y, 0) prepended (``:405-432``)."""
        first_two = torch.zeros(self.batch_size, self.num_estimates, 2, 3, device=self._world_points.device,
                                dtype=self._world_points.dtype)
        first_two[:, :, 1, 0] = 1.0
        third = torch.cat([self._world_points[:, :, 0:1, 0:2], torch.zeros_like(self._world_points[:, :, 0:1, 2:3])],
                          dim=-1)
        return torch.cat([first_two, third, self._world_points[:, :, 1:, :]], dim=2)

    def _get_camera_relative_points(self) -> torch.Tensor:
        """(B, E, M, N, 3) with z clamped in front of the camera (``:434-466``)."""
        rotated = self._orientation.rotate_vector(self._get_world_points()[:, :, None, :, :])
        rotated = rotated + self._translation[:, :, :, None, :]
        min_z = (self.maximum_pixel_ratio * rotated[..., 0:2]).abs().max(dim=-1).values
        min_z = torch.clamp(min_z, min=self.minimum_z_distance)
        return torch.cat([rotated[..., 0:2], torch.maximum(rotated[..., 2:3], min_z.unsqueeze(-1))], dim=-1)
