"""Legacy ``PinholeCameraModelL1`` error and hand-written gradient (oracle restatement,
test infrastructure only).

Restates ``camera_model/pinhole_camera_model_l1.py`` (get_error :132-190, get_gradient
:192-285, _get_world_points :405-432, _get_camera_relative_points :434-466, _get_u/_get_v
:468-500, _compute_gradient_from_intermediates :529-642, _stack_gradients :645-712) and the
``geometry/lie_rotation.py`` pieces it uses (rotate_vector, parameter_gradient,
vector_gradient), in the same op order, so values are bitwise equal to the reference's
(``tests/test_oracle_golden.py``).  Plain tensors instead of objects: focal, cx, cy (B, E);
translation (B, E, M, 3); lie (B, E, M, 1, 3); world (B, E, N-2, 3); true (B, M, N, 2);
vis (B, M, N).
"""
import torch

from .trig import sinc, sinc_slope, versine_ratio


def _d_term_value(x: torch.Tensor) -> torch.Tensor:
    near = torch.less(x.abs(), 0.25)
    far = torch.logical_not(near)
    out = torch.empty_like(x)
    x2 = x.square()
    x4 = x2.square()
    x6 = x4[near] * x2[near]
    out[near] = -1.0 / 12.0 + x2[near] / 180.0 - x4[near] / 6720.0 + x6 / 362880.0
    s = torch.sin(x[far])
    c = torch.cos(x[far])
    x3 = x[far] * x2[far]
    out[far] = s / x3 - 2.0 * (1.0 - c) / x4[far]
    return out


class _DTerm(torch.autograd.Function):
    """``SinXonXCubedMinusTwoOneMinusCosXonXFourth`` (:6-58): backward grad (C(x) - 4 D(x)) / x,
    1/x taken as 0 at 0."""

    @staticmethod
    def forward(ctx, x):
        out = _d_term_value(x)
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, grad):
        x, out = ctx.saved_tensors
        recip = 1 / x
        recip[x == 0] = 0.0
        return grad * recip * (sinc_slope(x) - 4.0 * out)


def _d_term(x: torch.Tensor) -> torch.Tensor:
    """sin x / x^3 - 2 (1 - cos x) / x^4, series below 0.25
    (``utils/func_sin_x_on_x_cubed_minus_two_one_minus_cos_x_on_x_fourth.py:8-40``), with the
    reference's backward."""
    return _DTerm.apply(x)


def world_points(world: torch.Tensor) -> torch.Tensor:
    b, e = world.shape[:2]
    first_two = torch.zeros(b, e, 2, 3, dtype=world.dtype)
    first_two[:, :, 1, 0] = 1.0
    third = torch.cat([world[:, :, 0:1, 0:2], torch.zeros_like(world[:, :, 0:1, 2:3])], dim=-1)
    return torch.cat([first_two, third, world[:, :, 1:, :]], dim=2)


def _rotate(lie, v):
    angle = torch.linalg.norm(lie, dim=-1, keepdim=True)
    dot = (v * lie).sum(dim=-1, keepdims=True)
    cross = torch.linalg.cross(lie, v, dim=-1)
    return v * torch.cos(angle) + versine_ratio(angle) * dot * lie + cross * sinc(angle)


def _parameter_gradient(lie, v):
    angle = torch.linalg.norm(lie, dim=-1, keepdim=True)
    s_on = sinc(angle)
    vers = versine_ratio(angle)
    c_term = sinc_slope(angle)
    d_term = _d_term(angle)
    dot = (v * lie).sum(dim=-1, keepdims=True)
    cross = torch.linalg.cross(lie, v, dim=-1)
    outer = lie.unsqueeze(-2) * v.unsqueeze(-1)
    axis_outer = lie.unsqueeze(-2) * lie.unsqueeze(-1)
    axis_cross_outer = lie.unsqueeze(-2) * cross.unsqueeze(-1)
    term_1 = -1.0 * outer * s_on.unsqueeze(-1)
    term_2 = (dot * d_term).unsqueeze(-1) * axis_outer
    term_3 = dot.unsqueeze(-1) * torch.eye(3)
    term_3 = vers.unsqueeze(-1) * (torch.transpose(outer, -2, -1) + term_3)
    term_4 = axis_cross_outer * c_term.unsqueeze(-1)
    x = v[..., 0:1]
    y = v[..., 1:2]
    z = v[..., 2:3]
    zeros = torch.zeros_like(x)
    term_5 = torch.stack([torch.cat([zeros, -z, y], dim=-1), torch.cat([z, zeros, -x], dim=-1),
                          torch.cat([-y, x, zeros], dim=-1)], dim=-1)
    term_5 = term_5 * s_on.unsqueeze(-1)
    return term_1 + term_2 + term_3 + term_4 + term_5


def _vector_gradient(lie):
    angle = torch.linalg.norm(lie, dim=-1, keepdim=True)
    cos_t = torch.cos(angle)
    s_on = sinc(angle)
    outer = lie.unsqueeze(-2) * lie.unsqueeze(-1)
    outer = outer * versine_ratio(angle).unsqueeze(-1)
    a = lie[..., 0:1] * s_on
    b = lie[..., 1:2] * s_on
    c = lie[..., 2:3] * s_on
    cross_d = torch.stack([torch.cat([cos_t, c, -b], dim=-1), torch.cat([-c, cos_t, a], dim=-1),
                           torch.cat([b, -a, cos_t], dim=-1)], dim=-1)
    return outer + cross_d


def camera_relative_points(translation, lie, world, minimum_z_distance=1e-3, maximum_pixel_ratio=5.0):
    ratio = 1.0 / abs(float(maximum_pixel_ratio))
    rotated = _rotate(lie, world_points(world)[:, :, None, :, :]) + translation[:, :, :, None, :]
    min_z = (ratio * rotated[:, :, :, :, 0:2]).abs().max(dim=-1).values
    min_z = torch.clamp(min_z, min=minimum_z_distance)
    return torch.cat([rotated[:, :, :, :, 0:2], torch.maximum(rotated[:, :, :, :, 2:3], min_z.unsqueeze(-1))], dim=-1)


def error_scale(num_views, num_points):
    return torch.tensor(1.0 / (num_views * num_points)).sqrt()


def uv(focal, cx, cy, p):
    u = focal.view(*focal.shape, 1, 1) * p[:, :, :, :, 0] / p[:, :, :, :, 2] + cx.view(*cx.shape, 1, 1)
    v = focal.view(*focal.shape, 1, 1) * p[:, :, :, :, 1] / p[:, :, :, :, 2] + cy.view(*cy.shape, 1, 1)
    return u, v


def l1_error(focal, cx, cy, translation, lie, world, true, vis, minimum_z_distance=1e-3, maximum_pixel_ratio=5.0):
    p = camera_relative_points(translation, lie, world, minimum_z_distance, maximum_pixel_ratio)
    u, v = uv(focal, cx, cy, p)
    scale = error_scale(true.size(1), true.size(2))
    ur = (u - true[:, None, :, :, 0]) * vis[:, None, :, :]
    vr = (v - true[:, None, :, :, 1]) * vis[:, None, :, :]
    return (scale * ur.abs()).sum(dim=(-2, -1)) + (scale * vr.abs()).sum(dim=(-2, -1))


def l1_gradient(focal, cx, cy, translation, lie, world, true, vis, minimum_z_distance=1e-3, maximum_pixel_ratio=5.0,
                max_gradient=-1.0, detach_points=False):
    """``detach_points``: the reference's enable_grad_gradients = False, which detaches the world
    points, the camera-relative points and u, v (``get_gradient`` :185-198) before the partials."""
    wp = world_points(world)
    og = _parameter_gradient(lie, (wp.detach() if detach_points else wp)[:, :, None, :, :])
    rg = _vector_gradient(lie)
    p = camera_relative_points(translation, lie, world, minimum_z_distance, maximum_pixel_ratio)
    u, v = uv(focal, cx, cy, p)
    if detach_points:
        p, u, v = p.detach(), u.detach(), v.detach()
    scale = error_scale(true.size(1), true.size(2))
    ru = scale * vis[:, None, :, :] * (u - true[:, None, :, :, 0]).sign()
    rv = scale * vis[:, None, :, :] * (v - true[:, None, :, :, 1]).sign()
    x_p, y_p, z_p = p[:, :, :, :, 0], p[:, :, :, :, 1], p[:, :, :, :, 2]
    f = focal
    while f.ndim < z_p.ndim:
        f = f.unsqueeze(-1)
    mg = max_gradient
    clip = lambda t: t.clip(min=-mg, max=mg)  # noqa: E731
    inv_z = 1.0 / z_p
    sf = (mg * inv_z).clip(max=1.0)
    mfm = (mg / f).abs()
    f_on_z = f * inv_z.clip(min=-mfm, max=mfm)
    x_on_z = x_p * inv_z
    y_on_z = y_p * inv_z
    du_dxp = clip(sf * f_on_z)
    dv_dyp = clip(sf * f_on_z)
    du_dzp = clip(-sf * f_on_z * x_on_z)
    dv_dzp = clip(-sf * f_on_z * y_on_z)
    du_df = clip(sf * x_on_z)
    dv_df = clip(sf * y_on_z)
    du_dtx = clip(sf * du_dxp)
    dv_dty = clip(sf * dv_dyp)
    du_dtz = clip(sf * du_dzp)
    dv_dtz = clip(sf * dv_dzp)

    def du_dw(j):
        return clip(sf * (du_dxp * og[:, :, :, :, 0, j] + du_dzp * og[:, :, :, :, 2, j]))

    def dv_dw(j):
        return clip(sf * (dv_dyp * og[:, :, :, :, 1, j] + dv_dzp * og[:, :, :, :, 2, j]))

    du_dx = clip(sf * (du_dxp * rg[:, :, :, :, 0, 0] + du_dzp * rg[:, :, :, :, 2, 0]))
    dv_dx = clip(sf * (dv_dyp * rg[:, :, :, :, 1, 0] + dv_dzp * rg[:, :, :, :, 2, 0]))
    du_dy = clip(sf * (du_dxp * rg[:, :, :, :, 0, 1] + dv_dzp * rg[:, :, :, :, 2, 1]))  # (sic) dv/dz'
    dv_dy = clip(sf * (dv_dyp * rg[:, :, :, :, 1, 1] + dv_dzp * rg[:, :, :, :, 2, 1]))
    du_dz = clip(sf * (du_dxp * rg[:, :, :, :, 0, 2] + du_dzp * rg[:, :, :, :, 2, 2]))
    dv_dz = clip(sf * (dv_dyp * rg[:, :, :, :, 1, 2] + dv_dzp * rg[:, :, :, :, 2, 2]))

    g_cx = ru.sum(dim=(-2, -1)).unsqueeze(-1)
    g_cy = rv.sum(dim=(-2, -1)).unsqueeze(-1)
    g_f = ((ru * du_df).sum(dim=(-2, -1)) + (rv * dv_df).sum(dim=(-2, -1))).unsqueeze(-1)
    g_abc = [(ru * du_dw(j)).sum(dim=-1) + (rv * dv_dw(j)).sum(dim=-1) for j in range(3)]
    g_tx = (ru * du_dtx).sum(dim=-1)
    g_ty = (rv * dv_dty).sum(dim=-1)
    g_tz = (ru * du_dtz).sum(dim=-1) + (rv * dv_dtz).sum(dim=-1)
    g_x = (ru[:, :, :, 2:] * du_dx[:, :, :, 2:]).sum(dim=-2) + (rv[:, :, :, 2:] * dv_dx[:, :, :, 2:]).sum(dim=-2)
    g_y = (ru[:, :, :, 2:] * du_dy[:, :, :, 2:] + rv[:, :, :, 2:] * dv_dy[:, :, :, 2:]).sum(dim=-2)
    g_z = (ru[:, :, :, 3:] * du_dz[:, :, :, 3:] + rv[:, :, :, 3:] * dv_dz[:, :, :, 3:]).sum(dim=-2)
    return torch.cat([g_cx, g_cy, g_f] + g_abc + [g_tx, g_ty, g_tz, g_x, g_y, g_z], dim=-1)


PARAMETERS = ("focal_length", "cx", "cy", "translation", "lie", "world")


def l1_autograd(parts, true, vis, enable_error_gradients=True, enable_grad_gradients=True, seed=5, weight_dtype=None,
                **kw):
    """d/d(parameters) of sum(we * error) + sum(wg * gradient) by autograd through the restatement,
    the reference's enable_* detaches applied (``get_error`` :139-141, ``get_gradient`` :185-198);
    weights from ``torch.Generator`` seed ``seed`` (drawn in ``weight_dtype``, default the
    parts' dtype), the error's drawn first.  ``parts`` maps
    PARAMETERS to tensors; returns the list of gradients in PARAMETERS order (zeros if unused)."""
    leaves = {k: parts[k].clone().requires_grad_(True) for k in PARAMETERS}
    args = [leaves[k] for k in PARAMETERS] + [true, vis]
    zkw = {k: v for k, v in kw.items() if k != "max_gradient"}
    err = l1_error(*args, **zkw)
    grad = l1_gradient(*args, max_gradient=kw.get("max_gradient", -1.0), detach_points=not enable_grad_gradients,
                       **zkw)
    gen = torch.Generator().manual_seed(seed)
    we = torch.randn(err.shape, generator=gen, dtype=weight_dtype or err.dtype).to(err.dtype)
    wg = torch.randn(grad.shape, generator=gen, dtype=weight_dtype or grad.dtype).to(grad.dtype)
    loss = (grad * wg).sum() + ((err * we).sum() if enable_error_gradients else 0.0)
    out = torch.autograd.grad(loss, [leaves[k] for k in PARAMETERS], allow_unused=True)
    return [o if o is not None else torch.zeros_like(leaves[k]) for o, k in zip(out, PARAMETERS)]
