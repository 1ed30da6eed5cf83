"""Taylor-branched trigonometric ratios (oracle restatement, test infrastructure only).

Each function reproduces the forward value AND the hand-written backward
formula of the reference's custom ``torch.autograd.Function`` so that
autograd through the oracle rounds exactly like autograd through the
reference:

* ``sinc``            -- ``utils/func_sin_x_on_x.py:5-41``       (|x| < 0.01 series)
* ``sinc_slope``      -- ``utils/func_sin_x_on_x.py:44-98``      (|x| < 0.01 series)
                        i.e. cos(x)/x^2 - sin(x)/x^3
* ``versine_ratio``   -- ``utils/func_one_minus_cos_x_on_x_squared.py:6-51`` (|x| < 0.05)
                        i.e. (1 - cos x)/x^2
* ``curvature_reciprocal`` -- ``utils/func_inverse_curvature.py:21-51``
"""
import torch

SINC_SERIES_BELOW = 0.01
SINC_SLOPE_SERIES_BELOW = 0.01
VERSINE_SERIES_BELOW = 0.05


def _sinc_value(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(x)
    small = x.abs() < SINC_SERIES_BELOW
    large = ~small
    xs = x[small]
    x2 = xs.square()
    x4 = x2.square()
    x6 = x4 * x2
    out[small] = 1.0 - x2 / 6.0 + x4 / 120 - x6 / 5040
    xl = x[large]
    out[large] = torch.sin(xl) / xl
    return out


def _sinc_slope_value(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(x)
    small = x.abs() < SINC_SLOPE_SERIES_BELOW
    large = ~small
    x2 = x.square()
    x2s = x2[small]
    x4 = x2s.square()
    x6 = x4 * x2s
    out[small] = -1.0 / 3.0 + x2s / 30.0 - x4 / 840 + x6 / 45360
    xl = x[large]
    c = torch.cos(xl)
    s = torch.sin(xl)
    x3 = xl * x2[large]
    out[large] = c / x2[large] - s / x3
    return out


def _safe_reciprocal(x: torch.Tensor) -> torch.Tensor:
    r = 1 / x
    r[x == 0] = 0.0
    return r


class _Sinc(torch.autograd.Function):
    """``SinXonX`` (func_sin_x_on_x.py:5-41): backward grad * x * sinc_slope(x)."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        ctx.set_materialize_grads(False)
        return _sinc_value(x)

    @staticmethod
    def backward(ctx, grad):
        if grad is None:
            return None
        (x,) = ctx.saved_tensors
        return grad * x * sinc_slope(x)


class _SincSlope(torch.autograd.Function):
    """``CosXonXSquaredMinusSinXonXCubed`` (func_sin_x_on_x.py:44-98): returns the value and
    1/x (0 at 0) as a second output, and differentiates both like the reference, so that
    second derivatives (differentiating through the solve) round the same way."""

    @staticmethod
    def forward(ctx, x):
        out = _sinc_slope_value(x)
        recip = _safe_reciprocal(x)
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
            g = -1.0 * grad * recip * (sinc(x) + 3.0 * out)
        if grad_recip is not None:
            g = g - grad_recip * recip * recip
        return g


class _VersineRatio(torch.autograd.Function):
    """``OneMinusCosXonXsquared`` (func_one_minus_cos_x_on_x_squared.py:6-51), value and 1/x."""

    @staticmethod
    def forward(ctx, x):
        out = torch.empty_like(x)
        small = x.abs() < VERSINE_SERIES_BELOW
        large = ~small
        x2 = x.square()
        x2s = x2[small]
        x4 = x2s.square()
        x6 = x4 * x2s
        out[small] = 0.5 - x2s / 24 + x4 / 720 - x6 / 40320
        out[large] = (1.0 - torch.cos(x[large])) / x2[large]
        recip = _safe_reciprocal(x)
        ctx.save_for_backward(x, out, recip)
        ctx.set_materialize_grads(False)
        return out, recip

    @staticmethod
    def backward(ctx, grad, grad_recip):
        if grad is None:
            return None
        x, out, recip = ctx.saved_tensors
        g = grad * recip * (sinc(x) - 2.0 * out)
        if grad_recip is not None:
            g = g - grad_recip * recip * recip
        return g


def sinc(x: torch.Tensor) -> torch.Tensor:
    """sin(x)/x with the reference's series branch and backward."""
    return _Sinc.apply(x)


def sinc_slope(x: torch.Tensor) -> torch.Tensor:
    """cos(x)/x^2 - sin(x)/x^3 with the reference's series branch and backward."""
    return _SincSlope.apply(x)[0]


def versine_ratio(x: torch.Tensor) -> torch.Tensor:
    """(1 - cos x)/x^2 with the reference's series branch and backward."""
    return _VersineRatio.apply(x)[0]


class _InverseCurvature(torch.autograd.Function):
    """1 / (s.y), 0 where s.y <= 0, with the reference's custom backward
    (``utils/func_inverse_curvature.py:21-51``: grad * -r * r, times y or s)."""

    @staticmethod
    def forward(ctx, step, delta_gradient):
        curvature = torch.sum(step * delta_gradient, dim=-1, keepdim=True)
        inv = 1.0 / curvature
        inv[curvature <= 0.0] = 0.0
        ctx.save_for_backward(step, delta_gradient, inv)
        return inv

    @staticmethod
    def backward(ctx, grad_output):
        step, delta_gradient, inv = ctx.saved_tensors
        grad_output = -1.0 * inv * inv * grad_output
        return delta_gradient * grad_output, step * grad_output


def curvature_reciprocal(step: torch.Tensor, delta_gradient: torch.Tensor) -> torch.Tensor:
    """1 / (s.y), forced to 0 where s.y <= 0 (``func_inverse_curvature.py:24-28``), differentiable
    like the reference's ``InverseCurvature`` when the solve is differentiated through."""
    return _InverseCurvature.apply(step, delta_gradient)
