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
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return _sinc_value(x)

    @staticmethod
    def backward(ctx, grad):
        (x,) = ctx.saved_tensors
        return grad * x * _sinc_slope_value(x)


class _VersineRatio(torch.autograd.Function):
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
        ctx.save_for_backward(x, out, _safe_reciprocal(x))
        return out

    @staticmethod
    def backward(ctx, grad):
        x, out, recip = ctx.saved_tensors
        return grad * recip * (_sinc_value(x) - 2.0 * out)


def sinc(x: torch.Tensor) -> torch.Tensor:
    """sin(x)/x with the reference's series branch and backward."""
    return _Sinc.apply(x)


def versine_ratio(x: torch.Tensor) -> torch.Tensor:
    """(1 - cos x)/x^2 with the reference's series branch and backward."""
    return _VersineRatio.apply(x)


def curvature_reciprocal(step: torch.Tensor, delta_gradient: torch.Tensor) -> torch.Tensor:
    """1 / (s.y), forced to 0 where s.y <= 0 (func_inverse_curvature.py:24-28).

    The oracle never differentiates through the solve, so no custom backward.
    """
    curv = (step * delta_gradient).sum(dim=-1, keepdim=True)
    out = 1.0 / curv
    out[curv <= 0.0] = 0.0
    return out
