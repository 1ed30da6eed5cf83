"""Bookkeeping helpers of the legacy ``IOptimisableFunction`` path (host-side tensor plumbing, no math
on the hot path).  Behaviour follows the reference's ``utils/masked_merge.py:4-60`` and
``utils/func_interpolate_alpha.py``; the formulation here is this project's own."""
from typing import Optional, Tuple

import torch


def merge_cached_values(
    values_1: Optional[torch.Tensor],
    valid_1: Optional[torch.Tensor],
    values_2: Optional[torch.Tensor],
    valid_2: Optional[torch.Tensor],
    take_second: torch.Tensor,
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Merge two per-estimate caches (e.g. a function's error or gradient) by selector.

    Each cache is ``(values, valid)``: ``values`` None = nothing cached; ``valid`` None = every
    cached row is valid, else a bool tensor over the leading (selector-shaped) dimensions.  Row
    ``i`` of the result comes from cache 2 where ``take_second[i]`` and from cache 1 elsewhere, and
    is valid iff the row it came from was.  A side with no values contributes no valid rows, and
    the result's values are then the other side's tensor as-is.  Returns ``(values, valid)``,
    ``valid`` None when every row is valid because both sides were fully valid."""
    if values_1 is None and values_2 is None:
        return None, None
    if values_1 is None or values_2 is None:
        present_is_2 = values_1 is None
        values = values_2 if present_is_2 else values_1
        own = valid_2 if present_is_2 else valid_1
        rows = take_second if present_is_2 else ~take_second
        return values, (rows if own is None else own & rows)
    selector = take_second.reshape(take_second.shape + (1,) * (values_1.ndim - take_second.ndim))
    values = torch.where(selector, values_2, values_1)
    if valid_1 is None and valid_2 is None:
        return values, None
    all_rows = torch.ones_like(take_second)
    return values, torch.where(take_second, all_rows if valid_2 is None else valid_2,
                               all_rows if valid_1 is None else valid_1)


class _SecantAlpha(torch.autograd.Function):
    """Secant root with a gradient that stays finite (the reference's ``InterpolateAlpha``,
    ``utils/func_interpolate_alpha.py:5-79``): rows that fall back to the midpoint pass half the
    gradient to each bracket end and none to the values; secant rows get the root's exact partials,
    written in the reference's factor order.  Plain autograd through ``torch.where`` would form
    ``0 * inf`` in the unused branch of a flat row (equal slopes, which the legacy L1 gradient's
    sign / clipping terms make common) and spread NaN to shared parameters."""

    @staticmethod
    def forward(ctx, alpha_1, alpha_2, value_1, value_2):
        low = torch.minimum(alpha_1, alpha_2)
        high = torch.maximum(alpha_1, alpha_2)
        rise = value_2 - value_1
        run_over_rise = (alpha_2 - alpha_1) / rise
        root = alpha_1 - value_1 * run_over_rise
        midpoint = (rise == 0.0) | (root < low + 1e-3) | (root > high - 1e-3)
        inv_rise = torch.where(midpoint, torch.zeros_like(rise), 1.0 / rise)
        ctx.save_for_backward(value_1, value_2, inv_rise, run_over_rise, midpoint)
        ctx.set_materialize_grads(False)
        return torch.where(midpoint, (alpha_1 + alpha_2) / 2.0, root)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        if grad is None:
            return None, None, None, None
        value_1, value_2, inv_rise, run_over_rise, midpoint = ctx.saved_tensors
        half = 0.5 * grad
        zero = torch.zeros_like(grad)
        need = ctx.needs_input_grad
        return (
            torch.where(midpoint, half, inv_rise * value_2 * grad) if need[0] else None,
            torch.where(midpoint, half, -1.0 * inv_rise * value_1 * grad) if need[1] else None,
            torch.where(midpoint, zero, -1.0 * value_2 * run_over_rise * inv_rise * grad) if need[2] else None,
            torch.where(midpoint, zero, value_1 * run_over_rise * inv_rise * grad) if need[3] else None,
        )


def secant_alpha(alpha_1: torch.Tensor, alpha_2: torch.Tensor, value_1: torch.Tensor,
                 value_2: torch.Tensor) -> torch.Tensor:
    """Step length where the straight line through ``(alpha_1, value_1)`` and ``(alpha_2, value_2)``
    crosses zero (the legacy zoom interpolates the directional derivative this way).  Where the
    line is flat, or its root is not at least 1e-3 inside the bracket, the bracket's midpoint is
    used instead.  A NaN root is kept, as the reference does (its comparisons with NaN are false).
    Differentiable with the reference's custom backward (see ``_SecantAlpha``)."""
    return _SecantAlpha.apply(alpha_1, alpha_2, value_1, value_2)
