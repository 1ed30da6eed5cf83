"""Small tensor utilities of the legacy solver path (``utils/masked_merge.py``,
``utils/func_interpolate_alpha.py``)."""
from typing import Optional, Tuple

import torch


def masked_merge_tensors(
    values_1: Optional[torch.Tensor],
    mask_1: Optional[torch.Tensor],
    values_2: Optional[torch.Tensor],
    mask_2: Optional[torch.Tensor],
    update_mask: torch.Tensor,
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Values from 1 where ``update_mask`` is false, from 2 where true, with the merged
    validity mask (None = all valid), exactly as ``utils/masked_merge.py``."""
    if values_1 is None and values_2 is None:
        return None, None
    if values_1 is not None and values_2 is not None:
        vmask = update_mask
        if update_mask.ndim < values_1.ndim:
            vmask = update_mask.reshape(*update_mask.shape, *(1 for _ in range(values_1.ndim - update_mask.ndim)))
            vmask = vmask.tile(*(1 for _ in range(update_mask.ndim)), *values_1.shape[update_mask.ndim:])
        merged = torch.where(vmask, values_2, values_1)
        if mask_1 is None and mask_2 is None:
            return merged, None
        if mask_1 is not None and mask_2 is not None:
            return merged, torch.where(update_mask, mask_2, mask_1)
        if mask_1 is not None:
            return merged, torch.logical_or(mask_1, update_mask)
        return merged, torch.logical_or(mask_2, torch.logical_not(update_mask))
    if values_1 is not None:
        if mask_1 is not None:
            return values_1, torch.logical_and(mask_1, torch.logical_not(update_mask))
        return values_1, torch.logical_not(update_mask)
    if mask_2 is not None:
        return values_2, torch.logical_and(mask_2, update_mask)
    return values_2, update_mask


def interpolate_alpha(alpha_1: torch.Tensor, alpha_2: torch.Tensor, value_1: torch.Tensor,
                      value_2: torch.Tensor) -> torch.Tensor:
    """Secant step to the zero of a value between two alphas, falling back to bisection when
    the values are equal or the candidate is within 1e-3 of (or outside) the bracket."""
    min_alpha = torch.minimum(alpha_1, alpha_2)
    max_alpha = torch.maximum(alpha_1, alpha_2)
    value_diff = value_2 - value_1
    inv_gradient = (alpha_2 - alpha_1) / value_diff
    candidate = alpha_1 - value_1 * inv_gradient
    non_linear = torch.logical_or(torch.eq(value_diff, 0.0),
                                  torch.logical_or(torch.less(candidate, min_alpha + 1e-3),
                                                   torch.greater(candidate, max_alpha - 1e-3)))
    candidate[non_linear] = (alpha_1[non_linear] + alpha_2[non_linear]) / 2.0
    return candidate
