"""``BFGSCameraSolver`` (reference: ``solvers/bfgs_camera_solver.py:13-95``).

BFGS over an :class:`IOptimisableFunction` holding B x E estimates: per iteration the search
direction -H g (HIP ``search_direction``), the reference's max/min step clamp, the line search
(a module, normally :class:`LineSearchStrongWolfeConditions`), then H0 = (s.y / max(y.y, 1e-5)) I
on the first iteration (N&W 6.20, no lower clamp in this legacy variant) and the rank-2 update
(HIP ``update_inverse_hessian``, the same formula as ``BFGSSolver``).  Estimates keep updating
while their error exceeds ``epsilon`` (an fp32 constant, as in the reference).
"""
from typing import Optional

import torch
import torch.nn as nn

from .. import native_ops
from .i_optimisable_function import IOptimisableFunction


def clamp_search_direction(search_direction: torch.Tensor, max_step_length: float,
                           min_step_length: float) -> torch.Tensor:
    """Rescale each direction so its largest component lies in [min, max] (``:98-112``)."""
    largest = search_direction.abs().max(dim=-1).values.clamp(min=1e-8)
    scale = torch.ones_like(largest)
    too_large = largest > max_step_length
    too_small = largest < min_step_length
    scale[too_large] = max_step_length / largest[too_large]
    scale[too_small] = min_step_length / largest[too_small]
    return scale.clamp(min=1e-16)[:, :, None] * search_direction


def estimate_initial_inverse_hessian(ndim: int, step: torch.Tensor, delta_gradient: torch.Tensor) -> torch.Tensor:
    """H0 = (s.y / clamp(y.y, 1e-5)) I per estimate (``:115-131``)."""
    denominator = delta_gradient.square().sum(dim=-1).clamp(min=1e-5)
    gamma = (step * delta_gradient).sum(dim=-1) / denominator
    return gamma[:, :, None, None] * torch.eye(ndim, device=step.device, dtype=step.dtype).reshape(1, 1, ndim, ndim)


class BFGSCameraSolver(nn.Module):
    def __init__(self, max_iterations: int, epsilon: float, max_step_distance: float, min_step_distance: float,
                 line_search: nn.Module, search_direction_network: Optional[nn.Module] = None):
        super().__init__()
        self.line_search = line_search
        self.search_direction_network = search_direction_network
        self.max_iterations = int(max_iterations)
        self.epsilon = torch.tensor(float(epsilon))
        self.max_step_distance = float(max_step_distance)
        self.min_step_distance = float(min_step_distance)

    def forward(self, function: IOptimisableFunction) -> IOptimisableFunction:
        h = None
        updating = torch.ones(function.batch_size, function.num_estimates, device=function.device, dtype=torch.bool)
        for it in range(self.max_iterations):
            g = function.get_gradient()
            d = -1.0 * g if it == 0 else native_ops.search_direction(h, g)
            d = clamp_search_direction(d, self.max_step_distance, self.min_step_distance)
            if self.search_direction_network is not None:
                d = self.search_direction_network(d, function.as_parameters_vector(), function.get_error(), it)
            next_fn, step = self.line_search(function, d)
            dg = next_fn.get_gradient() - g
            if it == 0:
                h = estimate_initial_inverse_hessian(g.size(2), step, dg)
            h = native_ops.update_inverse_hessian(h, step, dg)
            function = function.masked_update(next_fn, updating)
            updating = updating & torch.greater(function.get_error(), self.epsilon)
        return function
