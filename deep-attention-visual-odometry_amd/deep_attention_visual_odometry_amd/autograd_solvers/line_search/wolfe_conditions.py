"""Drop-in ``line_search_wolfe_conditions`` (reference:
``autograd_solvers/line_search/wolfe_conditions.py:23-239``).

Same signature, argument meaning, warning and return value.  The bracketing
state machine (N&W algorithms 3.5/3.6 with bisection zoom, at most 1000
trials, result = the upper bracket) runs in HIP kernels
(``dava_wolfe_{init,propose,update}``; on CPU tensors the library's host flavours
``dava_cpu_wolfe_*``); only the caller's ``error_function`` and its derivative w.r.t.
alpha are evaluated by PyTorch, where the tensors live.
The host loop still asks "which problems are active?" once per trial, exactly
where the reference synchronises (``wolfe_conditions.py:119-121``), and gathers
the active rows by index (no further host round trips of its own).

The fused BA solver does not use this function: it runs the same state
machine inside its persistent kernel with no host round-trips.
"""
import warnings
from typing import Callable

import torch

from ... import _native
from ...native_ops import WolfeState


def line_search_wolfe_conditions(
    parameters: torch.Tensor,
    search_direction: torch.Tensor,
    base_error: torch.Tensor,
    base_gradient: torch.Tensor,
    error_function: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
    sufficient_decrease: float = 1e-4,
    curvature: float = 0.9,
    strong: bool = False,
) -> torch.Tensor:
    """Step length alpha (shape ``parameters.shape[:-1]``) satisfying the (strong) Wolfe conditions
    along ``search_direction``; 0-ish when no decrease is possible."""
    if not 0.0 < sufficient_decrease < curvature < 1.0:
        warnings.warn(
            f"Line search conditions should satisfy 0 < c1 < c2 < 1. "
            f"Got c1={sufficient_decrease} and c2={curvature}"
        )
    _native.require_host_or_device_tensor(parameters, "parameters")
    parameters = parameters.detach()
    search_direction = search_direction.detach()
    base_error = base_error.detach()
    base_gradient = base_gradient.detach()
    batch_shape = parameters.shape[:-1]

    state = WolfeState(search_direction, base_error, base_gradient)
    flat_parameters = parameters.reshape(-1, parameters.shape[-1])
    flat_direction = search_direction.reshape(-1, search_direction.shape[-1])
    for trial in range(1000):
        active = state.active()
        # the active rows, once: the trial's only host sync besides the closure's own (where the reference
        # synchronises, wolfe_conditions.py:119-121); the gathers below index with them instead of the boolean
        # mask, whose every use is another nonzero() and host round trip -- the same rows, the same values
        rows = active.nonzero().squeeze(-1)
        if rows.numel() == 0:
            break
        if trial > 0:
            state.propose()
        mask = active.reshape(batch_shape)
        alpha = state.state.index_select(0, rows)[:, WolfeState.A].clone().unsqueeze(-1).requires_grad_(True)
        with torch.enable_grad():
            err = error_function(flat_parameters.index_select(0, rows) + alpha * flat_direction.index_select(0, rows),
                                 mask)
            (slope,) = torch.autograd.grad(err.sum(), alpha)
        state.state[rows, WolfeState.F_A] = err.detach().reshape(-1).to(state.state.dtype)
        state.state[rows, WolfeState.DPHI_A] = slope.detach().reshape(-1).to(state.state.dtype)
        state.update(trial, sufficient_decrease, curvature, strong)
    return state.state[:, WolfeState.A_HI].clone().reshape(batch_shape)
