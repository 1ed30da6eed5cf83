"""Drop-in ``BFGSSolver`` (reference: ``autograd_solvers/bfgs_solver.py:26-303``).

Same constructor keywords, defaults, ``forward(parameters, error_function)``
contract, static methods and output conventions (functional, output
``requires_grad`` iff the input's).  Two execution paths, both on the GPU:

1. **Fused** -- ``error_function`` is a :class:`ReprojectionError` (the BA
   objective of this project's hot path): the entire solve -- objective,
   gradient, inverse-Hessian updates, strong-Wolfe line search, stopping
   rules -- is ONE launch of ``dava_ba_solve`` (include/dava_ba.h).
2. **Generic closure** -- any other ``error_function(parameters, mask)``:
   the closure and ``torch.autograd.grad`` run in PyTorch on the device;
   the inverse-Hessian scale/update, search direction and the line-search
   state machine run in the library's HIP kernels.  The loop mirrors
   ``bfgs_solver.py:118-212`` including the mask contract of ``:99-104``.

Differentiating through the solve (``parameters.requires_grad``, the reference's
``create_graph`` mode, ``:85, :134, :213-215``) runs the generic loop with the
graph kept: the closure's gradient is taken with ``create_graph=True`` by
PyTorch, and every solver op (initial scale, rescale, update, search direction)
is an autograd node whose backward is a HIP kernel (csrc/bfgs_grad.hip); the
line search is detached, as in the reference.  A fused objective
(:class:`ReprojectionError`, :class:`RayAngleError`) then acts as a closure whose
double backward is the forward-over-reverse kernel (H v and the observation
cross term, csrc/ba_second_order.hip), so gradients reach captured observations.

Training mode's ``return_second_last`` runs fused too (a problem stopped by the minimum-step rule
keeps x before its last step); when the reference's scatter would have moved rows between problems
(``native_ops.second_last_moves_rows``) the solve is redone by the generic loop, which reproduces it.

CPU tensors with an ordinary closure run the generic loop on the library's host flavours of the
building blocks (csrc/bfgs_host.hip), as the reference runs wherever ``parameters`` live
(``:94-117``).  The fused objectives (:class:`ReprojectionError`, :class:`RayAngleError`) are
GPU-only and raise on CPU tensors; nothing ever falls back from the GPU to the CPU.
"""
from typing import Callable, Optional

import torch
from torch.nn import Module

from .. import _native, native_ops
from ..camera_model import ReprojectionError
from .line_search import line_search_wolfe_conditions


def _free_device_bytes(device) -> float:
    """Free memory on `device` (inf when it cannot be asked: tracing under torch.compile or fake
    tensors, where the choice must not touch the device)."""
    if device is None or device.type != "cuda" or torch.compiler.is_compiling():
        return float("inf")
    try:
        return float(torch.cuda.mem_get_info(device)[0])
    except RuntimeError:
        return float("inf")


class BFGSSolver(Module):
    """Broyden-Fletcher-Goldfarb-Shanno with a dense inverse Hessian per problem and a
    strong-Wolfe line search (Nocedal & Wright 2009, eq. 6.17, 6.20; alg. 3.5/3.6)."""

    def __init__(
        self,
        sufficient_decrease: float = 1e-4,
        curvature: float = 0.9,
        error_threshold: float = 1e-4,
        iterations: int = 1000,
        minimum_step: float = 1e-8,
        drop_path_p: float = 0.1,
        return_second_last: bool = False,
        training_iterations: int = None,
        training_error_threshold: float = None,
        hessian_mode: str = "auto",
    ):
        super().__init__()
        self.sufficient_decrease = float(sufficient_decrease)
        self.curvature = float(curvature)
        self.error_threshold = float(error_threshold)
        self.iterations = int(iterations)
        self.minimum_step = float(minimum_step)
        self.drop_path_p = float(drop_path_p)
        self.return_second_last = bool(return_second_last)
        self.training_iterations = int(training_iterations) if training_iterations is not None else self.iterations
        self.training_error_threshold = (
            float(training_error_threshold) if training_error_threshold is not None else self.error_threshold
        )
        if hessian_mode not in ("auto", "dense", "compact"):
            raise ValueError("hessian_mode must be 'auto', 'dense' or 'compact'")
        self.hessian_mode = hessian_mode
        self.last_status: Optional[torch.Tensor] = None

    # ---- public static helpers (bfgs_solver.py:217-303) ----
    @staticmethod
    def scale_initial_inverse_hessian(step: torch.Tensor, delta_gradient: torch.Tensor) -> torch.Tensor:
        return native_ops.initial_scale(step, delta_gradient)

    @staticmethod
    def update_inverse_hessian(inverse_hessian: torch.Tensor, step: torch.Tensor,
                               delta_gradient: torch.Tensor) -> torch.Tensor:
        return native_ops.update_inverse_hessian(inverse_hessian, step, delta_gradient)

    # ---- forward ----
    def forward(self, parameters: torch.Tensor,
                error_function: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]) -> torch.Tensor:
        if not isinstance(parameters, torch.Tensor) or parameters.device.type != "cpu":
            _native.require_device_tensor(parameters, "parameters")
        if isinstance(error_function, ReprojectionError) and parameters.device.type == "cpu":
            # CPU tensors: the fused objectives are GPU kernels, so the generic loop runs on the library's host
            # flavours with the objective's torch form (ReprojectionError on CPU tensors), as the reference solves
            # wherever the parameters live (bfgs_solver.py:94-117)
            self.last_status = None
            if self.training:
                return self._generic(parameters, error_function, self.training_error_threshold,
                                     self.training_iterations)
            return self._generic(parameters, error_function, self.error_threshold, self.iterations)
        if self.training:
            error_threshold, num_iterations = self.training_error_threshold, self.training_iterations
        else:
            error_threshold, num_iterations = self.error_threshold, self.iterations
        # training mode's drop path runs fused (counter-based draws, DAVA_STOP_DROP), and so does
        # return_second_last (:196-212) unless the reference's scatter would move rows between problems
        drop_p = self.drop_path_p if self.training else 0.0
        second_last = self.training and self.return_second_last
        generic_training = drop_p > 0.0 and _native.python_knob("GENERIC_TRAINING")  # torch-RNG generic loop
        if isinstance(error_function, ReprojectionError) and not generic_training:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if drop_p > 0.0 else 0  # from torch's default generator
            out = None
            if not parameters.requires_grad:
                out = self._fused(parameters, error_function, error_threshold, num_iterations, drop_p, seed,
                                  second_last)
            elif self._adjoint_available(parameters, error_function, num_iterations):
                out = self._fused_differentiable(parameters, error_function, error_threshold, num_iterations,
                                                 drop_p, seed, second_last)
            if out is not None and not (second_last and native_ops.second_last_moves_rows(self.last_status)):
                return out
            self.last_status = None  # the generic loop below has no status words
        if isinstance(error_function, ReprojectionError):
            self._check_generic_fits(parameters, num_iterations, second_last)
        return self._generic(parameters, error_function, error_threshold, num_iterations)

    # dense (B, P, P) tensors the generic loop holds at once in its first iterations: the inverse
    # Hessian, its masked gather / scatter copies and the update's temporaries (more with a graph)
    _GENERIC_FIRST_MATRICES = 8

    def _check_generic_fits(self, parameters, num_iterations, second_last=False) -> None:
        """A fused objective the fused kernels cannot take runs the generic loop, which holds the
        reference's dense (B, P, P) inverse Hessian -- and, with a graph, about three P x P tensors per
        problem per ITERATION RUN (problems usually stop long before the cap: 36-107 iterations at
        C2/C3 under the reference's defaults).  Refused up front only when even the first iterations
        cannot fit the device; a run that would fit only if it stopped early gets a warning, and the
        allocator reports an actual out-of-memory."""
        import warnings

        lead = parameters.shape[:-1]
        b = max(int(torch.tensor(lead).prod().item()) if len(lead) else 1, 1)
        p = parameters.size(-1)
        per_matrix = b * p * p * parameters.element_size()
        if parameters.requires_grad:
            what = ("differentiating through the solve (dense mode or the GENERIC_BACKWARD override)"
                    if self.hessian_mode == "dense" or _native.python_knob("GENERIC_BACKWARD")
                    else "differentiating through the solve (no fused adjoint for this shape)")
        elif second_last:
            what = "training mode's return_second_last, whose scatter moves rows between problems"
        else:
            what = "the generic loop (GENERIC_TRAINING override)"
        first = per_matrix * self._GENERIC_FIRST_MATRICES
        free = _free_device_bytes(parameters.device)
        if first > free:
            raise RuntimeError(
                f"{what} at B={b}, P={p} has no fused kernel here (the adjoint covers compact mode with "
                f"P <= 14336 and at most {self.MAX_COMPACT_ENTRIES + 1} iterations); the generic loop's dense "
                f"(B, P, P) inverse Hessian and its first temporaries alone need ~{first / 2 ** 30:.0f} GiB "
                f"against {free / 2 ** 30:.0f} GiB free. Reduce the batch.")
        cap = per_matrix * (3 * num_iterations + 2 if parameters.requires_grad else self._GENERIC_FIRST_MATRICES)
        if cap > free:
            warnings.warn(f"{what}: the generic loop needs ~{per_matrix * 3 / 2 ** 30:.1f} GiB more per iteration run "
                          f"with a graph ({free / 2 ** 30:.0f} GiB free); it fits only if the problems stop "
                          f"within ~{int((free / per_matrix - 2) / 3)} of the {num_iterations} iterations",
                          RuntimeWarning, stacklevel=3)

    def _adjoint_available(self, parameters, fn: ReprojectionError, num_iterations) -> bool:
        """Differentiating through a fused objective's solve runs the recording solve + adjoint
        kernel (compact history; P <= 14336: C1-C3 with the O(P) vectors in LDS, C5 with them in
        HBM) unless dense mode was asked for or
        the GENERIC_BACKWARD override is on (then: the generic loop, graph kept by torch; _native.debug_overrides)."""
        if self.hessian_mode == "dense" or _native.python_knob("GENERIC_BACKWARD"):
            return False
        if parameters.dtype != torch.float32 or num_iterations < 1 or num_iterations > self.MAX_COMPACT_ENTRIES + 1:
            return False
        return native_ops.solve_tape_supported(max(parameters.numel() // parameters.size(-1), 1), fn.num_views,
                                               fn.num_points, fn.distortion, num_iterations, fn.residual)

    def _fused_differentiable(self, parameters, fn: ReprojectionError, error_threshold, num_iterations, drop_p=0.0,
                              seed=0, second_last=False):
        lead = parameters.shape[:-1]
        if fn.batch_shape != lead:
            raise ValueError(f"ReprojectionError batch shape {tuple(fn.batch_shape)} != parameters {tuple(lead)}")
        x0 = parameters.reshape(-1, parameters.size(-1))
        x, status = native_ops.ba_solve_differentiable(
            x0, fn.observations.reshape(-1, fn.num_views, fn.num_points, 2),
            fn.visibility.reshape(-1, fn.num_views, fn.num_points), fn.num_views, fn.num_points, fn.distortion,
            sufficient_decrease=self.sufficient_decrease, curvature=self.curvature, error_threshold=error_threshold,
            iterations=num_iterations, minimum_step=self.minimum_step, residual=fn.residual, drop_path_p=drop_p,
            drop_seed=seed, return_second_last=second_last)
        self.last_status = status
        return x.reshape(parameters.shape)

    def _fused(self, parameters, fn: ReprojectionError, error_threshold, num_iterations, drop_p=0.0, seed=0,
               second_last=False):
        lead = parameters.shape[:-1]
        if fn.batch_shape != lead:
            raise ValueError(f"ReprojectionError batch shape {tuple(fn.batch_shape)} != parameters {tuple(lead)}")
        x0 = parameters.reshape(-1, parameters.size(-1))
        if x0.dtype != torch.float32:
            raise TypeError("the fused BA solver computes in float32")
        mode = self._resolve_mode(num_iterations, x0.size(-1), x0.shape[0], x0.device)
        x, _, status = native_ops.ba_solve(
            x0, fn.observations.reshape(-1, fn.num_views, fn.num_points, 2),
            fn.visibility.reshape(-1, fn.num_views, fn.num_points), fn.num_views, fn.num_points, fn.distortion,
            sufficient_decrease=self.sufficient_decrease, curvature=self.curvature,
            error_threshold=error_threshold, iterations=num_iterations, minimum_step=self.minimum_step,
            hessian_mode=mode, want_status=True, residual=fn.residual, drop_path_p=drop_p, drop_seed=seed,
            return_second_last=second_last)
        self.last_status = status
        return x.reshape(parameters.shape)

    MAX_COMPACT_ENTRIES = 1024  # kMaxCompactEntries in csrc/bfgs_solve.hip

    def _resolve_mode(self, num_iterations: int, p: int, batch: int = 1, device=None) -> int:
        """'auto': the compact history (exact BFGS in product form, O(k P) bytes at iteration k)
        whenever its entries fit the kernel (<= 1024) and its workspace fits the device; the dense
        P x P matrix (O(P^2) bytes per iteration) only beyond that.  The iteration CAP does not
        decide: with the reference's stopping rules problems stop long before it (reference defaults
        1e-4 / 1000 / 1e-8: 36 iterations on average at C2, 107 at C3), where compact moves a
        fraction of the dense bytes -- measured 642.6k vs 77.6k problems/s at C2 and 213.7k vs 9.3k
        at C3 (profiles/r03_defaults_c2_c3.jsonl).  Even a batch that ran every problem to
        K = 1000 would move K Pv / (2 P^2) x the dense bytes (1.27x at C2, 2.5x at C1), streamed
        at a higher fraction of the HBM peak than the dense sweep.
        Past 1025 iterations compact keeps its first 1024 updates as history and a problem still
        running at iteration 1025 folds them into the dense matrix and continues dense (the kernel's
        HYBRID form, csrc/bfgs_solve.hip fold_history): its workspace is the history plus the dense
        matrices, so 'auto' takes it while that fits and the dense mode otherwise."""
        if self.hessian_mode == "dense":
            return _native.DAVA_HESSIAN_DENSE
        if self.hessian_mode == "compact":
            return _native.DAVA_HESSIAN_COMPACT
        entries = min(max(num_iterations - 1, 1), self.MAX_COMPACT_ENTRIES)
        pv = (p + 3) // 4 * 4
        compact_bytes = batch * 2 * entries * pv * 4
        if num_iterations - 1 > self.MAX_COMPACT_ENTRIES:
            compact_bytes += batch * p * ((p + 31) // 32 * 32) * 4
        if compact_bytes > 0.9 * _free_device_bytes(device):  # e.g. B = 65536, K = 1000: 416 GB of history
            return _native.DAVA_HESSIAN_DENSE
        return _native.DAVA_HESSIAN_COMPACT

    def _generic(self, parameters, error_function, error_threshold, num_iterations):
        """The reference's loop (bfgs_solver.py:94-212) around any closure: closure + autograd in torch, every
        solver op a HIP kernel.  The active set is gathered and scattered by index (the rows of `updating`, taken
        once per use of a new active set) instead of by the reference's boolean masks: the same rows and values
        in the same order, but one host round trip where every boolean gather or masked_scatter takes one."""
        batch_dimensions = parameters.shape[:-1]
        parameter_dim = parameters.size(-1)
        device = parameters.device
        updating = torch.ones(batch_dimensions, dtype=torch.bool, device=device)
        n_total = updating.numel()
        rows = torch.arange(n_total, device=device)  # flat indices of the active problems, batch order
        rows_box = [rows]  # the closure wrapper's view of the current active rows

        def wrapped(inner_parameters: torch.Tensor, inner_mask: torch.Tensor) -> torch.Tensor:
            mask = torch.zeros((n_total,), dtype=torch.bool, device=device)
            mask[rows_box[0]] = inner_mask.reshape(-1)  # (index put: no host sync)
            return error_function(inner_parameters, mask.reshape(batch_dimensions))

        def take(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:  # t[updating], flattened as the reference's
            return t.reshape((n_total,) + t.shape[len(batch_dimensions):]).index_select(0, idx)

        def put(t: torch.Tensor, idx: torch.Tensor, v: torch.Tensor) -> torch.Tensor:  # t.masked_scatter(updating, v)
            flat = t.reshape((n_total,) + t.shape[len(batch_dimensions):])
            return flat.index_copy(0, idx, v.reshape((idx.numel(),) + flat.shape[1:])).reshape(t.shape)

        create_graph = parameters.requires_grad  # bfgs_solver.py:85
        if not create_graph:
            parameters = parameters.detach()
        step = torch.zeros_like(parameters)
        error = torch.empty(batch_dimensions, dtype=parameters.dtype, device=device)
        gradient = torch.empty_like(parameters)
        # The inverse Hessian: compact history rows on the device when no graph is kept (r06: no (B, P, P)
        # matrix, no masked gather / scatter of it; native_ops.CompactHistory), else the reference's dense
        # matrix, whose ops carry the VJP kernels the create_graph mode needs (and the host flavours on CPU).
        history = None
        if (not create_graph and device.type == "cuda" and self.hessian_mode != "dense"
                and not _native.python_knob("GENERIC_DENSE")
                and native_ops.CompactHistory.supported(parameter_dim, parameters.dtype, num_iterations - 1)):
            history = native_ops.CompactHistory(max(n_total, 1), parameter_dim, parameters.dtype, device,
                                                max_entries=num_iterations - 1)
            inverse_hessian = None
        else:
            inverse_hessian = torch.zeros(batch_dimensions + (parameter_dim, parameter_dim), dtype=parameters.dtype,
                                          device=device)
            inverse_hessian[..., range(parameter_dim), range(parameter_dim)] = 1.0
        self.last_generic_history = history
        for step_idx in range(num_iterations):
            prev_gradient = gradient
            if self.training and self.drop_path_p > 0.0:
                updating = updating & torch.greater(torch.rand_like(updating, dtype=torch.float32), self.drop_path_p)
                rows = updating.reshape(-1).nonzero().squeeze(1)
            rows_box[0] = rows
            upd_params = take(parameters, rows)
            if not upd_params.requires_grad:
                upd_params.requires_grad_(True)
            with torch.enable_grad():
                upd_error = error_function(upd_params, updating)
                (upd_grad,) = torch.autograd.grad(upd_error.sum(), upd_params, create_graph=create_graph)
            error = put(error, rows, upd_error.detach())
            gradient = put(gradient, rows, upd_grad)
            updating = updating & torch.greater(error, error_threshold)
            rows = updating.reshape(-1).nonzero().squeeze(1)
            if rows.numel() == 0:
                break
            rows_box[0] = rows
            upd_params = take(parameters, rows)
            upd_error = take(error, rows)
            upd_grad = take(gradient, rows)
            if step_idx == 0:
                direction = -1.0 * upd_grad
            elif history is not None:
                direction = history.direction(upd_grad, upd_grad - take(prev_gradient, rows), take(step, rows),
                                              rows).reshape(upd_grad.shape)
            else:
                delta = upd_grad - take(prev_gradient, rows)
                upd_h = take(inverse_hessian, rows)
                upd_step = take(step, rows)
                if step_idx == 1:
                    upd_h = native_ops.scale_matrix(native_ops.initial_scale(upd_step, delta), upd_h)
                upd_h = native_ops.update_inverse_hessian(upd_h, upd_step, delta)
                direction = native_ops.search_direction(upd_h, upd_grad)
                inverse_hessian = put(inverse_hessian, rows, upd_h)
            step_size = line_search_wolfe_conditions(
                upd_params, direction, upd_error, upd_grad, wrapped,
                sufficient_decrease=self.sufficient_decrease, curvature=self.curvature, strong=True)
            upd_step = step_size.unsqueeze(-1) * direction
            new_params = upd_params + upd_step
            step = put(step, rows, upd_step)
            if not self.training or not self.return_second_last:
                parameters = put(parameters, rows, new_params)
            updating = updating & torch.greater(torch.linalg.vector_norm(step, dim=-1), self.minimum_step)
            rows = updating.reshape(-1).nonzero().squeeze(1)
            if rows.numel() == 0:
                break
            if self.training and self.return_second_last:
                # the reference scatters the previous active set's new parameters into the smaller new active set
                # (bfgs_solver.py:208-212): masked_scatter takes new_params' leading rows, in order
                parameters = put(parameters, rows, new_params[: rows.numel()])
        return parameters if create_graph else parameters.detach()
