"""The C ABI (include/dava_ba.h) registered as PyTorch operators: ``torch.ops.dava.*``.

Every HIP entry point of ``libdava_ba.so`` is a ``torch.library`` custom op with a
fake (meta) implementation, so ``torch.compile`` and FakeTensor tracing see opaque
operators with known output shapes and dtypes (no graph break at a ctypes call),
and eager calls dispatch straight to the HIP launch on the tensor's current stream.

The ops are registered for the ``cuda`` (= ROCm/HIP) dispatch key only: a CPU tensor
reaching one of them raises ``NotImplementedError`` from the dispatcher -- there is no
CPU kernel and no fallback.  Outputs a caller did not ask for come back as empty
(numel 0) tensors so every op has a fixed schema; ``native_ops`` maps them to None.
Ops never alias or mutate their inputs, except the Wolfe state machine's
``state``/``flags`` (declared in ``mutates_args``) and a caller-supplied workspace.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _native as N

_CUDA = "cuda"
_POISON = N._DEBUG_ENV and bool(__import__("os").environ.get("DAVA_POISON_SCRATCH"))  # NaN-filled tapes (diagnostics)


def _dt(t: Tensor) -> str:
    if t.dtype == torch.float32:
        return "f32"
    if t.dtype == torch.float64:
        return "f64"
    raise TypeError(f"unsupported dtype {t.dtype}: the HIP kernels implement float32 and float64")


def _empty0(like: Tensor, dtype=None) -> Tensor:
    return like.new_empty((0,), dtype=dtype or like.dtype)


def num_parameters(num_views: int, num_points: int, distortion: bool) -> int:
    return 3 + 3 * num_points + 6 * (num_views - 1) + (5 if distortion else 0)


def scene_struct(observations: Optional[Tensor], visibility: Optional[Tensor], num_views: int, num_points: int,
                 distortion: bool, batch: int, residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION) -> N.DavaScene:
    return N.DavaScene(batch, num_views, num_points, 1 if distortion else 0,
                       num_parameters(num_views, num_points, distortion),
                       N.ptr(observations), N.ptr(visibility), residual)


def solver_config(sufficient_decrease, curvature, error_threshold, iterations, minimum_step, max_line_search_trials,
                  strong, hessian_mode, drop_path_p: float = 0.0, drop_seed: int = 0,
                  return_second_last: bool = False) -> N.DavaSolverConfig:
    seed = int(drop_seed) & 0xFFFFFFFFFFFFFFFF
    return N.DavaSolverConfig(float(sufficient_decrease), float(curvature), float(error_threshold),
                              float(minimum_step), int(iterations), int(max_line_search_trials),
                              1 if strong else 0, int(hessian_mode), float(drop_path_p), seed & 0xFFFFFFFF, seed >> 32,
                              1 if return_second_last else 0)


def _check_scene_tensors(x: Tensor, observations: Tensor, visibility: Tensor, num_views: int, num_points: int,
                         distortion: bool) -> None:
    """Host-side shape checks BEFORE a launch: the kernels index with exactly these extents."""
    b = x.shape[0]
    p = num_parameters(num_views, num_points, distortion)
    if x.dim() != 2 or x.shape[1] != p:
        raise ValueError(f"parameters must be (B, {p}), got {tuple(x.shape)}")
    if tuple(observations.shape) != (b, num_views, num_points, 2):
        raise ValueError(f"observations must be ({b}, {num_views}, {num_points}, 2), got {tuple(observations.shape)}")
    if tuple(visibility.shape) != (b, num_views, num_points):
        raise ValueError(f"visibility must be ({b}, {num_views}, {num_points}), got {tuple(visibility.shape)}")
    if observations.dtype != torch.float32 or visibility.dtype != torch.uint8:
        raise TypeError("observations must be float32 and visibility uint8")
    for t in (x, observations, visibility):
        if not t.is_contiguous() or t.device != x.device:
            raise ValueError("scene tensors must be contiguous and on one device")


# ---------------------------------------------------------------- fused BA ops

@torch.library.custom_op("dava::ba_solve", mutates_args=("workspace",), device_types=_CUDA)
def ba_solve(x0: Tensor, observations: Tensor, visibility: Tensor, num_views: int, num_points: int,
             distortion: bool, sufficient_decrease: float, curvature: float, error_threshold: float,
             iterations: int, minimum_step: float, max_line_search_trials: int, strong: bool, hessian_mode: int,
             residual: int, want_error: bool, workspace: Tensor, drop_path_p: float = 0.0,
             drop_seed: int = 0, return_second_last: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """``dava_ba_solve``: the whole eval-mode BFGS solve of a (B, P) fp32 batch in one launch.
    ``workspace``: a uint8 scratch buffer of at least ``dava_ba_solve_workspace_bytes`` (its contents
    are overwritten), or an empty tensor to allocate one per call.
    Returns (x, error (B,) or empty, status (B, 4) int32)."""
    lib = N.load_library()
    _check_scene_tensors(x0, observations, visibility, num_views, num_points, distortion)
    b = x0.shape[0]
    dev = x0.device
    sc = scene_struct(observations, visibility, num_views, num_points, distortion, b, residual)
    cfg = solver_config(sufficient_decrease, curvature, error_threshold, iterations, minimum_step,
                        max_line_search_trials, strong, hessian_mode, drop_path_p, drop_seed, return_second_last)
    need = int(lib.dava_ba_solve_workspace_bytes(sc, cfg))
    if workspace.numel() < need or workspace.device != dev or workspace.dtype != torch.uint8:
        if workspace.numel() > 0:
            raise ValueError(f"workspace holds {workspace.numel()} bytes, the solve needs {need} (uint8, same device)")
        workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    x_out = torch.empty_like(x0)
    err = torch.empty(b, device=dev, dtype=torch.float32) if want_error else _empty0(x0)
    status = torch.empty((b, N.STATUS_WORDS), device=dev, dtype=torch.int32)
    with torch.cuda.device(dev):
        N.check(lib.dava_ba_solve(sc, cfg, N.ptr(x0), N.ptr(x_out), N.ptr(err) if want_error else None,
                                  N.ptr(status), N.ptr(workspace), workspace.numel(), N.stream_of(dev)),
                "dava_ba_solve")
    return x_out, err, status


@ba_solve.register_fake
def _(x0, observations, visibility, num_views, num_points, distortion, sufficient_decrease, curvature,
      error_threshold, iterations, minimum_step, max_line_search_trials, strong, hessian_mode, residual, want_error,
      workspace, drop_path_p=0.0, drop_seed=0, return_second_last=False):
    b = x0.shape[0]
    return (torch.empty_like(x0), x0.new_empty((b,) if want_error else (0,)),
            x0.new_empty((b, N.STATUS_WORDS), dtype=torch.int32))


@torch.library.custom_op("dava::bfgs_solve", mutates_args=(), device_types=_CUDA)
def bfgs_solve(parameters: Tensor, observations: Tensor, visibility: Tensor, num_views: int, num_points: int,
               distortion: bool = False, iterations: int = 1000, error_threshold: float = 1e-4,
               minimum_step: float = 1e-8, sufficient_decrease: float = 1e-4, curvature: float = 0.9,
               residual: int = 0) -> Tuple[Tensor, Tensor]:
    """The functional entry SURVEY.md 8(b) names: ``BFGSSolver().eval()`` on the fused objective with
    the reference's defaults (``bfgs_solver.py:49-60``, strong Wolfe, ``wolfe_conditions.py:116``'s
    1000 trials), compact inverse-Hessian history, workspace allocated per call.
    Returns (x (B, P), status (B, 4) int32: steps, stop reason, evaluations, line-search trials)."""
    x, _, status = ba_solve(parameters, observations, visibility, num_views, num_points, distortion,
                            sufficient_decrease, curvature, error_threshold, iterations, minimum_step, 1000, True,
                            N.DAVA_HESSIAN_COMPACT, residual, False, _empty0(parameters, torch.uint8))
    return x, status


@bfgs_solve.register_fake
def _(parameters, observations, visibility, num_views, num_points, distortion=False, iterations=1000,
      error_threshold=1e-4, minimum_step=1e-8, sufficient_decrease=1e-4, curvature=0.9, residual=0):
    return torch.empty_like(parameters), parameters.new_empty((parameters.shape[0], N.STATUS_WORDS), dtype=torch.int32)


@torch.library.custom_op("dava::ba_evaluate", mutates_args=(), device_types=_CUDA)
def ba_evaluate(x: Tensor, observations: Tensor, visibility: Tensor, num_views: int, num_points: int,
                distortion: bool, direction: Optional[Tensor], alpha: Optional[Tensor], want_grad: bool,
                want_slope: bool, residual: int) -> Tuple[Tensor, Tensor, Tensor]:
    """``dava_ba_evaluate``: E, dE/dx and d . dE/dx at x + alpha d.  Unrequested outputs are empty."""
    lib = N.load_library()
    _check_scene_tensors(x, observations, visibility, num_views, num_points, distortion)
    b = x.shape[0]
    for t in (direction, alpha):
        if t is not None and (t.device != x.device or t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError("direction / alpha must be contiguous float32 on the parameters' device")
    if direction is not None and direction.shape != x.shape:
        raise ValueError("direction must have the parameters' shape")
    if alpha is not None and alpha.numel() != b:
        raise ValueError("alpha must hold one value per problem")
    if want_slope and direction is None:
        raise ValueError("the slope needs a direction")
    err = torch.empty(b, device=x.device, dtype=torch.float32)
    grad = torch.empty_like(x) if want_grad else _empty0(x)
    slope = torch.empty(b, device=x.device, dtype=torch.float32) if want_slope else _empty0(x)
    sc = scene_struct(observations, visibility, num_views, num_points, distortion, b, residual)
    with torch.cuda.device(x.device):
        N.check(lib.dava_ba_evaluate(sc, N.ptr(x), N.ptr(direction), N.ptr(alpha), N.ptr(err),
                                     N.ptr(grad) if want_grad else None, N.ptr(slope) if want_slope else None,
                                     N.stream_of(x.device)), "dava_ba_evaluate")
    return err, grad, slope


@ba_evaluate.register_fake
def _(x, observations, visibility, num_views, num_points, distortion, direction, alpha, want_grad, want_slope,
      residual):
    b = x.shape[0]
    return (x.new_empty((b,)), torch.empty_like(x) if want_grad else x.new_empty((0,)),
            x.new_empty((b,) if want_slope else (0,)))


@torch.library.custom_op("dava::ba_second_order", mutates_args=(), device_types=_CUDA)
def ba_second_order(x: Tensor, observations: Tensor, visibility: Tensor, num_views: int, num_points: int,
                    distortion: bool, direction: Optional[Tensor], residual: int, want_hv: bool,
                    want_obs: bool, obs_direction: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """``dava_ba_second_order_obs``: (E, dE/dx, H v + (d2E/dx dobs) u, dE/dobs, (d2E/dobs dx) v + (d2E/dobs2) u),
    forward-over-reverse.  direction / obs_direction None mean v = 0 / u = 0.  Unrequested outputs are empty."""
    lib = N.load_library()
    _check_scene_tensors(x, observations, visibility, num_views, num_points, distortion)
    if direction is not None and (direction.shape != x.shape or direction.dtype != torch.float32
                                  or not direction.is_contiguous()):
        raise ValueError("direction must be a contiguous float32 tensor of the parameters' shape")
    if obs_direction is not None and (obs_direction.shape != observations.shape or obs_direction.dtype != torch.float32
                                      or not obs_direction.is_contiguous()):
        raise ValueError("obs_direction must be a contiguous float32 tensor of the observations' shape")
    b = x.shape[0]
    err = torch.empty(b, device=x.device, dtype=torch.float32)
    grad = torch.empty_like(x)
    hv = torch.empty_like(x) if want_hv else _empty0(x)
    obs_grad = torch.empty_like(observations) if want_obs else _empty0(x)
    obs_hv = torch.empty_like(observations) if (want_obs and want_hv) else _empty0(x)
    sc = scene_struct(observations, visibility, num_views, num_points, distortion, b, residual)
    with torch.cuda.device(x.device):
        N.check(lib.dava_ba_second_order_obs(sc, N.ptr(x), N.ptr(direction), N.ptr(obs_direction), N.ptr(err),
                                             N.ptr(grad), N.ptr(hv) if want_hv else None,
                                             N.ptr(obs_grad) if want_obs else None,
                                             N.ptr(obs_hv) if (want_obs and want_hv) else None, N.stream_of(x.device)),
                "dava_ba_second_order_obs")
    return err, grad, hv, obs_grad, obs_hv


@ba_second_order.register_fake
def _(x, observations, visibility, num_views, num_points, distortion, direction, residual, want_hv, want_obs,
      obs_direction=None):
    b = x.shape[0]
    return (x.new_empty((b,)), torch.empty_like(x), torch.empty_like(x) if want_hv else x.new_empty((0,)),
            torch.empty_like(observations) if want_obs else x.new_empty((0,)),
            torch.empty_like(observations) if (want_obs and want_hv) else x.new_empty((0,)))


@torch.library.custom_op("dava::ba_solve_record", mutates_args=(), device_types=_CUDA)
def ba_solve_record(x0: Tensor, observations: Tensor, visibility: Tensor, num_views: int, num_points: int,
                    distortion: bool, sufficient_decrease: float, curvature: float, error_threshold: float,
                    iterations: int, minimum_step: float, max_line_search_trials: int, strong: bool,
                    residual: int, drop_path_p: float = 0.0, drop_seed: int = 0,
                    return_second_last: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """``dava_ba_solve_record``: the fused COMPACT solve (bitwise ``ba_solve``'s x and status) plus the
    tape the adjoint replays.  Returns (x, status (B, 4) int32, tape uint8)."""
    lib = N.load_library()
    _check_scene_tensors(x0, observations, visibility, num_views, num_points, distortion)
    b, dev = x0.shape[0], x0.device
    sc = scene_struct(observations, visibility, num_views, num_points, distortion, b, residual)
    cfg = solver_config(sufficient_decrease, curvature, error_threshold, iterations, minimum_step,
                        max_line_search_trials, strong, N.DAVA_HESSIAN_COMPACT, drop_path_p, drop_seed,
                        return_second_last)
    need = int(lib.dava_ba_solve_tape_bytes(sc, cfg))
    if need == 0:
        raise ValueError("this scene / configuration has no fused adjoint (compact mode, P <= 14336, "
                         "iterations >= 1)")
    tape = torch.empty(need, dtype=torch.uint8, device=dev)
    if _POISON:  # debugging aid: every byte the kernels do not write reads back as NaN
        tape.fill_(0xFF)
    x_out = torch.empty_like(x0)
    status = torch.empty((b, N.STATUS_WORDS), device=dev, dtype=torch.int32)
    with torch.cuda.device(dev):
        N.check(lib.dava_ba_solve_record(sc, cfg, N.ptr(x0), N.ptr(x_out), None, N.ptr(status), N.ptr(tape),
                                         tape.numel(), N.stream_of(dev)), "dava_ba_solve_record")
    return x_out, status, tape


@ba_solve_record.register_fake
def _(x0, observations, visibility, num_views, num_points, distortion, sufficient_decrease, curvature,
      error_threshold, iterations, minimum_step, max_line_search_trials, strong, residual, drop_path_p=0.0,
      drop_seed=0, return_second_last=False):
    b = x0.shape[0]
    ctx = torch.library.get_ctx()
    return (torch.empty_like(x0), x0.new_empty((b, N.STATUS_WORDS), dtype=torch.int32),
            x0.new_empty((ctx.new_dynamic_size(),), dtype=torch.uint8))


@torch.library.custom_op("dava::ba_solve_backward", mutates_args=(), device_types=_CUDA)
def ba_solve_backward(x_out_grad: Tensor, tape: Tensor, status: Tensor, observations: Tensor, visibility: Tensor,
                      num_views: int, num_points: int, distortion: bool, iterations: int, residual: int,
                      want_observations: bool) -> Tuple[Tensor, Tensor]:
    """``dava_ba_solve_backward``: (dL/dx0, dL/dobs or empty) of a recorded solve for dL/dx_out."""
    lib = N.load_library()
    _check_scene_tensors(x_out_grad, observations, visibility, num_views, num_points, distortion)
    b, dev = x_out_grad.shape[0], x_out_grad.device
    if tuple(status.shape) != (b, N.STATUS_WORDS) or status.dtype != torch.int32 or not status.is_contiguous():
        raise ValueError("status must be the recording call's contiguous (B, 4) int32 tensor")
    # the kernel dereferences tape and status as device memory of this launch: refuse anything else
    # loudly rather than fault the GPU (a CPU or other-device tensor, a short or strided tape)
    for what, t in (("tape", tape), ("status", status)):
        if t.device != dev:
            raise ValueError(f"{what} must be on {dev} (the cotangent's device), got {t.device}")
    if tape.dtype != torch.uint8 or tape.dim() != 1 or not tape.is_contiguous():
        raise ValueError("tape must be the recording call's contiguous 1-D uint8 tensor")
    sc = scene_struct(observations, visibility, num_views, num_points, distortion, b, residual)
    cfg = solver_config(1e-4, 0.9, 1e-4, iterations, 1e-8, 1000, True, N.DAVA_HESSIAN_COMPACT)
    tape_need = int(lib.dava_ba_solve_tape_bytes(sc, cfg))
    if tape.numel() < tape_need:
        raise ValueError(f"tape holds {tape.numel()} bytes; a recording of this scene and iteration count "
                         f"writes {tape_need}")
    need = int(lib.dava_ba_solve_backward_workspace_bytes(sc, cfg))
    if need == 0:
        raise ValueError("this scene / configuration has no fused adjoint")
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    if _POISON:
        ws.fill_(0xFF)
    gx = torch.empty_like(x_out_grad)
    gobs = torch.empty_like(observations) if want_observations else _empty0(x_out_grad)
    with torch.cuda.device(dev):
        N.check(lib.dava_ba_solve_backward(sc, cfg, N.ptr(tape), tape.numel(), N.ptr(status), N.ptr(x_out_grad),
                                           N.ptr(gx), N.ptr(gobs) if want_observations else None, N.ptr(ws),
                                           ws.numel(), N.stream_of(dev)), "dava_ba_solve_backward")
    return gx, gobs


@ba_solve_backward.register_fake
def _(x_out_grad, tape, status, observations, visibility, num_views, num_points, distortion, iterations, residual,
      want_observations):
    return (torch.empty_like(x_out_grad),
            torch.empty_like(observations) if want_observations else x_out_grad.new_empty((0,)))


# ------------------------------------------------- generic BFGS building blocks

def _square_batch(h: Tensor) -> Tuple[int, int]:
    # the kernels (GPU and host) read raw row-major pointers: a transposed or sliced view would be
    # computed on the wrong layout, and empty_like would copy its strides into the outputs
    if h.dim() != 3 or h.shape[1] != h.shape[2] or not h.is_contiguous():
        raise ValueError(f"expected a contiguous (B, n, n) batch of matrices, got {tuple(h.shape)} "
                         f"(contiguous={h.is_contiguous()})")
    return h.shape[0], h.shape[1]


def _row_batch(t: Tensor, what: str) -> Tuple[int, int]:
    """The primary (B, n) operand of an op: contiguous, for the same reason as _square_batch."""
    if t.dim() != 2 or not t.is_contiguous():
        raise ValueError(f"{what}: expected a contiguous (B, n) batch, got {tuple(t.shape)} "
                         f"(contiguous={t.is_contiguous()})")
    return t.shape[0], t.shape[1]


def _same(t: Tensor, like: Tensor, shape, what: str) -> None:
    if tuple(t.shape) != tuple(shape) or t.dtype != like.dtype or t.device != like.device or not t.is_contiguous():
        raise ValueError(f"{what}: expected contiguous {like.dtype} {tuple(shape)} on {like.device}, "
                         f"got {t.dtype} {tuple(t.shape)} on {t.device}")


@torch.library.custom_op("dava::bfgs_update_inverse_hessian", mutates_args=(), device_types=_CUDA)
def bfgs_update_inverse_hessian(h: Tensor, s: Tensor, y: Tensor) -> Tensor:
    """(B, n, n), (B, n), (B, n) -> H+ (``bfgs_solver.py:235-303``)."""
    b, n = _square_batch(h)
    _same(s, h, (b, n), "step")
    _same(y, h, (b, n), "delta_gradient")
    out = torch.empty_like(h)
    with torch.cuda.device(h.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_update_inverse_hessian_{_dt(h)}")(
            b, n, N.ptr(h), N.ptr(s), N.ptr(y), N.ptr(out), N.stream_of(h.device)), "dava_bfgs_update_inverse_hessian")
    return out


@bfgs_update_inverse_hessian.register_fake
def _(h, s, y):
    return torch.empty_like(h)


@torch.library.custom_op("dava::bfgs_update_inverse_hessian_backward", mutates_args=(), device_types=_CUDA)
def bfgs_update_inverse_hessian_backward(h: Tensor, s: Tensor, y: Tensor, grad: Tensor, need_h: bool, need_s: bool,
                                         need_y: bool) -> Tuple[Tensor, Tensor, Tensor]:
    b, n = _square_batch(h)
    _same(grad, h, (b, n, n), "grad")
    gh = torch.empty_like(h) if need_h else _empty0(h)
    gs = torch.empty_like(s) if need_s else _empty0(h)
    gy = torch.empty_like(y) if need_y else _empty0(h)
    with torch.cuda.device(h.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_update_inverse_hessian_backward_{_dt(h)}")(
            b, n, N.ptr(h), N.ptr(s), N.ptr(y), N.ptr(grad), N.ptr(gh) if need_h else None,
            N.ptr(gs) if need_s else None, N.ptr(gy) if need_y else None, N.stream_of(h.device)),
            "dava_bfgs_update_inverse_hessian_backward")
    return gh, gs, gy


@bfgs_update_inverse_hessian_backward.register_fake
def _(h, s, y, grad, need_h, need_s, need_y):
    return (torch.empty_like(h) if need_h else h.new_empty((0,)), torch.empty_like(s) if need_s else h.new_empty((0,)),
            torch.empty_like(y) if need_y else h.new_empty((0,)))


@torch.library.custom_op("dava::bfgs_initial_scale", mutates_args=(), device_types=_CUDA)
def bfgs_initial_scale(s: Tensor, y: Tensor) -> Tensor:
    """(B, n), (B, n) -> gamma (B,) (``bfgs_solver.py:217-233``)."""
    b, n = _row_batch(s, "step")
    _same(y, s, (b, n), "delta_gradient")
    out = s.new_empty((b,))
    with torch.cuda.device(s.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_initial_scale_{_dt(s)}")(
            b, n, N.ptr(s), N.ptr(y), N.ptr(out), N.stream_of(s.device)), "dava_bfgs_initial_scale")
    return out


@bfgs_initial_scale.register_fake
def _(s, y):
    return s.new_empty((s.shape[0],))


@torch.library.custom_op("dava::bfgs_initial_scale_backward", mutates_args=(), device_types=_CUDA)
def bfgs_initial_scale_backward(s: Tensor, y: Tensor, grad: Tensor, need_s: bool,
                                need_y: bool) -> Tuple[Tensor, Tensor]:
    b, n = _row_batch(s, "step")
    _same(grad, s, (b,), "grad")
    gs = torch.empty_like(s) if need_s else _empty0(s)
    gy = torch.empty_like(y) if need_y else _empty0(s)
    with torch.cuda.device(s.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_initial_scale_backward_{_dt(s)}")(
            b, n, N.ptr(s), N.ptr(y), N.ptr(grad), N.ptr(gs) if need_s else None, N.ptr(gy) if need_y else None,
            N.stream_of(s.device)), "dava_bfgs_initial_scale_backward")
    return gs, gy


@bfgs_initial_scale_backward.register_fake
def _(s, y, grad, need_s, need_y):
    return (torch.empty_like(s) if need_s else s.new_empty((0,)), torch.empty_like(y) if need_y else s.new_empty((0,)))


@torch.library.custom_op("dava::bfgs_scale_matrix", mutates_args=(), device_types=_CUDA)
def bfgs_scale_matrix(scale: Tensor, h: Tensor) -> Tensor:
    """scale (B,) * H (B, n, n): the k == 1 rescale of H0 (``bfgs_solver.py:159-167``)."""
    b, n = _square_batch(h)
    _same(scale, h, (b,), "scale")
    out = torch.empty_like(h)
    with torch.cuda.device(h.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_scale_matrix_{_dt(h)}")(
            b, n, N.ptr(scale), N.ptr(h), N.ptr(out), N.stream_of(h.device)), "dava_bfgs_scale_matrix")
    return out


@bfgs_scale_matrix.register_fake
def _(scale, h):
    return torch.empty_like(h)


@torch.library.custom_op("dava::bfgs_scale_matrix_backward", mutates_args=(), device_types=_CUDA)
def bfgs_scale_matrix_backward(scale: Tensor, h: Tensor, grad: Tensor, need_scale: bool,
                               need_h: bool) -> Tuple[Tensor, Tensor]:
    b, n = _square_batch(h)
    _same(grad, h, (b, n, n), "grad")
    gsc = torch.empty_like(scale) if need_scale else _empty0(h)
    gh = torch.empty_like(h) if need_h else _empty0(h)
    with torch.cuda.device(h.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_scale_matrix_backward_{_dt(h)}")(
            b, n, N.ptr(scale), N.ptr(h), N.ptr(grad), N.ptr(gsc) if need_scale else None,
            N.ptr(gh) if need_h else None, N.stream_of(h.device)), "dava_bfgs_scale_matrix_backward")
    return gsc, gh


@bfgs_scale_matrix_backward.register_fake
def _(scale, h, grad, need_scale, need_h):
    return (torch.empty_like(scale) if need_scale else h.new_empty((0,)),
            torch.empty_like(h) if need_h else h.new_empty((0,)))


@torch.library.custom_op("dava::bfgs_search_direction", mutates_args=(), device_types=_CUDA)
def bfgs_search_direction(h: Tensor, g: Tensor) -> Tensor:
    """d = -H g (``bfgs_solver.py:173-176``)."""
    b, n = _square_batch(h)
    _same(g, h, (b, n), "gradient")
    out = torch.empty_like(g)
    with torch.cuda.device(h.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_search_direction_{_dt(h)}")(
            b, n, N.ptr(h), N.ptr(g), N.ptr(out), N.stream_of(h.device)), "dava_bfgs_search_direction")
    return out


@bfgs_search_direction.register_fake
def _(h, g):
    return torch.empty_like(g)


@torch.library.custom_op("dava::bfgs_compact_direction",
                         mutates_args=("history_s", "history_w", "history_rho", "history_c", "gamma"),
                         device_types=_CUDA)
def bfgs_compact_direction(g: Tensor, y: Tensor, s: Tensor, problem_index: Tensor, count: int, history_s: Tensor,
                           history_w: Tensor, history_rho: Tensor, history_c: Tensor, gamma: Tensor) -> Tensor:
    """The generic loop's update + search direction on compact history rows (no dense matrix): appends
    entry ``count`` to the history of the problems ``problem_index`` and returns d = -H g (n_active, P)."""
    n_act, p = _row_batch(g, "gradient")
    _same(y, g, (n_act, p), "delta_gradient")
    _same(s, g, (n_act, p), "step")
    if problem_index.dtype != torch.int64 or tuple(problem_index.shape) != (n_act,) \
            or problem_index.device != g.device or not problem_index.is_contiguous():
        raise ValueError("problem_index must be a contiguous int64 (n_active,) tensor on the gradient's device")
    if history_s.dim() != 3 or history_w.shape != history_s.shape or history_s.dtype != g.dtype \
            or history_w.dtype != g.dtype or history_s.shape[2] < p:
        raise ValueError("history rows must be (B, capacity, >= P) in the gradient's dtype")
    b_all, cap, stride = history_s.shape
    for t, shape, what in ((history_rho, (b_all, cap), "history_rho"), (history_c, (b_all, cap), "history_c"),
                           (gamma, (b_all,), "gamma")):
        if tuple(t.shape) != shape or t.dtype != g.dtype:
            raise ValueError(f"{what} must be {shape} in the gradient's dtype")
    for t in (history_s, history_w, history_rho, history_c, gamma):
        if not t.is_contiguous() or t.device != g.device:
            raise ValueError("history tensors must be contiguous and on the gradient's device")
    if not 0 <= count < cap:
        raise ValueError(f"count {count} outside the history capacity {cap}")
    out = torch.empty_like(g)
    with torch.cuda.device(g.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_compact_direction_{_dt(g)}")(
            n_act, p, stride, cap, count, N.ptr(problem_index), N.ptr(g), N.ptr(y), N.ptr(s), N.ptr(history_s),
            N.ptr(history_w), N.ptr(history_rho), N.ptr(history_c), N.ptr(gamma), N.ptr(out),
            N.stream_of(g.device)), "dava_bfgs_compact_direction")
    return out


@bfgs_compact_direction.register_fake
def _(g, y, s, problem_index, count, history_s, history_w, history_rho, history_c, gamma):
    return torch.empty_like(g)


@torch.library.custom_op("dava::bfgs_search_direction_backward", mutates_args=(), device_types=_CUDA)
def bfgs_search_direction_backward(h: Tensor, g: Tensor, grad: Tensor, need_h: bool,
                                   need_g: bool) -> Tuple[Tensor, Tensor]:
    b, n = _square_batch(h)
    _same(grad, h, (b, n), "grad")
    gh = torch.empty_like(h) if need_h else _empty0(h)
    gg = torch.empty_like(g) if need_g else _empty0(h)
    with torch.cuda.device(h.device):
        N.check(getattr(N.load_library(), f"dava_bfgs_search_direction_backward_{_dt(h)}")(
            b, n, N.ptr(h), N.ptr(g), N.ptr(grad), N.ptr(gh) if need_h else None, N.ptr(gg) if need_g else None,
            N.stream_of(h.device)), "dava_bfgs_search_direction_backward")
    return gh, gg


@bfgs_search_direction_backward.register_fake
def _(h, g, grad, need_h, need_g):
    return (torch.empty_like(h) if need_h else h.new_empty((0,)), torch.empty_like(g) if need_g else h.new_empty((0,)))


# ------------------------------------------------------- batched Wolfe state machine

WOLFE_STATE_COLUMNS = 9
WOLFE_FLAG_COLUMNS = 2


@torch.library.custom_op("dava::wolfe_init", mutates_args=(), device_types=_CUDA)
def wolfe_init(direction: Tensor, f0: Tensor, g0: Tensor) -> Tuple[Tensor, Tensor]:
    """(state (B, 9), flags (B, 2) uint8) for a line search along ``direction`` from (f0, g0)."""
    b, n = _row_batch(direction, "search_direction")
    _same(g0, direction, (b, n), "base_gradient")
    _same(f0, direction, (b,), "base_error")
    state = direction.new_empty((b, WOLFE_STATE_COLUMNS))
    flags = direction.new_empty((b, WOLFE_FLAG_COLUMNS), dtype=torch.uint8)
    with torch.cuda.device(direction.device):
        N.check(getattr(N.load_library(), f"dava_wolfe_init_{_dt(direction)}")(
            b, n, N.ptr(direction), N.ptr(f0), N.ptr(g0), N.ptr(state), N.ptr(flags), N.stream_of(direction.device)),
            "dava_wolfe_init")
    return state, flags


@wolfe_init.register_fake
def _(direction, f0, g0):
    b = direction.shape[0]
    return direction.new_empty((b, WOLFE_STATE_COLUMNS)), direction.new_empty((b, WOLFE_FLAG_COLUMNS),
                                                                               dtype=torch.uint8)


def _check_wolfe(state: Tensor, flags: Tensor) -> int:
    b = state.shape[0]
    if tuple(state.shape) != (b, WOLFE_STATE_COLUMNS) or tuple(flags.shape) != (b, WOLFE_FLAG_COLUMNS) \
            or flags.dtype != torch.uint8 or not state.is_contiguous() or not flags.is_contiguous():
        raise ValueError("Wolfe state must be (B, 9) and flags (B, 2) uint8, contiguous")
    return b


@torch.library.custom_op("dava::wolfe_propose", mutates_args=("state",), device_types=_CUDA)
def wolfe_propose(state: Tensor, flags: Tensor) -> None:
    """Next trial alpha of every active line search (widen x2 or bisect), in place."""
    b = _check_wolfe(state, flags)
    with torch.cuda.device(state.device):
        N.check(getattr(N.load_library(), f"dava_wolfe_propose_{_dt(state)}")(
            b, N.ptr(state), N.ptr(flags), N.stream_of(state.device)), "dava_wolfe_propose")


@wolfe_propose.register_fake
def _(state, flags):
    return None


@torch.library.custom_op("dava::wolfe_update", mutates_args=("state", "flags"), device_types=_CUDA)
def wolfe_update(state: Tensor, flags: Tensor, trial: int, c1: float, c2: float, strong: bool) -> None:
    """Consume (f(alpha), phi'(alpha)) already written into ``state`` and advance the brackets."""
    b = _check_wolfe(state, flags)
    with torch.cuda.device(state.device):
        N.check(getattr(N.load_library(), f"dava_wolfe_update_{_dt(state)}")(
            b, int(trial), float(c1), float(c2), 1 if strong else 0, N.ptr(state), N.ptr(flags),
            N.stream_of(state.device)), "dava_wolfe_update")


@wolfe_update.register_fake
def _(state, flags, trial, c1, c2, strong):
    return None


# ------------------------------------------------ the same building blocks on CPU tensors
# The reference's solver runs wherever `parameters` live (bfgs_solver.py:94-117; BASELINE C1 is "BFGS on
# PyTorch CPU").  These CPU kernels call the host C++ flavours of the same library (csrc/bfgs_host.hip,
# dava_cpu_*): explicit dispatch on the tensor's device, never a fallback for device tensors (a ROCm
# tensor still goes to the HIP kernels and raises without them).  The fused BA objectives stay GPU-only.

def _cpu(name: str, t: Tensor, *args) -> None:
    N.check(getattr(N.load_library(), f"dava_cpu_{name}_{_dt(t)}")(*args), f"dava_cpu_{name}")


def _cpu_ptr(t: Optional[Tensor]):
    return None if t is None else N.ptr(t)


@bfgs_update_inverse_hessian.register_kernel("cpu")
def _(h, s, y):
    b, n = _square_batch(h)
    _same(s, h, (b, n), "step")
    _same(y, h, (b, n), "delta_gradient")
    out = torch.empty_like(h)
    _cpu("bfgs_update_inverse_hessian", h, b, n, N.ptr(h), N.ptr(s), N.ptr(y), N.ptr(out))
    return out


@bfgs_update_inverse_hessian_backward.register_kernel("cpu")
def _(h, s, y, grad, need_h, need_s, need_y):
    b, n = _square_batch(h)
    _same(grad, h, (b, n, n), "grad")
    gh = torch.empty_like(h) if need_h else _empty0(h)
    gs = torch.empty_like(s) if need_s else _empty0(h)
    gy = torch.empty_like(y) if need_y else _empty0(h)
    _cpu("bfgs_update_inverse_hessian_backward", h, b, n, N.ptr(h), N.ptr(s), N.ptr(y), N.ptr(grad),
         _cpu_ptr(gh if need_h else None), _cpu_ptr(gs if need_s else None), _cpu_ptr(gy if need_y else None))
    return gh, gs, gy


@bfgs_initial_scale.register_kernel("cpu")
def _(s, y):
    b, n = _row_batch(s, "step")
    _same(y, s, (b, n), "delta_gradient")
    out = s.new_empty((b,))
    _cpu("bfgs_initial_scale", s, b, n, N.ptr(s), N.ptr(y), N.ptr(out))
    return out


@bfgs_initial_scale_backward.register_kernel("cpu")
def _(s, y, grad, need_s, need_y):
    b, n = _row_batch(s, "step")
    _same(grad, s, (b,), "grad")
    gs = torch.empty_like(s) if need_s else _empty0(s)
    gy = torch.empty_like(y) if need_y else _empty0(s)
    _cpu("bfgs_initial_scale_backward", s, b, n, N.ptr(s), N.ptr(y), N.ptr(grad), _cpu_ptr(gs if need_s else None),
         _cpu_ptr(gy if need_y else None))
    return gs, gy


@bfgs_scale_matrix.register_kernel("cpu")
def _(scale, h):
    b, n = _square_batch(h)
    _same(scale, h, (b,), "scale")
    out = torch.empty_like(h)
    _cpu("bfgs_scale_matrix", h, b, n, N.ptr(scale), N.ptr(h), N.ptr(out))
    return out


@bfgs_scale_matrix_backward.register_kernel("cpu")
def _(scale, h, grad, need_scale, need_h):
    b, n = _square_batch(h)
    _same(grad, h, (b, n, n), "grad")
    gsc = torch.empty_like(scale) if need_scale else _empty0(h)
    gh = torch.empty_like(h) if need_h else _empty0(h)
    _cpu("bfgs_scale_matrix_backward", h, b, n, N.ptr(scale), N.ptr(h), N.ptr(grad),
         _cpu_ptr(gsc if need_scale else None), _cpu_ptr(gh if need_h else None))
    return gsc, gh


@bfgs_search_direction.register_kernel("cpu")
def _(h, g):
    b, n = _square_batch(h)
    _same(g, h, (b, n), "gradient")
    out = torch.empty_like(g)
    _cpu("bfgs_search_direction", h, b, n, N.ptr(h), N.ptr(g), N.ptr(out))
    return out


@bfgs_search_direction_backward.register_kernel("cpu")
def _(h, g, grad, need_h, need_g):
    b, n = _square_batch(h)
    _same(grad, h, (b, n), "grad")
    gh = torch.empty_like(h) if need_h else _empty0(h)
    gg = torch.empty_like(g) if need_g else _empty0(h)
    _cpu("bfgs_search_direction_backward", h, b, n, N.ptr(h), N.ptr(g), N.ptr(grad), _cpu_ptr(gh if need_h else None),
         _cpu_ptr(gg if need_g else None))
    return gh, gg


@wolfe_init.register_kernel("cpu")
def _(direction, f0, g0):
    b, n = _row_batch(direction, "search_direction")
    _same(g0, direction, (b, n), "base_gradient")
    _same(f0, direction, (b,), "base_error")
    state = direction.new_empty((b, WOLFE_STATE_COLUMNS))
    flags = direction.new_empty((b, WOLFE_FLAG_COLUMNS), dtype=torch.uint8)
    _cpu("wolfe_init", direction, b, n, N.ptr(direction), N.ptr(f0), N.ptr(g0), N.ptr(state), N.ptr(flags))
    return state, flags


@wolfe_propose.register_kernel("cpu")
def _(state, flags):
    b = _check_wolfe(state, flags)
    _cpu("wolfe_propose", state, b, N.ptr(state), N.ptr(flags))


@wolfe_update.register_kernel("cpu")
def _(state, flags, trial, c1, c2, strong):
    b = _check_wolfe(state, flags)
    _cpu("wolfe_update", state, b, int(trial), float(c1), float(c2), 1 if strong else 0, N.ptr(state), N.ptr(flags))


# ------------------------------------------------ legacy L1 camera model evaluation

@torch.library.custom_op("dava::l1_camera_evaluate", mutates_args=(), device_types=_CUDA)
def l1_camera_evaluate(focal: Tensor, cx: Tensor, cy: Tensor, translation: Tensor, lie: Tensor, world: Tensor,
                       target: Tensor, visibility: Tensor, minimum_z_distance: float, maximum_pixel_ratio: float,
                       max_gradient: float, error_scale: float, want_error: bool,
                       want_gradient: bool) -> Tuple[Tensor, Tensor]:
    """``dava_l1_camera_evaluate``: PinholeCameraModelL1 error (B, E) and its hand-written gradient
    (B, E, P) (``camera_model/pinhole_camera_model_l1.py:132-285``).  Shapes: focal/cx/cy (B, E),
    translation/lie (B, E, M, 3), world (B, E, N-2, 3), target (B, M, N, 2), visibility (B, M, N) uint8."""
    b, e = focal.shape
    m, n = target.shape[1], target.shape[2]
    p = 3 + 6 * m + 3 * n - 7
    for t, shape, what in ((cx, (b, e), "cx"), (cy, (b, e), "cy"), (translation, (b, e, m, 3), "translation"),
                           (lie, (b, e, m, 3), "orientation"), (world, (b, e, n - 2, 3), "world_points"),
                           (target, (b, m, n, 2), "true_projected_points")):
        _same(t, focal, shape, what)
    if tuple(visibility.shape) != (b, m, n) or visibility.dtype != torch.uint8 or not visibility.is_contiguous():
        raise ValueError("visibility must be a contiguous (B, M, N) uint8 tensor")
    err = focal.new_empty((b, e)) if want_error else _empty0(focal)
    grad = focal.new_empty((b, e, p)) if want_gradient else _empty0(focal)
    with torch.cuda.device(focal.device):
        N.check(getattr(N.load_library(), f"dava_l1_camera_evaluate_{_dt(focal)}")(
            b, e, m, n, N.ptr(focal), N.ptr(cx), N.ptr(cy), N.ptr(translation), N.ptr(lie), N.ptr(world),
            N.ptr(target), N.ptr(visibility), minimum_z_distance, maximum_pixel_ratio, max_gradient, error_scale,
            N.ptr(err) if want_error else None, N.ptr(grad) if want_gradient else None, N.stream_of(focal.device)),
            "dava_l1_camera_evaluate")
    return err, grad


@l1_camera_evaluate.register_fake
def _(focal, cx, cy, translation, lie, world, target, visibility, minimum_z_distance, maximum_pixel_ratio,
      max_gradient, error_scale, want_error, want_gradient):
    b, e = focal.shape
    m, n = target.shape[1], target.shape[2]
    return (focal.new_empty((b, e) if want_error else (0,)),
            focal.new_empty((b, e, 3 + 6 * m + 3 * n - 7) if want_gradient else (0,)))


@torch.library.custom_op("dava::l1_camera_vjp", mutates_args=(), device_types=_CUDA)
def l1_camera_vjp(focal: Tensor, cx: Tensor, cy: Tensor, translation: Tensor, lie: Tensor, world: Tensor,
                  target: Tensor, visibility: Tensor, minimum_z_distance: float, maximum_pixel_ratio: float,
                  max_gradient: float, error_scale: float, error_cotangent: Optional[Tensor],
                  gradient_cotangent: Optional[Tensor], detach_points: bool) -> Tensor:
    """``dava_l1_camera_vjp``: the model's inputs' cotangent (B, E, D), D = 3 + 6M + 3(N-2) in the
    order focal, cx, cy, translation (M, 3), lie (M, 3), world (N-2, 3), from the error's (B, E)
    and / or the gradient's (B, E, P) cotangents.  Same input shapes as ``l1_camera_evaluate``."""
    b, e = focal.shape
    m, n = target.shape[1], target.shape[2]
    p = 3 + 6 * m + 3 * n - 7
    for t, shape, what in ((cx, (b, e), "cx"), (cy, (b, e), "cy"), (translation, (b, e, m, 3), "translation"),
                           (lie, (b, e, m, 3), "orientation"), (world, (b, e, n - 2, 3), "world_points"),
                           (target, (b, m, n, 2), "true_projected_points")):
        _same(t, focal, shape, what)
    if error_cotangent is not None:
        _same(error_cotangent, focal, (b, e), "error cotangent")
    if gradient_cotangent is not None:
        _same(gradient_cotangent, focal, (b, e, p), "gradient cotangent")
    if tuple(visibility.shape) != (b, m, n) or visibility.dtype != torch.uint8 or not visibility.is_contiguous():
        raise ValueError("visibility must be a contiguous (B, M, N) uint8 tensor")
    out = focal.new_zeros((b, e, 3 + 6 * m + 3 * (n - 2)))
    if error_cotangent is None and gradient_cotangent is None:
        return out
    with torch.cuda.device(focal.device):
        N.check(getattr(N.load_library(), f"dava_l1_camera_vjp_{_dt(focal)}")(
            b, e, m, n, N.ptr(focal), N.ptr(cx), N.ptr(cy), N.ptr(translation), N.ptr(lie), N.ptr(world),
            N.ptr(target), N.ptr(visibility), minimum_z_distance, maximum_pixel_ratio, max_gradient, error_scale,
            N.ptr(error_cotangent) if error_cotangent is not None else None,
            N.ptr(gradient_cotangent) if gradient_cotangent is not None else None, int(detach_points), N.ptr(out),
            N.stream_of(focal.device)), "dava_l1_camera_vjp")
    return out


@l1_camera_vjp.register_fake
def _(focal, cx, cy, translation, lie, world, target, visibility, minimum_z_distance, maximum_pixel_ratio,
      max_gradient, error_scale, error_cotangent, gradient_cotangent, detach_points):
    b, e = focal.shape
    m, n = target.shape[1], target.shape[2]
    return focal.new_empty((b, e, 3 + 6 * m + 3 * (n - 2)))


OPS = ("bfgs_solve", "ba_solve", "ba_solve_record", "ba_solve_backward", "ba_evaluate", "ba_second_order", "bfgs_update_inverse_hessian",
       "bfgs_update_inverse_hessian_backward", "bfgs_initial_scale", "bfgs_initial_scale_backward",
       "bfgs_scale_matrix", "bfgs_scale_matrix_backward", "bfgs_search_direction", "bfgs_search_direction_backward",
       "wolfe_init", "wolfe_propose", "wolfe_update", "l1_camera_evaluate", "l1_camera_vjp")
