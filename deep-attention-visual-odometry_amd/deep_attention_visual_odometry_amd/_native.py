"""ctypes binding of the C ABI in include/dava_ba.h (libdava_ba.so, gfx950).

The library is built in-tree by ``make`` (see __graft_entry__.build()).  There
is deliberately NO fallback: if the library or a ROCm device is missing, every
product entry point raises.  torch is imported first so the library binds to
the HIP runtime torch already loaded (both carry SONAME libamdhip64.so.7),
which lets it run on torch's streams and torch-allocated memory.

Launch choices (LDS or global-vector mode, waves per workgroup, on-chip history entries, work queue,
the generic loops below) are the library's own: neither it nor this module reads them from the
environment, so a user's stray variable cannot change a launch.  Tests override them through
:func:`debug_overrides`; A/B measurements set ``DAVA_DEBUG_OVERRIDES=1`` and the ``DAVA_<NAME>``
variables, read ONCE when the library is loaded (``tools/ab_env.sh``).
"""
import contextlib
import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before the library, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEBUG_ENV = os.environ.get("DAVA_DEBUG_OVERRIDES") == "1"  # the one gate: A/B and diagnostic runs only
# DAVA_LIB (with the gate): another build of the library, for A/B runs (tools/build_prev.sh)
LIB_PATH = (_DEBUG_ENV and os.environ.get("DAVA_LIB")) or os.path.join(_HERE, "_lib", "libdava_ba.so")

# Overridable launch choices of the library (csrc/dava_debug.hpp), and of this package's Python side
LIBRARY_KNOBS = ("FORCE_GV", "GV_NO_XL", "SOLVE_WAVES", "WG_PER_CU", "LDS_HISTORY", "STAGGER", "STAGGER_LEVELS",
                 "NO_PPT", "NO_QUEUE", "ADJ_GV_WAVES", "ADJ_FORCE_GV", "ADJ_LDS_ENTRIES", "ADJ_GD_HBM",
                 "COMPACT_SWITCH", "GV_SCALAR_SLICE", "ADJ_SC_GLOBAL")
# GENERIC_BACKWARD: differentiate a fused objective's solve with the generic loop, not the adjoint;
# GENERIC_TRAINING: training mode's drop path with the generic loop and torch's own RNG;
# GENERIC_DENSE: the generic loop keeps the reference's dense (B, P, P) inverse Hessian even without a graph
PYTHON_KNOBS = ("GENERIC_BACKWARD", "GENERIC_TRAINING", "GENERIC_DENSE")
_py_knobs = {k: -1 for k in PYTHON_KNOBS}

DAVA_OK = 0
DAVA_HESSIAN_DENSE = 0
DAVA_HESSIAN_COMPACT = 1
DAVA_RESIDUAL_SQUARED_REPROJECTION = 0
DAVA_RESIDUAL_RAY_ANGLE = 1
ABI_VERSION = 4  # include/dava_ba.h DAVA_ABI_VERSION
STOP_ITERATIONS, STOP_ERROR, STOP_STEP, STOP_DROP = 0, 1, 2, 3
STATUS_WORDS = 4

_c_i64 = ctypes.c_int64
_c_i32 = ctypes.c_int32
_vp = ctypes.c_void_p


class DavaScene(ctypes.Structure):
    _fields_ = [
        ("batch", _c_i32),
        ("num_views", _c_i32),
        ("num_points", _c_i32),
        ("distortion", _c_i32),
        ("num_parameters", _c_i32),
        ("observations", _vp),
        ("visibility", _vp),
        ("residual", _c_i32),
    ]


class DavaSolverConfig(ctypes.Structure):
    _fields_ = [
        ("sufficient_decrease", ctypes.c_float),
        ("curvature", ctypes.c_float),
        ("error_threshold", ctypes.c_float),
        ("minimum_step", ctypes.c_float),
        ("iterations", _c_i32),
        ("max_line_search_trials", _c_i32),
        ("strong_wolfe", _c_i32),
        ("hessian_mode", _c_i32),
        ("drop_path_p", ctypes.c_float),
        ("drop_seed_lo", ctypes.c_uint32),
        ("drop_seed_hi", ctypes.c_uint32),
        ("return_second_last", _c_i32),
    ]


class DavaSolvePlan(ctypes.Structure):
    _fields_ = [
        ("global_vectors", _c_i32),
        ("workgroup_threads", _c_i32),
        ("lds_bytes", _c_i32),
        ("lds_history_entries", _c_i32),
    ]


# name -> (restype, argtypes); every symbol declared in include/dava_ba.h
SIGNATURES = {
    "dava_ba_solve_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig)]),
    "dava_ba_solve_plan": (ctypes.c_int, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig),
                                          ctypes.POINTER(DavaSolvePlan)]),
    "dava_ba_solve": (ctypes.c_int, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig), _vp, _vp, _vp, _vp,
                                     _vp, ctypes.c_size_t, _vp]),
    "dava_ba_evaluate": (ctypes.c_int, [ctypes.POINTER(DavaScene), _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dava_ba_second_order": (ctypes.c_int, [ctypes.POINTER(DavaScene)] + [_vp] * 8),
    "dava_ba_second_order_obs": (ctypes.c_int, [ctypes.POINTER(DavaScene)] + [_vp] * 9),
    "dava_ba_solve_tape_bytes": (ctypes.c_size_t, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig)]),
    "dava_ba_solve_record": (ctypes.c_int, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig), _vp, _vp,
                                            _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "dava_ba_solve_backward_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(DavaScene),
                                                                 ctypes.POINTER(DavaSolverConfig)]),
    "dava_ba_solve_backward": (ctypes.c_int, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig), _vp,
                                              ctypes.c_size_t, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "dava_ba_solve_backward_lds_entries": (ctypes.c_int, [ctypes.POINTER(DavaScene), ctypes.POINTER(DavaSolverConfig)]),
    "dava_debug_set_override": (ctypes.c_int, [ctypes.c_char_p, _c_i64]),
    "dava_debug_clear_overrides": (None, []),
    "dava_abi_version": (ctypes.c_int, []),
    "dava_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "dava_device_arch": (ctypes.c_char_p, []),
}
for _t in ("f32", "f64"):
    _scalar = ctypes.c_float if _t == "f32" else ctypes.c_double
    SIGNATURES.update({
        f"dava_bfgs_update_inverse_hessian_{_t}": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp]),
        f"dava_bfgs_update_inverse_hessian_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 8),
        f"dava_l1_camera_evaluate_{_t}": (ctypes.c_int, [_c_i64, _c_i32, _c_i32, _c_i32] + [_vp] * 8
                                          + [_scalar] * 4 + [_vp, _vp, _vp]),
        f"dava_l1_camera_vjp_{_t}": (ctypes.c_int, [_c_i64, _c_i32, _c_i32, _c_i32] + [_vp] * 8 + [_scalar] * 4
                                     + [_vp, _vp, _c_i32, _vp, _vp]),
        f"dava_bfgs_initial_scale_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 6),
        f"dava_bfgs_scale_matrix_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 6),
        f"dava_bfgs_search_direction_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 6),
        f"dava_bfgs_initial_scale_{_t}": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
        f"dava_bfgs_scale_matrix_{_t}": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
        f"dava_bfgs_search_direction_{_t}": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
        f"dava_bfgs_compact_direction_{_t}": (ctypes.c_int, [_c_i64] * 5 + [_vp] * 11),
        f"dava_wolfe_init_{_t}": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
        f"dava_wolfe_propose_{_t}": (ctypes.c_int, [_c_i64, _vp, _vp, _vp]),
        f"dava_wolfe_update_{_t}": (ctypes.c_int, [_c_i64, _c_i32, _scalar, _scalar, _c_i32, _vp, _vp, _vp]),
        # host-memory flavours (csrc/bfgs_host.hip): the same signatures without the stream
        f"dava_cpu_bfgs_update_inverse_hessian_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 4),
        f"dava_cpu_bfgs_update_inverse_hessian_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 7),
        f"dava_cpu_bfgs_initial_scale_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 3),
        f"dava_cpu_bfgs_initial_scale_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 5),
        f"dava_cpu_bfgs_scale_matrix_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 3),
        f"dava_cpu_bfgs_scale_matrix_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 5),
        f"dava_cpu_bfgs_search_direction_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 3),
        f"dava_cpu_bfgs_search_direction_backward_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 5),
        f"dava_cpu_wolfe_init_{_t}": (ctypes.c_int, [_c_i64, _c_i64] + [_vp] * 5),
        f"dava_cpu_wolfe_propose_{_t}": (ctypes.c_int, [_c_i64, _vp, _vp]),
        f"dava_cpu_wolfe_update_{_t}": (ctypes.c_int, [_c_i64, _c_i32, _scalar, _scalar, _c_i32, _vp, _vp]),
    })

_lock = threading.Lock()
_lib = None


class NativeLibraryError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load and type the C ABI.  Raises NativeLibraryError if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeLibraryError(
                f"{path} not found: build it with `make -C deep-attention-visual-odometry_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if path != _DEFAULT_LIB and not hasattr(lib, name):
                continue  # an older A/B build (tools/build_prev.sh) may predate some entry points
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dava_abi_version() != ABI_VERSION:
            raise NativeLibraryError("libdava_ba.so ABI version mismatch")
        _lib = lib
        if _DEBUG_ENV:  # A/B runs: the DAVA_<NAME> variables, read once, here
            for k in LIBRARY_KNOBS + PYTHON_KNOBS:
                v = os.environ.get("DAVA_" + k)
                if v is None:
                    continue
                v = int(v) if v.lstrip("-").isdigit() else 1
                if k in PYTHON_KNOBS:
                    _py_knobs[k] = v
                elif hasattr(lib, "dava_debug_set_override"):
                    lib.dava_debug_set_override(k.encode(), v)
        return lib


_DEFAULT_LIB = os.path.join(_HERE, "_lib", "libdava_ba.so")


def set_debug_override(name: str, value: int) -> None:
    """Override one launch choice (LIBRARY_KNOBS, PYTHON_KNOBS); value < 0 restores the default."""
    if name in PYTHON_KNOBS:
        _py_knobs[name] = int(value) if value >= 0 else -1
        return
    if name not in LIBRARY_KNOBS:
        raise ValueError(f"unknown override {name!r}")
    lib = load_library()
    if hasattr(lib, "dava_debug_set_override"):
        check(lib.dava_debug_set_override(name.encode(), int(value)), "dava_debug_set_override")


def clear_debug_overrides() -> None:
    for k in PYTHON_KNOBS:
        _py_knobs[k] = -1
    lib = load_library()
    if hasattr(lib, "dava_debug_clear_overrides"):
        lib.dava_debug_clear_overrides()


def python_knob(name: str) -> bool:
    """Is the Python-side override `name` (PYTHON_KNOBS) switched on?"""
    return _py_knobs[name] > 0


@contextlib.contextmanager
def debug_overrides(**knobs):
    """with debug_overrides(FORCE_GV=1, SOLVE_WAVES=2): ... -- tests only; cleared on exit."""
    try:
        for k, v in knobs.items():
            set_debug_override(k, int(v))
        yield
    finally:
        for k in knobs:
            set_debug_override(k, -1)


def check(status: int, what: str) -> None:
    if status != DAVA_OK:
        msg = load_library().dava_status_string(status).decode()
        raise RuntimeError(f"{what} failed: {msg} (status {status})")


def require_host_or_device_tensor(t: torch.Tensor, what: str) -> None:
    """The generic building blocks run on ROCm tensors (HIP kernels) and on CPU tensors (the library's
    host flavours, csrc/bfgs_host.hip) -- chosen by the tensor's device, never as a fallback."""
    if not isinstance(t, torch.Tensor) or t.device.type not in ("cuda", "cpu"):
        raise RuntimeError(f"{what} must be a ROCm device or CPU tensor; got {getattr(t, 'device', type(t))}")


def require_device_tensor(t: torch.Tensor, what: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(
            f"{what} must be a ROCm device tensor: this solver runs only on the GPU (no CPU fallback); "
            f"got {getattr(t, 'device', type(t))}")


def stream_of(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())
