"""The C-ABI library loads and exports exactly what include/dava_ba.h declares (CPU only).

No compute is launched here: only argument validation paths that return
before touching a device."""
import ctypes
import os
import re

import pytest

from conftest import REPO


def _declared_symbols():
    text = open(os.path.join(REPO, "include", "dava_ba.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dava_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from deep_attention_visual_odometry_amd import _native

    return _native.load_library()


def test_header_declares_the_expected_entry_points():
    syms = _declared_symbols()
    for name in ("dava_ba_solve", "dava_ba_solve_workspace_bytes", "dava_ba_evaluate",
                 "dava_bfgs_update_inverse_hessian_f32", "dava_bfgs_update_inverse_hessian_f64",
                 "dava_wolfe_update_f32", "dava_abi_version"):
        assert name in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_types_every_declared_symbol():
    from deep_attention_visual_odometry_amd import _native

    assert sorted(_native.SIGNATURES) == _declared_symbols()


def test_library_is_built_for_gfx950(lib):
    assert lib.dava_device_arch() == b"gfx950"
    assert lib.dava_abi_version() == 4
    blob = open(lib._name, "rb").read()
    assert b"gfx950" in blob


def test_status_strings(lib):
    assert lib.dava_status_string(0) == b"ok"
    assert b"invalid" in lib.dava_status_string(1)
    assert lib.dava_status_string(99) == b"unknown status"


def test_invalid_arguments_are_rejected_without_a_device(lib):
    from deep_attention_visual_odometry_amd import _native as N

    assert lib.dava_ba_solve(None, None, None, None, None, None, None, 0, None) == 1
    bad = N.DavaScene(4, 1, 16, 0, 3 + 48, None, None)  # one view
    cfg = N.DavaSolverConfig(1e-4, 0.9, 1e-4, 1e-8, 10, 1000, 1, 0)
    assert lib.dava_ba_solve(ctypes.byref(bad), ctypes.byref(cfg), None, None, None, None, None, 0, None) == 1
    wrong_p = N.DavaScene(4, 2, 16, 0, 50, None, None)
    assert lib.dava_ba_evaluate(ctypes.byref(wrong_p), None, None, None, None, None, None, None) == 1
    empty = N.DavaScene(0, 2, 16, 0, 3 + 48 + 6, None, None)
    assert lib.dava_ba_solve(ctypes.byref(empty), ctypes.byref(cfg), None, None, None, None, None, 0, None) == 0
    bad_residual = N.DavaScene(0, 2, 16, 0, 3 + 48 + 6, None, None, 7)
    assert lib.dava_ba_solve(ctypes.byref(bad_residual), ctypes.byref(cfg), None, None, None, None, None, 0, None) == 1
    ray_distorted = N.DavaScene(0, 2, 16, 1, 3 + 48 + 6 + 5, None, None, N.DAVA_RESIDUAL_RAY_ANGLE)
    assert lib.dava_ba_solve(ctypes.byref(ray_distorted), ctypes.byref(cfg), None, None, None, None, None, 0, None) == 4
    assert lib.dava_bfgs_update_inverse_hessian_f32(-1, 3, None, None, None, None, None) == 1
    assert lib.dava_bfgs_update_inverse_hessian_f64(0, 3, None, None, None, None, None) == 0


def test_workspace_size_dense(lib):
    from deep_attention_visual_odometry_amd import native_ops

    p = 3 + 3 * 256 + 6 * 3 + 5
    # dense inverse Hessians + the 256-byte work-queue counter
    assert native_ops.solve_workspace_bytes(8192, 4, 256, True) == 8192 * p * ((p + 31) // 32 * 32) * 4 + 256


def test_workspace_size_compact_and_hybrid(lib, overrides):
    """COMPACT keeps one history entry per update up to 1024 (2 rows of Pv floats each); past 1025
    iterations it is HYBRID: the 1024-entry history plus the dense matrices it folds into.  The
    COMPACT_SWITCH override lowers the capacity (the GPU tests' switch at K = 30); a hybrid solve has
    no tape (the adjoint reads the history of every step)."""
    from deep_attention_visual_odometry_amd import native_ops

    b, m, n = 64, 4, 256
    p = 3 + 3 * n + 6 * (m - 1) + 5
    pv, pld = (p + 3) // 4 * 4, (p + 31) // 32 * 32
    dense = b * p * pld * 4
    ws = lambda k: native_ops.solve_workspace_bytes(b, m, n, True, 1, k)  # noqa: E731
    assert ws(100) == b * 2 * 99 * pv * 4 + 256
    assert ws(1025) == b * 2 * 1024 * pv * 4 + 256
    assert ws(1026) == ws(5000) == b * 2 * 1024 * pv * 4 + dense + 256
    assert native_ops.solve_plan(b, m, n, True, 1, 5000)["workgroup_threads"] == 256  # no longer refused
    sc = native_ops.scene_struct(None, None, m, n, True, b)
    tape = lambda k: lib.dava_ba_solve_tape_bytes(  # noqa: E731
        sc, native_ops.solver_config(1e-4, 0.9, -1.0, k, -1.0, 1000, True, 1))
    assert tape(30) > 0 and tape(1025) > 0 and tape(1026) == 0
    overrides("COMPACT_SWITCH", 8)
    assert ws(30) == b * 2 * 8 * pv * 4 + dense + 256
    assert ws(9) == b * 2 * 8 * pv * 4 + 256
    assert tape(30) == 0 and tape(9) > 0


def test_c5_keeps_its_lds_image_at_any_iteration_cap(lib):
    """C5 (P = 12,381, global-vector mode): the LDS image keeps x, d and the gradient (XL, 3 Pv floats) at
    every cap.  The history's rho_j, c_j stay in LDS while they fit beside it (8 B per entry; the product
    coefficients are not reserved for the single-pass forms) and past ~950 iterations -- the reference's
    default 1,000 included -- move to the workspace slice (2 x round_up(K - 1, 64) floats per problem after
    its 9 vectors)."""
    from deep_attention_visual_odometry_amd import native_ops

    b, m, n = 256, 16, 4096
    p = 3 + 3 * n + 6 * (m - 1)
    pv = (p + 3) // 4 * 4
    plan = {k: native_ops.solve_plan(b, m, n, False, 1, k) for k in (100, 400, 900, 1000, 2000)}
    assert all(3 * pv * 4 < q["lds_bytes"] <= 160 * 1024 for q in plan.values()), plan
    assert plan[1000]["lds_bytes"] == plan[2000]["lds_bytes"] < plan[100]["lds_bytes"] < plan[400]["lds_bytes"]
    ws = lambda k: native_ops.solve_workspace_bytes(b, m, n, False, 1, k)  # noqa: E731
    assert ws(100) == b * 9 * pv * 4 + b * 2 * 99 * pv * 4 + 256
    assert ws(400) == b * 9 * pv * 4 + b * 2 * 399 * pv * 4 + 256
    assert ws(1000) == b * (9 * pv + 2 * 1024) * 4 + b * 2 * 999 * pv * 4 + 256


def test_solve_plan(lib, overrides):
    """Host-only plan query: C3 keeps its oldest history entries in LDS within two workgroups
    per CU; C5 (P = 12381) runs the O(P) state from HBM in 512-thread workgroups."""
    from deep_attention_visual_odometry_amd import native_ops

    overrides("LDS_HISTORY", -1)
    c3 = native_ops.solve_plan(8192, 4, 256, True, 1, 100)
    assert c3["global_vectors"] == 0 and c3["workgroup_threads"] == 256
    assert c3["lds_history_entries"] > 0 and c3["lds_bytes"] <= 80 * 1024
    assert native_ops.solve_plan(8192, 4, 256, True, 0, 100)["lds_history_entries"] == 0  # dense
    c5 = native_ops.solve_plan(256, 16, 4096, False, 1, 100)
    assert c5["global_vectors"] == 1 and c5["workgroup_threads"] == 512 and c5["lds_history_entries"] == 0
    # two waves while a history row is at most 128 float4 column groups: C1 (P = 201), C2 (P = 393)
    overrides("SOLVE_WAVES", -1)
    assert native_ops.solve_plan(1024, 2, 64, False, 1, 100)["workgroup_threads"] == 128
    assert native_ops.solve_plan(1024, 2, 128, False, 1, 100)["workgroup_threads"] == 128
    assert native_ops.solve_plan(1024, 2, 128, False, 0, 100)["workgroup_threads"] == 256  # dense keeps 4
    overrides("SOLVE_WAVES", 4)
    assert native_ops.solve_plan(1024, 2, 64, False, 1, 100)["workgroup_threads"] == 256
    overrides("LDS_HISTORY", 1000)  # clamped to one workgroup's LDS
    big = native_ops.solve_plan(8192, 4, 256, True, 1, 100)
    assert big["lds_bytes"] <= 160 * 1024 and big["lds_history_entries"] > c3["lds_history_entries"]


def test_adjoint_shapes(lib):
    """Host-only: which shapes have the fused adjoint.  C3 (P = 794) runs it with the O(P) vectors in
    LDS; C5 (P = 12381, the forward's global-vector mode) with them in the adjoint's workspace, and its
    tape holds the forward's vector slices too; past P = 14336 (14 float4 groups per thread) there is
    none, and the dense mode never records."""
    from deep_attention_visual_odometry_amd import _native as N, native_ops

    assert native_ops.solve_tape_supported(8192, 4, 256, True, 100)
    assert native_ops.solve_tape_supported(256, 16, 4096, False, 100)
    assert not native_ops.solve_tape_supported(2, 16, 5000, False, 100)  # P = 15093
    sc = native_ops.scene_struct(None, None, 16, 4096, False, 256, N.DAVA_RESIDUAL_SQUARED_REPROJECTION)
    cfg = native_ops.solver_config(1e-4, 0.9, -1.0, 100, -1.0, 1000, True, N.DAVA_HESSIAN_COMPACT)
    p, pv, k = 12381, 12384, 100
    t = (3 * k + 1 + 3) // 4 * 4
    floats = 256 * (2 * (k - 1) * pv + 2 * k * pv + t + 9 * pv)  # history, x, g, scalars, GV vectors
    assert lib.dava_ba_solve_tape_bytes(sc, cfg) == floats * 4 + 256
    # adjoint workspace: the a rows (B, K, Pv) plus 18 Pv floats of vectors per problem
    assert lib.dava_ba_solve_backward_workspace_bytes(sc, cfg) == 256 * (k + 18) * pv * 4 + 256
    assert lib.dava_ba_solve_backward_lds_entries(sc, cfg) == 0
    cfg_dense = native_ops.solver_config(1e-4, 0.9, -1.0, 100, -1.0, 1000, True, N.DAVA_HESSIAN_DENSE)
    assert lib.dava_ba_solve_tape_bytes(sc, cfg_dense) == 0


def test_fused_kernels_refuse_cpu_tensors():
    """The fused solve and evaluation are GPU kernels: handed CPU tensors they raise, they never run elsewhere.
    (BFGSSolver with a fused objective on CPU tensors takes the generic loop and the objective's torch form by
    design, tests/test_cpu_solver.py -- not these kernels.)"""
    import torch

    from deep_attention_visual_odometry_amd import native_ops

    obs = torch.zeros(1, 2, 4, 2)
    vis = torch.ones(1, 2, 4, dtype=torch.bool)
    with pytest.raises(RuntimeError, match="ROCm device"):
        native_ops.ba_solve(torch.zeros(1, 3 + 12 + 6), obs, vis, 2, 4, False)
    with pytest.raises(RuntimeError, match="ROCm device"):
        native_ops.ba_evaluate(torch.zeros(1, 3 + 12 + 6), obs, vis, 2, 4, False)


def test_unpack_matches_reference_layout():
    import torch

    from deep_attention_visual_odometry_amd import unpack_calibration_parameters

    x = torch.arange(3 + 3 * 5 + 6 * 2, dtype=torch.float32).reshape(1, -1)
    parts = unpack_calibration_parameters(x, 3, 5)
    assert parts.intrinsics.shape == (1, 1, 1, 3)
    assert parts.world_points.shape == (1, 1, 5, 3)
    assert parts.camera_translations.shape == (1, 2, 1, 3)
    assert parts.camera_rotations.shape == (1, 2, 1, 3)
    assert parts.camera_rotations[0, 1, 0, 2].item() == x[0, -1].item()
    with pytest.raises(ValueError):
        unpack_calibration_parameters(x[:, :-1], 3, 5)


# ---- the operator boundary (torch.ops.dava, _ops.py): registration and fake kernels, no device ----

def test_every_operator_is_registered():
    import torch

    from deep_attention_visual_odometry_amd import _ops

    for name in _ops.OPS:
        op = getattr(torch.ops.dava, name)
        assert op.default._schema.name == f"dava::{name}"


def test_fake_kernels_give_output_shapes_without_a_device():
    """Under FakeTensorMode (what torch.compile traces with) every operator -- and the whole fused
    BFGSSolver forward on ReprojectionError -- runs on fake ROCm tensors and yields the shapes and
    dtypes the HIP kernels produce, with no GPU and no library call."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode

    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    with FakeTensorMode():
        dev = "cuda"
        x = torch.empty(5, 3 + 3 * 16 + 6, device=dev)
        obs = torch.empty(5, 2, 16, 2, device=dev)
        vis = torch.empty(5, 2, 16, dtype=torch.uint8, device=dev)
        ws = torch.empty(0, dtype=torch.uint8, device=dev)
        xo, err, st = torch.ops.dava.ba_solve(x, obs, vis, 2, 16, False, 1e-4, 0.9, -1.0, 7, -1.0, 1000, True, 1, 0,
                                              False, ws)
        assert xo.shape == x.shape and err.shape == (0,) and st.shape == (5, 4) and st.dtype == torch.int32
        xo, st = torch.ops.dava.bfgs_solve(x, obs, vis, 2, 16)
        assert xo.shape == x.shape and st.shape == (5, 4) and st.dtype == torch.int32
        e, g, sl = torch.ops.dava.ba_evaluate(x, obs, vis, 2, 16, False, x, None, True, True, 0)
        assert e.shape == (5,) and g.shape == x.shape and sl.shape == (5,)
        e, g, hv, og, ohv = torch.ops.dava.ba_second_order(x, obs, vis, 2, 16, False, None, 0, False, True)
        assert hv.shape == (0,) and og.shape == obs.shape and ohv.shape == (0,)
        h = torch.empty(4, 6, 6, device=dev, dtype=torch.float64)
        v = torch.empty(4, 6, device=dev, dtype=torch.float64)
        assert torch.ops.dava.bfgs_update_inverse_hessian(h, v, v).shape == h.shape
        assert torch.ops.dava.bfgs_initial_scale(v, v).shape == (4,)
        assert torch.ops.dava.bfgs_search_direction(h, v).shape == v.shape
        gh, gs, gy = torch.ops.dava.bfgs_update_inverse_hessian_backward(h, v, v, h, True, False, True)
        assert gh.shape == h.shape and gs.shape == (0,) and gy.shape == v.shape
        state, flags = torch.ops.dava.wolfe_init(v, v[:, 0].contiguous(), v)
        assert state.shape == (4, 9) and flags.shape == (4, 2) and flags.dtype == torch.uint8
        fe, fg = torch.ops.dava.l1_camera_evaluate(*(torch.empty(2, 3, device=dev),) * 3,
                                                   torch.empty(2, 3, 4, 3, device=dev),
                                                   torch.empty(2, 3, 4, 3, device=dev),
                                                   torch.empty(2, 3, 6, 3, device=dev),
                                                   torch.empty(2, 4, 8, 2, device=dev),
                                                   torch.empty(2, 4, 8, dtype=torch.uint8, device=dev),
                                                   0.1, 1e3, 1e3, 1.0, True, True)
        assert fe.shape == (2, 3) and fg.shape == (2, 3, 3 + 6 * 4 + 3 * 8 - 7)
        vj = torch.ops.dava.l1_camera_vjp(*(torch.empty(2, 3, device=dev),) * 3, torch.empty(2, 3, 4, 3, device=dev),
                                          torch.empty(2, 3, 4, 3, device=dev), torch.empty(2, 3, 6, 3, device=dev),
                                          torch.empty(2, 4, 8, 2, device=dev),
                                          torch.empty(2, 4, 8, dtype=torch.uint8, device=dev), 0.1, 1e3, 1e3, 1.0,
                                          torch.empty(2, 3, device=dev), None, False)
        assert vj.shape == (2, 3, 3 + 6 * 4 + 3 * 6)
        fn = ReprojectionError(obs, vis, 2, 16)
        out = BFGSSolver(iterations=7, error_threshold=-1.0, minimum_step=-1.0).eval()(x, fn)
        assert out.shape == x.shape and out.device.type == "cuda"


def test_operator_shape_checks_run_before_any_launch():
    """Mis-shaped scene tensors are refused on the host, before the library is even asked."""
    import pytest as _pytest
    import torch

    from deep_attention_visual_odometry_amd import _ops

    x = torch.zeros(2, 3 + 3 * 16 + 6)
    with _pytest.raises(ValueError):
        _ops._check_scene_tensors(x, torch.zeros(2, 2, 15, 2), torch.zeros(2, 2, 15, dtype=torch.uint8), 2, 16, False)
    with _pytest.raises(ValueError):
        _ops._check_scene_tensors(x[:, :-1], torch.zeros(2, 2, 16, 2), torch.zeros(2, 2, 16, dtype=torch.uint8), 2,
                                  16, False)
    with _pytest.raises(TypeError):
        _ops._check_scene_tensors(x, torch.zeros(2, 2, 16, 2, dtype=torch.float64),
                                  torch.zeros(2, 2, 16, dtype=torch.uint8), 2, 16, False)


def test_launch_choices_ignore_the_environment():
    """The library reads no environment and the binding reads the DAVA_<NAME> overrides only behind
    DAVA_DEBUG_OVERRIDES=1: a user's stray DAVA_FORCE_GV / DAVA_SOLVE_WAVES / DAVA_LIB changes nothing."""
    import json
    import subprocess
    import sys

    from conftest import SRC

    code = ("import sys, json; sys.path.insert(0, %r)\n"
            "from deep_attention_visual_odometry_amd import native_ops, _native\n"
            "print(json.dumps([native_ops.solve_plan(8192, 4, 256, True, 1, 100),"
            " native_ops.solve_plan(1024, 2, 128, False, 1, 100), _native.LIB_PATH]))") % SRC
    env = dict(os.environ, DAVA_FORCE_GV="1", DAVA_SOLVE_WAVES="4", DAVA_LIB="/nonexistent/libdava_ba.so",
               DAVA_GENERIC_BACKWARD="1")
    env.pop("DAVA_DEBUG_OVERRIDES", None)
    c3, c2, path = json.loads(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                             check=True, timeout=120).stdout.strip().splitlines()[-1])
    assert c3["global_vectors"] == 0 and c2["workgroup_threads"] == 128 and path.endswith("_lib/libdava_ba.so")
    env.update(DAVA_DEBUG_OVERRIDES="1")
    env.pop("DAVA_LIB")
    c3, c2, _ = json.loads(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                          check=True, timeout=120).stdout.strip().splitlines()[-1])
    assert c3["global_vectors"] == 1 and c2["global_vectors"] == 1  # the A/B gate: read once, at load


def test_debug_overrides_are_scoped(lib):
    from deep_attention_visual_odometry_amd import _native, native_ops

    base = native_ops.solve_plan(8192, 4, 256, True, 1, 100)
    with _native.debug_overrides(FORCE_GV=1, GENERIC_BACKWARD=1):
        assert native_ops.solve_plan(8192, 4, 256, True, 1, 100)["global_vectors"] == 1
        assert _native.python_knob("GENERIC_BACKWARD")
    assert native_ops.solve_plan(8192, 4, 256, True, 1, 100) == base
    assert not _native.python_knob("GENERIC_BACKWARD")
    with pytest.raises(ValueError):
        _native.set_debug_override("NOT_A_KNOB", 1)
    assert lib.dava_debug_set_override(b"NOT_A_KNOB", 1) == 1


@pytest.mark.parametrize("m", [200, 260, 300, 336])
def test_adjoint_support_matches_its_launch_image(lib, m):
    """Many views (the eight-wave global-vector image grows with the per-wave view partials): the size
    queries accept a shape only if the launch that will run fits the LDS -- eight waves where they fit,
    else four -- so a recorded forward never meets a backward that cannot launch."""
    from deep_attention_visual_odometry_amd import native_ops

    n = 64
    assert native_ops.solve_tape_supported(2, m, n, False, 50)
    from deep_attention_visual_odometry_amd import _native as N

    sc = native_ops.scene_struct(None, None, m, n, False, 2, N.DAVA_RESIDUAL_SQUARED_REPROJECTION)
    cfg = native_ops.solver_config(1e-4, 0.9, -1.0, 50, -1.0, 1000, True, N.DAVA_HESSIAN_COMPACT)
    assert lib.dava_ba_solve_backward_workspace_bytes(sc, cfg) > 0


def test_generic_fallback_check_sizes_the_first_iterations(monkeypatch):
    """BFGSSolver._check_generic_fits refuses only what cannot fit even at the first iterations and warns
    (does not refuse) when only the iteration cap would not fit."""
    import warnings

    import torch

    from deep_attention_visual_odometry_amd.autograd_solvers import bfgs_solver as mod

    monkeypatch.setattr(mod, "_free_device_bytes", lambda device: 192 * 2.0 ** 30)
    s = mod.BFGSSolver(hessian_mode="dense").eval()
    x = torch.zeros(64, 789, requires_grad=True)  # C3 pinhole, B = 64: 0.16 GB per dense matrix
    with pytest.warns(RuntimeWarning, match="stop"):
        s._check_generic_fits(x, 1000)  # 3 x 1000 matrices would not fit; the run still goes ahead
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        s._check_generic_fits(x, 100)  # fits outright
    with pytest.raises(RuntimeError, match="first temporaries"):
        s._check_generic_fits(torch.zeros(48, 15093, requires_grad=True), 100)
    with pytest.raises(RuntimeError, match="return_second_last"):
        mod.BFGSSolver()._check_generic_fits(torch.zeros(48, 15093), 100, second_last=True)
