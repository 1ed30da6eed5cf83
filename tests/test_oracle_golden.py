"""The CPU oracle against golden vectors produced by the real reference.

These run without a GPU.  They pin ``oracle/`` (the checker every GPU parity
test compares against) to the reference's own outputs.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import objective, solver

SHAPES = {"c1": (2, 64), "c2": (2, 128), "c3": (4, 256)}


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_objective_and_gradient_match_reference_bitwise(shape, dt):
    g = _load("ba_eval.npz")
    m, n = SHAPES[shape]
    key = f"{shape}_{dt}"
    x = torch.tensor(g[key + "_x"]).requires_grad_(True)
    e = objective.reprojection_error(x, torch.tensor(g[key + "_obs"]), torch.tensor(g[key + "_vis"]), m, n)
    (grad,) = torch.autograd.grad(e.sum(), x)
    assert np.array_equal(e.detach().numpy(), g[key + "_err"])
    assert np.array_equal(grad.numpy(), g[key + "_grad"])


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("p", [3, 17, 64])
def test_bfgs_update_matches_reference_bitwise(dt, p):
    g = _load("bfgs_update.npz")
    key = f"{dt}_p{p}"
    h, s, y = (torch.tensor(g[key + k]) for k in ("_h", "_s", "_y"))
    assert np.array_equal(solver.bfgs_update(h, s, y).numpy(), g[key + "_out"])
    assert np.array_equal(solver.initial_scale(s, y).numpy(), g[key + "_scale"])
    # problem 1 has negative curvature: the update is skipped exactly
    assert np.array_equal(g[key + "_out"][1], g[key + "_h"][1])


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("strong", [True, False])
def test_line_search_matches_reference_bitwise(shape, dt, strong):
    g = _load("line_search.npz")
    m, n = SHAPES[shape]
    key = f"{shape}_{dt}"
    obs = torch.tensor(g[key + "_obs"])
    vis = torch.tensor(g[key + "_vis"])
    fn = objective.ReprojectionClosure(obs, vis, m, n)
    alpha = solver.wolfe_line_search(
        torch.tensor(g[key + "_x"]), torch.tensor(g[key + "_dir"]), torch.tensor(g[key + "_err"]),
        torch.tensor(g[key + "_grad"]), fn, strong=strong,
    )
    ref = g[f"{key}_{'strong' if strong else 'weak'}_alpha"]
    assert np.array_equal(alpha.numpy(), ref)
    assert abs(ref[2]) < 1e-30  # uphill direction -> bisects down to (almost) no step


@pytest.mark.parametrize("case,ks", [("c1", (5, 20, 100)), ("c2", (5, 20, 100)), ("c3", (5, 20))])
def test_bfgs_trajectories_match_reference_bitwise(case, ks):
    g = _load("bfgs_traj.npz")
    m, n = SHAPES[case]
    x0 = torch.tensor(g[case + "_x0"])
    fn = objective.ReprojectionClosure(torch.tensor(g[case + "_obs"]), torch.tensor(g[case + "_vis"]), m, n)
    for k in ks:
        if case == "c3" and k > 5:
            continue  # keep the CPU suite short; k=20 for c3 is covered by the GPU parity tests
        out = solver.bfgs_solve(x0, fn, iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        assert np.array_equal(out.numpy(), g[f"{case}_k{k}"]), f"{case} K={k}"


def test_bfgs_default_thresholds_match_reference_bitwise():
    g = _load("bfgs_traj.npz")
    m, n = SHAPES["c1"]
    fn = objective.ReprojectionClosure(torch.tensor(g["c1def_obs"]), torch.tensor(g["c1def_vis"]), m, n)
    out = solver.bfgs_solve(torch.tensor(g["c1def_x0"]), fn)
    assert np.array_equal(out.numpy(), g["c1def_out"])


def test_bfgs_textbook_kat():
    """Known-answer test of the reference (tests/autograd_solvers/test_bfgs_solver.py:307-332)."""
    s = torch.tensor([-1.26262069, -0.78272035, 0.98543104], dtype=torch.float64)
    y = torch.tensor([0.15339519, -0.28944666, 0.54194925], dtype=torch.float64)
    h = torch.tensor([[2.0, 1.0, 0.0], [1.0, 1.0, 0.0], [0.0, 0.0, 3.0]], dtype=torch.float64)
    c = (s * y).sum()
    left = torch.eye(3, dtype=torch.float64) - (s[:, None] * y[None, :]) / c
    right = torch.eye(3, dtype=torch.float64) - (y[:, None] * s[None, :]) / c
    expected = left @ h @ right + s[:, None] * s[None, :] / c
    assert torch.isclose(expected, solver.bfgs_update(h, s, y)).all()


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_ray_angle_objective_matches_reference_bitwise(shape, dt):
    """CalibrationNetwork's error (calibration_network.py:58-67) and its autograd gradient."""
    g = _load("ray_angle.npz")
    m, n = SHAPES[shape]
    key = f"eval_{shape}_{dt}"
    x = torch.tensor(g[key + "_x"]).requires_grad_(True)
    e = objective.ray_angle_error(x, torch.tensor(g[key + "_obs"]), torch.tensor(g[key + "_vis"]), m, n)
    (grad,) = torch.autograd.grad(e.sum(), x)
    assert np.array_equal(e.detach().numpy(), g[key + "_err"])
    assert np.array_equal(grad.numpy(), g[key + "_grad"])


@pytest.mark.parametrize("case,ks", [("c1", (5, 20, 100)), ("c2", (5, 20))])
def test_ray_angle_trajectories_match_reference_bitwise(case, ks):
    g = _load("ray_angle.npz")
    m, n = SHAPES[case]
    key = f"traj_{case}"
    x0 = torch.tensor(g[key + "_x0"])
    fn = objective.RayAngleClosure(torch.tensor(g[key + "_obs"]), torch.tensor(g[key + "_vis"]), m, n)
    for k in ks:
        out = solver.bfgs_solve(x0, fn, iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        assert np.array_equal(out.numpy(), g[f"{key}_k{k}"]), f"{case} K={k}"


def test_gradient_through_the_solve_matches_reference_bitwise():
    """The reference's create_graph mode (bfgs_solver.py:85,134,213-215; its test
    test_bfgs_solver.py:263-273): d loss / d x0 (and d loss / d obs for a closure that
    captures the observations) equal the reference's own autograd result."""
    g = _load("solve_grad.npz")
    x0 = torch.tensor(g["log_x0"]).requires_grad_(True)
    out = solver.bfgs_solve(x0, lambda x, _: (x.square().sum(dim=-1) + 1.0).log(), error_threshold=1e-6)
    out.square().sum().backward()
    assert np.array_equal(out.detach().numpy(), g["log_out"])
    assert np.array_equal(x0.grad.numpy(), g["log_grad"])
    assert (x0.grad.abs() > 0).all()

    x0 = torch.tensor(g["rosen_x0"]).requires_grad_(True)

    def rosen(p, _):
        return (1.0 - p[..., 0]).square() + 100.0 * (p[..., 1] - p[..., 0].square()).square()

    out = solver.bfgs_solve(x0, rosen, iterations=10, error_threshold=-1.0, minimum_step=-1.0)
    (out * torch.tensor(g["rosen_w"])).sum().backward()
    assert np.array_equal(x0.grad.numpy(), g["rosen_grad"])

    x0 = torch.tensor(g["ba_x0"]).requires_grad_(True)
    obs = torch.tensor(g["ba_obs"]).requires_grad_(True)
    fn = objective.ReprojectionClosure(obs, torch.tensor(g["ba_vis"]), 2, 8)
    out = solver.bfgs_solve(x0, fn, iterations=5, error_threshold=-1.0, minimum_step=-1.0)
    (out * torch.tensor(g["ba_w"])).sum().backward()
    assert np.array_equal(out.detach().numpy(), g["ba_out"])
    assert np.array_equal(x0.grad.numpy(), g["ba_grad"])
    assert np.array_equal(obs.grad.numpy(), g["ba_obs_grad"])


TRAINING = {
    "rosen_drop": (dict(drop_path_p=0.3, training_iterations=30, training_error_threshold=1e-3), 9101),
    "rosen_second_last": (dict(drop_path_p=0.0, return_second_last=True, training_iterations=40,
                               training_error_threshold=1e-6), 9102),
    "rosen_both": (dict(drop_path_p=0.2, return_second_last=True, training_iterations=25), 9103),
}


def _oracle_training(x0, fn, kw):
    return solver.bfgs_solve(x0, fn, training=True, drop_path_p=kw.get("drop_path_p", 0.1),
                             return_second_last=kw.get("return_second_last", False),
                             iterations=kw.get("training_iterations", 1000),
                             error_threshold=kw.get("training_error_threshold", 1e-4),
                             minimum_step=kw.get("minimum_step", 1e-8))


@pytest.mark.parametrize("case", list(TRAINING))
def test_training_mode_matches_reference_bitwise(case):
    """Training-mode semantics (bfgs_solver.py:88-93, :121-125, :196-212) with the drop-path
    draws made deterministic (tests/rng_patch.py), including return_second_last's scatter
    of the previous active rows into the new active set."""
    from rng_patch import deterministic_rand_like

    g = _load("training.npz")
    kw, seed = TRAINING[case]

    def rosen(p, _):
        return (1.0 - p[..., 0]).square() + 100.0 * (p[..., 1] - p[..., 0].square()).square()

    with deterministic_rand_like(seed):
        out = _oracle_training(torch.tensor(g["rosen_x0"]), rosen, kw)
    assert np.array_equal(out.numpy(), g[case])


def test_training_mode_ba_drop_path_matches_reference_bitwise():
    from rng_patch import deterministic_rand_like

    g = _load("training.npz")
    fn = objective.ReprojectionClosure(torch.tensor(g["ba_obs"]), torch.tensor(g["ba_vis"]), 2, 64)
    kw = dict(drop_path_p=0.25, training_iterations=12, training_error_threshold=-1.0, minimum_step=-1.0)
    with deterministic_rand_like(9201):
        out = _oracle_training(torch.tensor(g["ba_x0"]), fn, kw)
    assert np.array_equal(out.numpy(), g["ba_drop"])


@pytest.mark.parametrize("case", ["mg1e3", "default", "behind"])
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_camera_l1_error_and_gradient_match_reference_bitwise(case, dt):
    """Legacy PinholeCameraModelL1 (camera_model/pinhole_camera_model_l1.py) get_error and its
    hand-written get_gradient, max_gradient clipping and z clamping included."""
    from oracle import camera_l1

    g = _load("camera_l1.npz")
    key = f"{case}_{dt}"
    kw = {"mg1e3": dict(max_gradient=1e3), "default": dict(), "behind": dict(max_gradient=50.0,
                                                                             minimum_z_distance=0.5)}[case]
    args = [torch.tensor(g[f"{key}_{k}"]) for k in ("focal_length", "cx", "cy", "translation", "lie", "world",
                                                      "true", "vis")]
    ez = {k: v for k, v in kw.items() if k != "max_gradient"}
    err = camera_l1.l1_error(*args, **ez)
    grad = camera_l1.l1_gradient(*args, **kw)
    assert np.array_equal(err.numpy(), g[key + "_error"])
    assert np.array_equal(grad.numpy(), g[key + "_gradient"])


@pytest.mark.parametrize("name", ["ba32", "ray32"])
def test_gradient_through_fp32_solves_matches_reference_bitwise(name):
    g = _load("solve_grad.npz")
    x0 = torch.tensor(g[name + "_x0"]).requires_grad_(True)
    obs = torch.tensor(g[name + "_obs"]).requires_grad_(True)
    vis = torch.tensor(g[name + "_vis"])
    closure = objective.ReprojectionClosure if name == "ba32" else objective.RayAngleClosure
    fn = closure(obs, vis, 2, 8)
    out = solver.bfgs_solve(x0, fn, iterations=5, error_threshold=-1.0, minimum_step=-1.0)
    (out * torch.tensor(g[name + "_w"])).sum().backward()
    assert np.array_equal(out.detach().numpy(), g[name + "_out"])
    assert np.array_equal(x0.grad.numpy(), g[name + "_grad"])
    assert np.array_equal(obs.grad.numpy(), g[name + "_obs_grad"])


@pytest.mark.parametrize("case", ["mg1e3", "default", "behind"])
@pytest.mark.parametrize("flags", ["11", "10", "01"])
def test_camera_l1_autograd_matches_reference(case, flags):
    """Autograd THROUGH PinholeCameraModelL1's error and hand-written gradient (second order),
    with the enable_error_gradients / enable_grad_gradients detaches, fp64."""
    from oracle import camera_l1

    g = _load("camera_l1_autograd.npz")
    kw = {"mg1e3": dict(max_gradient=1e3), "default": dict(), "behind": dict(max_gradient=50.0,
                                                                             minimum_z_distance=0.5)}[case]
    parts = {k: torch.tensor(g[f"{case}_{k}"]) for k in camera_l1.PARAMETERS}
    got = camera_l1.l1_autograd(parts, torch.tensor(g[case + "_true"]), torch.tensor(g[case + "_vis"]),
                                flags[0] == "1", flags[1] == "1", **kw)
    assert bool(g[f"{case}_{flags}_error_requires_grad"]) == (flags[0] == "1")
    for k, a in zip(camera_l1.PARAMETERS, got):
        want = g[f"{case}_{flags}_d_{k}"]
        assert np.allclose(a.numpy(), want, rtol=1e-10, atol=1e-12 * max(np.abs(want).max(), 1.0)), k


# ---- Brown-Conrady, pinned to the reference's own distorted model (tests/golden/distortion.npz) ----

@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_distorted_projection_matches_reference_bitwise(dt):
    """distorted_camera_model.py:24-103 (_full_forward_model, loaded by path with the slot table
    its test lists) on camera rows in the BA's tie (fx = fy = f, s = R = T = 0): u', v' and the
    autograd gradients w.r.t. points and the BA parameters; the f64 case holds a z' == 0 point
    (the model's nudge, :57).  Eager-mode reference bitwise; under TorchScript (the file's
    decorator) the values are the same bits and the gradients within the executor's last-ulp
    reordering."""
    g = _load("distortion.npz")
    key = f"proj_{dt}"
    p = torch.tensor(g[key + "_points"]).requires_grad_(True)
    x = torch.tensor(g[key + "_x"]).requires_grad_(True)
    u, v = objective.distorted_rows(p, objective.camera_rows(x, 1))
    loss = (u * torch.tensor(g[key + "_wu"])).sum() + (v * torch.tensor(g[key + "_wv"])).sum()
    gp, gx = torch.autograd.grad(loss, [p, x])
    assert np.array_equal(u.detach().numpy(), g[key + "_u"])
    assert np.array_equal(v.detach().numpy(), g[key + "_v"])
    assert np.array_equal(gp.numpy(), g[key + "_grad_points"])
    assert np.array_equal(gx.numpy(), g[key + "_grad_x"])
    assert np.array_equal(g[key + "_jit_u"], g[key + "_u"]) and np.array_equal(g[key + "_jit_v"], g[key + "_v"])
    eps = np.finfo(g[key + "_u"].dtype).eps
    for k, got in (("_grad_points", gp), ("_grad_x", gx)):
        jit = g[key + "_jit" + k]
        assert np.abs(got.numpy() - jit).max() <= 64 * eps * np.abs(jit).max(), k
    if dt == "f64":
        assert g[key + "_points"][2, 5, 2] == 0.0 and np.isfinite(g[key + "_u"][2, 5])


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_distorted_objective_and_gradient_match_reference_bitwise(shape, dt):
    """The BA objective with the reference's distorted model (tests/golden/make_golden.py
    ref_objective_bc): error and autograd gradient."""
    g = _load("distortion.npz")
    m, n = SHAPES[shape]
    key = f"eval_{shape}_{dt}"
    x = torch.tensor(g[key + "_x"]).requires_grad_(True)
    e = objective.reprojection_error(x, torch.tensor(g[key + "_obs"]), torch.tensor(g[key + "_vis"]), m, n, True)
    (grad,) = torch.autograd.grad(e.sum(), x)
    assert np.array_equal(e.detach().numpy(), g[key + "_err"])
    assert np.array_equal(grad.numpy(), g[key + "_grad"])
    assert np.array_equal(g[key + "_jit_err"], g[key + "_err"])


def test_distorted_trajectories_match_reference_bitwise():
    """BFGSSolver().eval() on the headline model (C3 + Brown-Conrady, fp32) after K = 5, 20, 100:
    the oracle reproduces the eager-mode reference bit for bit.  The reference's TorchScript mode
    (same forward bits, its own symbolic backward) parts from it by ~1e-7 normwise at K = 100 and
    by up to ~1e-3 on the five distortion coefficients -- the reference's own spread on that block."""
    g = _load("distortion.npz")
    x0 = torch.tensor(g["traj_c3_x0"])
    fn = objective.ReprojectionClosure(torch.tensor(g["traj_c3_obs"]), torch.tensor(g["traj_c3_vis"]), 4, 256, True)
    for k in (5, 20, 100):
        out = solver.bfgs_solve(x0, fn, iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        assert np.array_equal(out.numpy(), g[f"traj_c3_k{k}"]), k
        jit = torch.tensor(g[f"traj_c3_jit_k{k}"]).double()
        rel = (jit - out.double()).norm(dim=-1) / out.double().norm(dim=-1)
        assert rel.max() < 1e-6, (k, rel)


# ---- the headline model under visibility masks and to the reference's stopping rules
#      (tests/golden/distortion_masked.npz) ----

@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_masked_distorted_objective_matches_reference_bitwise(shape, dt):
    """10 % of the (view, point) pairs masked (calibration_network.py:58-67 multiplies by vis)."""
    g = _load("distortion_masked.npz")
    m, n = SHAPES[shape]
    key = f"eval_{shape}_{dt}"
    vis = torch.tensor(g[key + "_vis"])
    assert not vis.all()
    x = torch.tensor(g[key + "_x"]).requires_grad_(True)
    e = objective.reprojection_error(x, torch.tensor(g[key + "_obs"]), vis, m, n, True)
    (grad,) = torch.autograd.grad(e.sum(), x)
    assert np.array_equal(e.detach().numpy(), g[key + "_err"])
    assert np.array_equal(grad.numpy(), g[key + "_grad"])


def test_masked_and_converged_distorted_trajectories_match_reference_bitwise():
    """BFGSSolver().eval() on the headline model with masked pairs after K = 5, 20, 100 and with the
    reference's DEFAULT stopping rules (bfgs_solver.py:53-55), plus the unmasked headline batch run to
    those rules: bit for bit, NaN rows included (2 of the 8 masked problems overflow at a trial point,
    where a masked pair's inf * 0 = NaN, and walk to NaN -- in the reference too)."""
    g = _load("distortion_masked.npz")
    x0 = torch.tensor(g["traj_c3m_x0"])
    fn = objective.ReprojectionClosure(torch.tensor(g["traj_c3m_obs"]), torch.tensor(g["traj_c3m_vis"]), 4, 256, True)
    for k in (5, 20, 100):
        out = solver.bfgs_solve(x0, fn, iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        assert np.array_equal(out.numpy(), g[f"traj_c3m_k{k}"], equal_nan=True), k
    out = solver.bfgs_solve(x0, fn)
    assert np.array_equal(out.numpy(), g["traj_c3m_default"], equal_nan=True)
    assert np.isfinite(g["traj_c3m_default"]).all(axis=1).sum() == 6
    d = _load("distortion.npz")
    fnu = objective.ReprojectionClosure(torch.tensor(d["traj_c3_obs"]), torch.tensor(d["traj_c3_vis"]), 4, 256, True)
    out = solver.bfgs_solve(torch.tensor(d["traj_c3_x0"]), fnu)
    assert np.array_equal(out.numpy(), g["traj_c3_default"])


def test_c5_trajectory_matches_reference_bitwise():
    """The oracle at the C5 shape (16 views x 4096 points, P = 12,381, B = 2, pinhole) after K = 20 against
    the REAL reference's BFGSSolver().eval() (tests/golden/c5_traj.npz, make_golden.py c5): bit for bit.
    The fixture's K = 100 runs (and their 1-ulp-nudged twins) are what the GPU test compares the fused
    global-vector kernel with; this pins that the oracle is the same algorithm at that size too.  The dense
    613 MB-per-problem inverse Hessian makes this the slowest CPU test (~1 min at 8 threads)."""
    g = np.load(os.path.join(GOLDEN, "c5_traj.npz"))
    x0, obs, vis = torch.tensor(g["x0"]), torch.tensor(g["obs"]), torch.tensor(g["vis"])
    out = solver.bfgs_solve(x0, objective.ReprojectionClosure(obs, vis, 16, 4096), iterations=20,
                            error_threshold=-1.0, minimum_step=-1.0)
    assert np.array_equal(out.numpy(), g["k20"])


def test_c5_eight_problem_fixture_extends_the_pinned_one():
    """tests/golden/c5_traj8.npz (the real reference at K = 20 on the bench's first EIGHT C5 problems, with its
    1-ulp-nudged runs) starts with the two problems of c5_traj.npz, which the oracle reproduces bit for bit
    (test above): the same x0 rows and the same reference results there, so the eight-problem fixture comes
    from the same algorithm."""
    g2 = np.load(os.path.join(GOLDEN, "c5_traj.npz"))
    g8 = np.load(os.path.join(GOLDEN, "c5_traj8.npz"))
    assert g8["x0"].shape == (8, 12381) and g8["k20"].shape == (8, 12381)
    assert np.array_equal(g8["x0"][:2], g2["x0"])
    for key in ("k20", "k20_up", "k20_down"):
        assert np.array_equal(g8[key][:2], g2[key]), key
        assert np.isfinite(g8[key]).all()
