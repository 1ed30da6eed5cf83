"""The drop-in solver with arbitrary closures (generic path: closure in torch on the
GPU, every solver computation in the HIP building blocks), modelled on the
reference's own suites:
  tests/autograd_solvers/test_bfgs_solver.py                 (23 tests)
  tests/autograd_solvers/line_search/test_wolffe_conditions.py (22 tests)
The solver runs in eval mode (the reference's default drop-path makes its own
suite flaky).  Known-answer tests are kept verbatim in value.
"""
import math
import os
from unittest.mock import Mock

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


# ---- analytic test functions (same definitions as the reference's reference_functions.py) ----
def sphere(x, _=None):
    return x.square().sum(dim=-1)


def log_sphere(x, _=None):
    return (x.square().sum(dim=-1) + 1.0).log()


def rosenbrock(p, _=None):
    return (1.0 - p[..., 0]).square() + 100.0 * (p[..., 1] - p[..., 0].square()).square()


def cosine_error(x, _=None):
    norm = torch.linalg.vector_norm(x, dim=-1, keepdim=True)
    return (1.0 - (x / norm)[..., 0]) + (1.0 - norm[..., 0]).square()


def wavy(x, _=None):
    r = torch.linalg.vector_norm(x, dim=-1)
    return r.square() * (r.sin() + 2.0)


def bukin6(p, _=None):
    return 100.0 * (p[..., 1] - 0.01 * p[..., 0].square()).abs().sqrt() + 0.01 * (p[..., 0] + 10.0).abs()


def _solver(**kw):
    from deep_attention_visual_odometry_amd import BFGSSolver

    return BFGSSolver(**kw).eval()


# ---- BFGSSolver ----
def test_optimises_sphere(device):
    out = _solver(error_threshold=1e-6)(torch.tensor([1.1, 2.3], device=device), sphere)
    assert sphere(out).item() <= 1e-6


def test_optimises_offset_sphere(device):
    out = _solver(error_threshold=1e-6)(torch.tensor([1.1, 2.3], device=device), lambda x, m: sphere(x) + 10.0)
    assert sphere(out).item() <= 1e-6


def test_optimises_log_function_from_large_estimate_fp64(device):
    x0 = torch.tensor([-1700.3, 24942.8], dtype=torch.float64, device=device)
    out = _solver(error_threshold=1e-6)(x0, log_sphere)
    assert log_sphere(out).item() <= 1e-6


def test_optimises_cosine_function(device):
    out = _solver(error_threshold=1e-6)(torch.tensor([0.03, -18.8, 23.8, 19.0], device=device), cosine_error)
    assert cosine_error(out).item() <= 1e-6


def test_local_minima_behaviour(device):
    m1, m2 = -10.8060458497138, 14.5496166081312
    stuck = torch.tensor([[17.8885, 35.7771], [m1 * math.sqrt(2) / 2, m1 * math.sqrt(2) / 2],
                          [m2 * math.sqrt(2) / 2, -m2 * math.sqrt(2) / 2]], device=device)
    out = _solver(error_threshold=1e-6)(stuck, wavy)
    assert torch.isclose(out, stuck, rtol=0.2).all()
    m1, m2 = 10.8060458497138 + 2.25, 14.5496166081312 + 3.0
    free = torch.tensor([[m1 * math.sqrt(2) / 2, m1 * math.sqrt(2) / 2], [m2 * math.sqrt(2) / 2, -m2 * math.sqrt(2) / 2],
                         [-18.025, 6.0083]], device=device)
    out = _solver(error_threshold=1e-6)(free, wavy)
    assert torch.isclose(out, torch.zeros_like(out), atol=1e-3).all()


def test_few_iterations_still_improve(device):
    x0 = torch.tensor([27.7, -4.8], device=device)
    out = _solver(error_threshold=1e-6, iterations=3)(x0, cosine_error)
    assert cosine_error(out) < cosine_error(x0)
    assert cosine_error(out) > 1e-6


def test_batch_dimensions(device, fixed_random_seed):
    rng = np.random.default_rng(fixed_random_seed)
    x0 = torch.tensor(rng.normal(size=(3, 8, 4)), device=device)
    out = _solver(error_threshold=1e-6)(x0, log_sphere)
    assert out.shape == x0.shape
    assert (log_sphere(out) <= 1e-6).all()


def test_mask_contract(device, fixed_random_seed):
    """The closure sees a full-batch mask with mask.sum() == rows (bfgs_solver.py:99-104)."""
    rng = np.random.default_rng(fixed_random_seed)
    shifts = torch.tensor(rng.normal(0.0, 3.0, size=(3, 8, 2)), device=device)
    x0 = torch.tensor(rng.normal(size=(3, 8, 2)), device=device)
    seen_partial = []

    def fn(x, mask):
        assert mask.shape == (3, 8)
        assert int(mask.sum()) == x.size(0) and bool(mask.any())
        seen_partial.append(int(mask.sum()) < 24)
        x = x + shifts[mask]
        n1, n2 = int(mask[0].sum()), int(mask[1].sum())
        return torch.cat([bukin6(x[:n1]), rosenbrock(x[n1:n1 + n2]), sphere(x[n1 + n2:])])

    out = _solver(error_threshold=1e-6)(x0, fn)
    assert out.shape == x0.shape
    assert any(seen_partial)


def test_more_iterations_never_increase_error(device, fixed_random_seed):
    rng = np.random.default_rng(fixed_random_seed)
    x0 = torch.tensor(rng.normal(size=(5,)), device=device)
    prev = log_sphere(x0)
    for k in range(1, 15):
        e = log_sphere(_solver(error_threshold=1e-6, iterations=k)(x0, log_sphere))
        assert e <= prev
        prev = e


@pytest.mark.parametrize("fn,minimum,tol", [(sphere, (0.0, 0.0), 1e-6), (log_sphere, (0.0, 0.0), 1e-4),
                                            (rosenbrock, (1.0, 1.0), 0.02)])
def test_reference_functions(device, fixed_random_seed, fn, minimum, tol):
    rng = np.random.default_rng(fixed_random_seed)
    m = torch.tensor(minimum, dtype=torch.float64, device=device)
    x0 = torch.tensor(rng.normal(0.0, max(float(m.abs().max()), 1.0), size=(16, 2)), device=device)
    out = _solver(iterations=2000, error_threshold=1e-8)(x0, fn)
    assert torch.isclose(out, m.expand_as(out), atol=tol).all()


def test_plane_fit(device, fixed_random_seed):
    rng = np.random.default_rng(fixed_random_seed)
    plane = rng.normal(size=(4,))
    plane = plane / np.linalg.norm(plane[:3])
    pts = rng.normal(0.0, 15.0, size=(128, 3))
    origin = -plane[3] * plane[:3]
    pts = pts - origin
    pts = pts - (pts @ plane[:3])[:, None] * plane[None, :3] + origin + rng.normal(0.0, 0.01, size=(128, 3))
    p = torch.tensor(pts.reshape(1, 128, 3), device=device)

    def fn(x, _):
        return ((x[..., 0:3].unsqueeze(-2) * p).sum(-1) + x[..., 3:4]).square().sum(-1)

    out = _solver(error_threshold=1e-10, minimum_step=1e-8, iterations=500)(
        torch.tensor(rng.normal(size=(4,)), device=device), fn)
    out = (out / torch.linalg.vector_norm(out[0:3])).cpu()
    ref = torch.tensor(plane)
    assert torch.isclose(out, ref, atol=0.1).all() or torch.isclose(-out, ref, atol=0.1).all()


def test_output_does_not_require_grad_and_no_grad_block(device):
    x0 = torch.tensor([1.1, 2.3], device=device)
    assert _solver(error_threshold=1e-6)(x0, sphere).requires_grad is False
    with torch.no_grad():
        out = _solver(error_threshold=1e-6)(x0, sphere)
    assert sphere(out).item() <= 1e-6


def test_update_kat_textbook(device):
    """tests/autograd_solvers/test_bfgs_solver.py:307-332 known answer."""
    from deep_attention_visual_odometry_amd import BFGSSolver

    s = torch.tensor([-1.26262069, -0.78272035, 0.98543104], dtype=torch.float64)
    y = torch.tensor([0.15339519, -0.28944666, 0.54194925], dtype=torch.float64)
    h = torch.tensor([[2.0, 1.0, 0.0], [1.0, 1.0, 0.0], [0.0, 0.0, 3.0]], dtype=torch.float64)
    c = (s * y).sum()
    expected = ((torch.eye(3, dtype=torch.float64) - s[:, None] * y[None, :] / c) @ h
                @ (torch.eye(3, dtype=torch.float64) - y[:, None] * s[None, :] / c) + s[:, None] * s[None, :] / c)
    out = BFGSSolver.update_inverse_hessian(h.to(device), s.to(device), y.to(device)).cpu()
    assert torch.isclose(expected, out).all()


@pytest.mark.parametrize("y", [[0.0, 0.0, -3.0], [0.0, -1.0, -3.0]])
def test_update_skipped_for_nonpositive_curvature(device, y):
    """tests/autograd_solvers/test_bfgs_solver.py:335-361: exactly the input."""
    from deep_attention_visual_odometry_amd import BFGSSolver

    h = torch.tensor([[2.0, -1.0, 0.0], [-1.0, 2.0, -1.0], [0.0, -1.0, 2.0]], dtype=torch.float64, device=device)
    out = BFGSSolver.update_inverse_hessian(h, torch.tensor([1.0, 2.0, 0.0], dtype=torch.float64, device=device),
                                            torch.tensor(y, dtype=torch.float64, device=device))
    assert torch.equal(out, h)


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("p", [3, 17, 64])
def test_update_and_scale_match_reference_golden(device, dt, p):
    from deep_attention_visual_odometry_amd import BFGSSolver

    g = np.load(os.path.join(GOLDEN, "bfgs_update.npz"))
    key = f"{dt}_p{p}"
    h, s, y = (torch.tensor(g[key + k]).to(device) for k in ("_h", "_s", "_y"))
    out = BFGSSolver.update_inverse_hessian(h, s, y).cpu()
    ref = torch.tensor(g[key + "_out"])
    tol = 1e-12 if dt == "f64" else 2e-5
    assert ((out - ref).norm(dim=(-1, -2)) / ref.norm(dim=(-1, -2))).max() <= tol
    assert torch.equal(out[1], torch.tensor(g[key + "_h"])[1])  # negative curvature: exact skip
    sc = BFGSSolver.scale_initial_inverse_hessian(s, y).cpu()
    assert torch.allclose(sc, torch.tensor(g[key + "_scale"]), rtol=1e-5 if dt == "f32" else 1e-12)


# ---- line_search_wolfe_conditions ----
@pytest.fixture(params=[False, True])
def strong(request):
    return request.param


def _ls(*a, **k):
    from deep_attention_visual_odometry_amd import line_search_wolfe_conditions

    return line_search_wolfe_conditions(*a, **k)


def _base(fn, x):
    x = x.clone().requires_grad_(True)
    e = fn(x, None)
    (g,) = torch.autograd.grad(e.sum(), x)
    return e.detach(), g


def test_ls_reduces_error(device, strong):
    target = torch.tensor([1.8, 1.2], device=device)
    x = torch.tensor([2.0, -3.0], device=device)
    d = torch.tensor([0.2, 1.0], device=device)
    fn = lambda v, _: torch.linalg.vector_norm(v - target, dim=-1)  # noqa: E731
    e, g = _base(fn, x)
    a = _ls(x, d, e, g, fn, strong=strong)
    assert a.shape == torch.Size([]) and a > 0
    assert fn(x + a * d, None) < e


def test_ls_batch_dimensions(device, strong):
    t = torch.tensor([[[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]], [[4.3, -10], [-9.7, 2.2], [2.8, -8.2]]], device=device)
    x = torch.zeros_like(t)
    d = torch.tensor([[[0.1, 1.0], [10.0, -0.1], [0.1, 0.1]], [[1.0, -1.0], [-1.0, -0.1], [2.0, 0.1]]], device=device)

    def fn(v, mask=None):
        tt = t[mask] if mask is not None else t
        return (torch.linalg.vector_norm(v - tt, dim=-1) - 0.5).square()

    e, g = _base(fn, x)
    a = _ls(x, d, e, g, fn, strong=strong)
    assert a.shape == (2, 3) and (a > 0).all()
    assert (fn(x + a.unsqueeze(-1) * d) <= e).all()


def _skewed_problem(device, seed):
    rng = np.random.default_rng(seed)
    t = torch.tensor(rng.normal(0.0, 2.0, size=(3, 4, 2)), device=device)
    x = torch.tensor(rng.normal(size=(3, 4, 2)), device=device)
    skew = torch.tensor(rng.uniform(-0.2, 0.2, size=(3, 4, 1)), device=device)

    def fn(v, mask=None):
        tt = t[mask] if mask is not None else t
        return ((torch.linalg.vector_norm(v - tt, dim=-1) - 0.5).square() + 1.0).log()

    e, g = _base(fn, x)
    d = torch.cat([-skew.cos() * g[..., 0:1] + skew.sin() * g[..., 1:2],
                   -skew.sin() * g[..., 0:1] - skew.cos() * g[..., 1:2]], dim=-1)
    return x, d, e, g, fn


def test_ls_trial_points_lie_on_the_ray(device, strong, fixed_random_seed):
    x, d, e, g, fn = _skewed_problem(device, fixed_random_seed)
    mock = Mock(spec_set=["__call__"], side_effect=fn)
    _ls(x, d, e, g, mock, strong=strong)
    assert mock.called
    for call in mock.call_args_list:
        mask = call.args[1]
        ratio = (call.args[0] - x[mask]) / d[mask]
        assert torch.isclose(ratio[..., 0], ratio[..., 1]).all()


def test_ls_result_satisfies_wolfe_conditions(device, strong, fixed_random_seed):
    x, d, e, g, fn = _skewed_problem(device, fixed_random_seed)
    c1, c2 = 0.1, 0.6
    a = _ls(x, d, e, g, fn, sufficient_decrease=c1, curvature=c2, strong=strong)
    slope0 = (d * g).sum(-1)
    xr = (x + a.unsqueeze(-1) * d).requires_grad_(True)
    er = fn(xr)
    (gr,) = torch.autograd.grad(er.sum(), xr)
    slope = (d * gr).sum(-1)
    assert (er <= e + c1 * a * slope0).all()
    if strong:
        assert (slope.abs() <= c2 * slope0.abs()).all()
    else:
        assert (-slope <= -c2 * slope0).all()


def test_ls_shrinks_and_widens(device):
    fn = lambda v, _: torch.linalg.vector_norm(v - torch.tensor([1.0, 1.0], device=device), dim=-1)  # noqa: E731
    x = torch.zeros(2, device=device)
    e, g = _base(fn, x)
    assert _ls(x, torch.tensor([10.0, 0.0], device=device), e, g, fn, strong=True) < 1.0
    fn2 = lambda v, _: torch.linalg.vector_norm(v - torch.tensor([10.0, 10.0], device=device), dim=-1)  # noqa: E731
    e, g = _base(fn2, x)
    assert _ls(x, torch.tensor([0.2, 0.1], device=device), e, g, fn2, strong=True) > 1.0


def test_ls_known_answer_quarter(device, strong):
    """tests/autograd_solvers/line_search/test_wolffe_conditions.py:260-280: alpha == 0.25 exactly."""
    fn = lambda v, _: torch.linalg.vector_norm(v - torch.tensor([0.25, 0.25], device=device), dim=-1)  # noqa: E731
    x = torch.zeros(2, device=device)
    e, g = _base(fn, x)
    assert _ls(x, torch.tensor([1.0, 1.0], device=device), e, g, fn, strong=strong).item() == 0.25


def test_ls_wrong_direction_gives_no_step(device, strong):
    fn = lambda v, _: torch.linalg.vector_norm(v - torch.tensor([-9.7, 2.2], device=device), dim=-1)  # noqa: E731
    x = torch.zeros(2, device=device)
    e, g = _base(fn, x)
    a = _ls(x, torch.tensor([1.0, 0.0], device=device), e, g, fn, strong=strong)
    assert torch.isclose(a, torch.zeros_like(a))


def test_ls_moves_out_of_local_minimum(device, strong):
    x = torch.tensor([-13.9922246512961], device=device)
    e, g = _base(wavy, x)
    assert _ls(x, -g, e, g, wavy, strong=strong) > 0.01


def test_ls_does_not_propagate_gradients(device, strong):
    target = torch.tensor([0.25, 0.25], device=device, requires_grad=True)
    fn = lambda v, _: torch.linalg.vector_norm(v - target, dim=-1)  # noqa: E731
    x = torch.zeros(2, device=device)
    e, g = _base(fn, x)
    assert not _ls(x, torch.tensor([1.0, -0.1], device=device, requires_grad=True), e, g, fn,
                   strong=strong).requires_grad


def test_ls_warns_on_bad_constants(device):
    fn = lambda v, _: sphere(v)  # noqa: E731
    x = torch.ones(2, device=device)
    e, g = _base(fn, x)
    with pytest.warns(UserWarning):
        _ls(x, -g, e, g, fn, sufficient_decrease=0.5, curvature=0.4)


@pytest.mark.parametrize("shape", ["c1", "c2", "c3"])
@pytest.mark.parametrize("strong", [True, False])
def test_ls_reference_golden_alphas(device, shape, strong):
    """Golden alphas of the REAL reference on the BA objective (tests/golden/line_search.npz),
    with the HIP objective as the closure."""
    from deep_attention_visual_odometry_amd import ReprojectionError

    g = np.load(os.path.join(GOLDEN, "line_search.npz"))
    m, n = {"c1": (2, 64), "c2": (2, 128), "c3": (4, 256)}[shape]
    key = f"{shape}_f32"
    fn = ReprojectionError(torch.tensor(g[key + "_obs"]).to(device), torch.tensor(g[key + "_vis"]).to(device), m, n)
    a = _ls(torch.tensor(g[key + "_x"]).to(device), torch.tensor(g[key + "_dir"]).to(device),
            torch.tensor(g[key + "_err"]).to(device), torch.tensor(g[key + "_grad"]).to(device), fn, strong=strong)
    ref = torch.tensor(g[f"{key}_{'strong' if strong else 'weak'}_alpha"])
    a = a.cpu()
    assert torch.equal(a[[0, 1, 3]], ref[[0, 1, 3]]), (a, ref)
    # uphill direction: the bisection stops where rounding noise in E decides, ~0 in both
    # (the reference's own test_produces_small_change_when_search_direction_is_wrong uses isclose(., 0))
    assert torch.isclose(a[2], torch.zeros(())) and torch.isclose(ref[2], torch.zeros(()))


def test_generic_path_with_native_objective_matches_fused(device):
    """Same BA problem through the generic path (closure = HIP objective, HIP update kernels,
    Python loop) and through the fused kernel: equal to the parity bar."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, make_scenes

    s = make_scenes(3, 2, 64, seed=31)
    x0 = torch.tensor(s.initial).to(device)
    fn = ReprojectionError(torch.tensor(s.observations).to(device), torch.tensor(s.visibility).to(device), 2, 64)
    fused = BFGSSolver(iterations=20, error_threshold=-1.0, minimum_step=-1.0).eval()(x0, fn)
    generic = BFGSSolver(iterations=20, error_threshold=-1.0, minimum_step=-1.0).eval()._generic(x0, fn, -1.0, 20)
    rel = (fused - generic).double().norm(dim=-1) / generic.double().norm(dim=-1)
    assert rel.max().item() <= 1e-5


# ---- training-mode semantics (bfgs_solver.py:88-93, :121-125, :196-212) ----

TRAINING = {
    "rosen_drop": (dict(drop_path_p=0.3, training_iterations=30, training_error_threshold=1e-3), 9101),
    "rosen_second_last": (dict(drop_path_p=0.0, return_second_last=True, training_iterations=40,
                               training_error_threshold=1e-6), 9102),
    "rosen_both": (dict(drop_path_p=0.2, return_second_last=True, training_iterations=25), 9103),
}


@pytest.mark.parametrize("case", list(TRAINING))
def test_training_mode_matches_reference(device, case):
    """The module's default training mode against the REAL reference (tests/golden/training.npz),
    drop-path draws made deterministic by the same stand-in for torch.rand_like (fp64)."""
    from deep_attention_visual_odometry_amd import BFGSSolver
    from rng_patch import deterministic_rand_like

    g = np.load(os.path.join(GOLDEN, "training.npz"))
    kw, seed = TRAINING[case]
    solver = BFGSSolver(**kw)
    assert solver.training
    with deterministic_rand_like(seed):
        out = solver(torch.tensor(g["rosen_x0"], device=device), rosenbrock).cpu()
    ref = torch.tensor(g[case])
    assert ((out - ref).norm(dim=-1) / ref.norm(dim=-1)).max().item() < 1e-7  # fp64, reduction order only


def test_training_mode_ba_drop_path_matches_reference(device):
    from deep_attention_visual_odometry_amd import BFGSSolver
    from oracle import objective

    from rng_patch import deterministic_rand_like

    g = np.load(os.path.join(GOLDEN, "training.npz"))
    obs, vis = torch.tensor(g["ba_obs"], device=device), torch.tensor(g["ba_vis"], device=device)
    fn = objective.ReprojectionClosure(obs, vis, 2, 64)
    solver = BFGSSolver(drop_path_p=0.25, training_iterations=12, training_error_threshold=-1.0, minimum_step=-1.0)
    with deterministic_rand_like(9201):
        out = solver(torch.tensor(g["ba_x0"], device=device), fn).cpu()
    ref = torch.tensor(g["ba_drop"])
    assert ((out - ref).norm(dim=-1) / ref.norm(dim=-1)).max().item() < 1e-5


def test_training_mode_uses_training_threshold_and_iterations(device):
    from deep_attention_visual_odometry_amd import BFGSSolver

    x0 = torch.tensor([[1.5, -2.0]], device=device)
    solver = BFGSSolver(iterations=500, error_threshold=1e-12, training_iterations=3,
                        training_error_threshold=1e-12, drop_path_p=0.0)
    trained = solver(x0, rosenbrock)
    evald = solver.eval()(x0, rosenbrock)
    assert rosenbrock(evald).item() < rosenbrock(trained).item()


# ---- the generic loop's compact history (r06: dava_bfgs_compact_direction, no (B, P, P) matrix) ----

def _dense_reference_directions(g_seq, y_seq, s_seq):
    """d_k from the dense building blocks exactly as the reference's loop forms them (bfgs_solver.py:157-176):
    H_0 = I scaled by gamma at k = 1, then the rank-2 update and d = -H g, for k = 1 .. len."""
    from deep_attention_visual_odometry_amd import native_ops

    b, n = g_seq[0].shape
    h = torch.eye(n, dtype=g_seq[0].dtype, device=g_seq[0].device).expand(b, n, n).contiguous()
    out = []
    for k, (g, y, s) in enumerate(zip(g_seq, y_seq, s_seq)):
        if k == 0:
            h = native_ops.scale_matrix(native_ops.initial_scale(s, y), h)
        h = native_ops.update_inverse_hessian(h, s, y)
        out.append(native_ops.search_direction(h, g))
    return out


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-10), (torch.float32, 1e-5)])
def test_compact_direction_matches_the_dense_update(device, dtype, tol, fixed_random_seed):
    """The op's d after k updates equals the dense matrix's d (same rank-2 terms, product form): 6 problems,
    n = 37, 12 iterations, one update with s.y <= 0 (skipped by rho = 0 in both forms)."""
    from deep_attention_visual_odometry_amd import native_ops

    b, n, iters = 6, 37, 12
    a = torch.randn(b, n, n, dtype=torch.float64)
    spd = (a @ a.transpose(1, 2) / n + torch.eye(n, dtype=torch.float64)).to(dtype).to(device)
    g_seq, y_seq, s_seq = [], [], []
    for k in range(iters):
        s = torch.randn(b, n, dtype=dtype, device=device)
        y = torch.einsum("bij,bj->bi", spd, s)
        if k == 5:
            y[2] = -y[2]  # negative curvature for problem 2 at this step
        g_seq.append(torch.randn(b, n, dtype=dtype, device=device))
        y_seq.append(y)
        s_seq.append(s)
    want = _dense_reference_directions(g_seq, y_seq, s_seq)
    hist = native_ops.CompactHistory(b, n, dtype, device, max_entries=iters, capacity=2)  # grows 2 -> 4 -> 8 -> 12
    idx = torch.arange(b, device=device)
    for k in range(iters):
        d = hist.direction(g_seq[k], y_seq[k], s_seq[k], idx)
        rel = ((d - want[k]).norm(dim=-1) / want[k].norm(dim=-1)).max().item()
        assert rel <= tol, (k, rel)
    assert hist.count == iters and hist.capacity == iters
    assert hist.rho[2, 5].item() == 0.0 and bool((hist.rho[:, :iters] != 0).sum() == b * iters - 1)


def test_compact_direction_touches_only_the_active_problems(device, fixed_random_seed):
    """Rows of problems outside problem_index keep their history bit for bit (the mask contract: a stopped
    problem's inverse Hessian is never updated, bfgs_solver.py:178-180)."""
    from deep_attention_visual_odometry_amd import native_ops

    b, n = 5, 20
    hist = native_ops.CompactHistory(b, n, torch.float32, device, max_entries=4)
    all_idx = torch.arange(b, device=device)
    r = lambda m: torch.randn(m, n, device=device)  # noqa: E731
    hist.direction(r(b), r(b).abs(), r(b).abs(), all_idx)
    before = [t.clone() for t in (hist.s, hist.w, hist.rho, hist.c, hist.gamma)]
    active = torch.tensor([0, 3], device=device)
    hist.direction(r(2), r(2).abs(), r(2).abs(), active)
    for t0, t1 in zip(before, (hist.s, hist.w, hist.rho, hist.c, hist.gamma)):
        for i in (1, 2, 4):
            assert torch.equal(t0[i], t1[i])
    assert not torch.equal(before[0][0], hist.s[0])


@pytest.mark.parametrize("fn,x0", [(rosenbrock, [[1.5, -2.0], [-1.2, 1.0], [0.3, 0.4]]),
                                   (wavy, [[0.7, -0.2, 1.1], [2.0, 0.1, -0.5], [-0.3, 0.9, 0.2]])])
def test_generic_loop_compact_matches_dense(device, fn, x0):
    """The whole generic loop (reference stopping rules, masks) with the compact history vs the dense matrix
    (the GENERIC_DENSE override), fp64: the same iterates to reordering."""
    from deep_attention_visual_odometry_amd import _native

    x = torch.tensor(x0, dtype=torch.float64, device=device)
    compact = _solver(iterations=200, error_threshold=1e-12, minimum_step=1e-12)
    out_c = compact(x, fn)
    assert compact.last_generic_history is not None
    with _native.debug_overrides(GENERIC_DENSE=1):
        dense = _solver(iterations=200, error_threshold=1e-12, minimum_step=1e-12)
        out_d = dense(x, fn)
        assert dense.last_generic_history is None
    assert torch.allclose(out_c, out_d, rtol=1e-8, atol=1e-10), (out_c, out_d)


def test_calibration_network_closure_through_the_generic_loop(device):
    """The reference caller's own closure (CalibrationNetwork's ray-angle error in torch) through the drop-in:
    the compact generic loop against the oracle solve of the oracle's ray-angle closure (fp64, K = 10), and the
    fp32 solve against the fused RayAngleError solve of the same problems."""
    from deep_attention_visual_odometry_amd import BFGSSolver, RayAngleError, make_scenes
    from deep_attention_visual_odometry_amd.geometry import calibration_network_error
    from oracle import objective, solver

    s = make_scenes(6, 2, 32, distortion=False, seed=77, ray_angle=True)
    obs, vis, x0 = (torch.tensor(a) for a in (s.observations, s.visibility, s.initial))
    kw = dict(iterations=10, error_threshold=-1.0, minimum_step=-1.0)
    fn64 = calibration_network_error(obs.double().to(device), vis.double().to(device), 2, 32)
    m = BFGSSolver(**kw).eval()
    out = m(x0.double().to(device), fn64).cpu()
    assert m.last_generic_history is not None
    ref = solver.bfgs_solve(x0.double(), objective.RayAngleClosure(obs.double(), vis, 2, 32), **kw)
    assert ((out - ref).norm(dim=-1) / ref.norm(dim=-1)).max().item() <= 1e-9
    fn32 = calibration_network_error(obs.to(device), vis.float().to(device), 2, 32)
    out32 = BFGSSolver(**kw).eval()(x0.to(device), fn32)
    fused = BFGSSolver(**kw).eval()(x0.to(device), RayAngleError(obs.to(device), vis.to(device), 2, 32))
    assert ((out32 - fused).double().norm(dim=-1) / fused.double().norm(dim=-1)).max().item() <= 1e-4


def test_compact_generic_loop_memory_is_o_kp(device):
    """C3's shape (P = 789) at B = 64, K = 30 through a closure: the compact rows grow with the iterations run
    (O(k P) per problem), never to the dense (B, P, P) matrix (160 MB here)."""
    from deep_attention_visual_odometry_amd import ReprojectionError, make_scenes

    s = make_scenes(64, 4, 256, distortion=False, seed=3)
    fn = ReprojectionError(torch.tensor(s.observations).to(device), torch.tensor(s.visibility).to(device), 4, 256)
    x0 = torch.tensor(s.initial).to(device)
    m = _solver(iterations=30, error_threshold=-1.0, minimum_step=-1.0)
    m._generic(x0, fn, -1.0, 30)
    hist = m.last_generic_history
    assert hist is not None and hist.count == 29 and hist.capacity == 29
    dense = 64 * 789 * 789 * 4
    assert hist.nbytes() < dense / 6
