"""BASELINE configuration C1 as BASELINE states it: "BFGS on PyTorch CPU -- plumbing, runs without a GPU".

`BFGSSolver` on CPU tensors with an ordinary torch closure runs the generic loop (bfgs_solver.py:118-212)
on the library's HOST flavours of its building blocks (csrc/bfgs_host.hip, dava_cpu_*), dispatched by
the tensors' device.  Checked against the REAL reference's outputs (tests/golden/bfgs_traj.npz: C1,
BFGSSolver(...).eval() after K = 5, 20, 100, and the c1def run with the reference's default stopping
rules in float64), and the building blocks op by op against the reference's own goldens
(tests/golden/bfgs_update.npz).  The closure is the caller's own code, written here in torch (the BA
objective of SURVEY 8(a): unpack -> scale-normalised camera-relative points -> Rodrigues -> pinhole ->
squared residual weighted by visibility); the oracle only supplies the 1-ulp envelopes at K = 100.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import objective, solver

TOL = 1e-5


def _closure(obs, vis, m, n):
    """The caller's error_function(parameters, batch_mask) in plain torch."""
    from deep_attention_visual_odometry_amd import unpack_calibration_parameters

    def error(x, mask):
        parts = unpack_calibration_parameters(x, m, n)
        pts, t, w = parts.world_points, parts.camera_translations, parts.camera_rotations
        scale = (pts.abs().mean(dim=(-1, -2, -3), keepdim=True) * n
                 + t.abs().mean(dim=(-1, -2, -3), keepdim=True) * m) / (n + m)
        pts, t = pts / scale, t / scale
        theta = torch.linalg.vector_norm(w, dim=-1, keepdim=True)
        vw = (pts * w).sum(dim=-1, keepdim=True)
        moved = (pts * torch.cos(theta) + (1.0 - torch.cos(theta)) / theta.square() * vw * w
                 + torch.linalg.cross(w.expand_as(pts), pts, dim=-1) * (torch.sin(theta) / theta) + t)
        p = torch.cat([pts, moved], dim=-3)
        k = parts.intrinsics
        uv = k[..., 0:1] * p[..., 0:2] / p[..., 2:3] + k[..., 1:3]
        sq = (uv - obs[mask]).square().sum(dim=-1)
        return (sq * vis[mask].to(sq.dtype)).sum(dim=(-1, -2))

    return error


def _rel(a, b):
    a, b = a.double(), b.double()
    return (a - b).norm(dim=-1) / b.norm(dim=-1)


def test_cpu_solve_matches_reference_c1_trajectories():
    from oracle import objective, solver

    from deep_attention_visual_odometry_amd import BFGSSolver

    g = np.load(os.path.join(GOLDEN, "bfgs_traj.npz"))
    x0 = torch.tensor(g["c1_x0"])
    obs, vis = torch.tensor(g["c1_obs"]), torch.tensor(g["c1_vis"])
    fn = _closure(obs, vis, 2, 64)
    for k in (5, 20, 100):
        out = BFGSSolver(iterations=k, error_threshold=-1.0, minimum_step=-1.0).eval()(x0, fn)
        assert out.device.type == "cpu" and out.dtype == torch.float32
        ref = torch.tensor(g[f"c1_k{k}"])
        rel = _rel(out, ref)
        if k < 100:
            assert (rel <= TOL).all(), (k, rel)
            continue
        # K = 100: each problem inside max(1e-5, 5x the reference's own change under a 1-ulp nudge of x0)
        oc = objective.ReprojectionClosure(obs, vis, 2, 64)
        env = torch.full((x0.shape[0],), TOL, dtype=torch.float64)
        for to in (float("inf"), -float("inf")):
            nudged = solver.bfgs_solve(torch.nextafter(x0, torch.full_like(x0, to)), oc, iterations=k,
                                       error_threshold=-1.0, minimum_step=-1.0)
            env = torch.maximum(env, 5.0 * _rel(nudged, ref))
        assert (rel <= env).all() and (rel <= TOL).all(), (rel, env)


def test_cpu_solve_reference_defaults_float64():
    """BFGSSolver() with every default, float64, the reference's own run to its stopping rules."""
    from deep_attention_visual_odometry_amd import BFGSSolver

    g = np.load(os.path.join(GOLDEN, "bfgs_traj.npz"))
    x0, obs, vis = torch.tensor(g["c1def_x0"]), torch.tensor(g["c1def_obs"]), torch.tensor(g["c1def_vis"])
    out = BFGSSolver().eval()(x0, _closure(obs, vis, 2, 64))
    assert out.dtype == torch.float64
    assert _rel(out, torch.tensor(g["c1def_out"])).max() <= 1e-9


def test_cpu_building_blocks_match_reference_goldens():
    """update_inverse_hessian / scale_initial_inverse_hessian (the static methods, bfgs_solver.py:217-303)
    on CPU tensors against the reference's outputs (tests/golden/bfgs_update.npz), fp64 and fp32."""
    from deep_attention_visual_odometry_amd import BFGSSolver

    g = np.load(os.path.join(GOLDEN, "bfgs_update.npz"))
    cases = sorted({k[: -len("_h")] for k in g.keys() if k.endswith("_h")})
    assert cases
    for c in cases:
        h, s, y = (torch.tensor(g[f"{c}_{k}"]) for k in ("h", "s", "y"))
        got = BFGSSolver.update_inverse_hessian(h, s, y)
        want = torch.tensor(g[f"{c}_out"])
        tol = 1e-12 if h.dtype == torch.float64 else 2e-6
        assert torch.allclose(got, want, rtol=tol, atol=tol * want.abs().max().item()), c
        if f"{c}_scale" in g:
            sc = BFGSSolver.scale_initial_inverse_hessian(s, y)
            assert torch.allclose(sc.reshape(-1), torch.tensor(g[f"{c}_scale"]).reshape(-1), rtol=tol), c


def test_cpu_gradient_through_the_solve():
    """create_graph mode on CPU (bfgs_solver.py:85, :134, :213-215): the CPU building blocks' VJPs
    (dava_cpu_*_backward) against torch's own autograd of the same algebra, through a 6-step solve."""
    from deep_attention_visual_odometry_amd import BFGSSolver
    from deep_attention_visual_odometry_amd import native_ops

    gen = torch.Generator().manual_seed(3)
    n = 7
    a = torch.randn(4, n, n, dtype=torch.float64, generator=gen)
    spd = a @ a.transpose(-1, -2) + n * torch.eye(n, dtype=torch.float64)

    def quad(x, mask):  # a batch of convex quadratics with a quartic term
        xs = x.unsqueeze(-1)
        return 0.5 * (xs.transpose(-1, -2) @ spd[mask] @ xs).reshape(-1) + 0.1 * x.pow(4).sum(-1)

    x0 = torch.randn(4, n, dtype=torch.float64, generator=gen).requires_grad_(True)
    out = BFGSSolver(iterations=6, error_threshold=-1.0, minimum_step=-1.0).eval()(x0, quad)
    (gx,) = torch.autograd.grad(out.square().sum(), x0)
    assert torch.isfinite(gx).all() and gx.abs().max() > 0
    # the VJPs themselves, against autograd of the same formulas
    h = spd.clone().requires_grad_(True)
    s = torch.randn(4, n, dtype=torch.float64, generator=gen).requires_grad_(True)
    y = (spd @ s.detach().unsqueeze(-1)).squeeze(-1).requires_grad_(True)
    w = torch.randn(4, n, n, dtype=torch.float64, generator=gen)
    got = torch.autograd.grad((native_ops.update_inverse_hessian(h, s, y) * w).sum(), (h, s, y))
    sy = (s * y).sum(-1, keepdim=True)
    rho = 1.0 / sy
    yH = (y.unsqueeze(-2) @ h).squeeze(-2)
    Hy = (h @ y.unsqueeze(-1)).squeeze(-1)
    c = 1.0 + (yH * y * rho).sum(-1, keepdim=True)
    sr = s * rho
    ref_out = h + (sr.unsqueeze(-1) * s.unsqueeze(-2)) * c.unsqueeze(-1) - sr.unsqueeze(-1) * yH.unsqueeze(-2) \
        - Hy.unsqueeze(-1) * sr.unsqueeze(-2)
    want = torch.autograd.grad((ref_out * w).sum(), (h, s, y))
    for a_, b_ in zip(got, want):
        assert torch.allclose(a_, b_, rtol=1e-10, atol=1e-10)


def _cpu_scene(b, m, n, distortion, ray=False, seed=5):
    from deep_attention_visual_odometry_amd import make_scenes

    s = make_scenes(b, m, n, distortion=distortion, seed=seed, ray_angle=ray)
    return torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)


@pytest.mark.parametrize("case", ["pinhole", "brown_conrady", "ray_angle"])
def test_cpu_fused_objectives_match_the_oracle(case):
    """ReprojectionError / RayAngleError on CPU tensors: the objective's torch form (geometry.closure_ops) --
    E and its autograd gradient against the oracle's at the same points, float32 and float64."""
    from deep_attention_visual_odometry_amd import RayAngleError, ReprojectionError

    m, n = (4, 32) if case == "brown_conrady" else (2, 32)
    x0, obs, vis = _cpu_scene(3, m, n, case == "brown_conrady", case == "ray_angle")
    for dtype in (torch.float32, torch.float64):
        x = x0.to(dtype).requires_grad_(True)
        xr = x0.to(dtype).requires_grad_(True)
        if case == "ray_angle":
            fn, ref_fn = RayAngleError(obs.to(dtype), vis, m, n), objective.RayAngleClosure(obs.to(dtype), vis, m, n)
        else:
            d = case == "brown_conrady"
            fn = ReprojectionError(obs.to(dtype), vis, m, n, d)
            ref_fn = objective.ReprojectionClosure(obs.to(dtype), vis, m, n, d)
        mask = torch.ones(3, dtype=torch.bool)
        e, e_ref = fn(x, mask), ref_fn(xr, mask)
        (g,), (g_ref,) = torch.autograd.grad(e.sum(), x), torch.autograd.grad(e_ref.sum(), xr)
        tol = 1e-6 if dtype == torch.float32 else 1e-13
        assert torch.allclose(e, e_ref, rtol=tol, atol=0), (case, dtype)
        assert ((g - g_ref).norm(dim=-1) / g_ref.norm(dim=-1)).max() <= 10 * tol, (case, dtype)


@pytest.mark.parametrize("case", ["pinhole", "brown_conrady", "ray_angle"])
def test_cpu_fused_objectives_solve_where_the_parameters_live(case):
    """BFGSSolver with a fused objective on CPU tensors (the reference solves wherever the parameters live,
    bfgs_solver.py:94-117): the generic loop on the library's host flavours, against the oracle's solve of the
    same problems at K = 20, per problem <= 1e-5."""
    from deep_attention_visual_odometry_amd import BFGSSolver, RayAngleError, ReprojectionError

    m, n = (4, 32) if case == "brown_conrady" else (2, 32)
    x0, obs, vis = _cpu_scene(4, m, n, case == "brown_conrady", case == "ray_angle", seed=6)
    if case == "ray_angle":
        fn, ref_fn = RayAngleError(obs, vis, m, n), objective.RayAngleClosure(obs, vis, m, n)
    else:
        d = case == "brown_conrady"
        fn, ref_fn = ReprojectionError(obs, vis, m, n, d), objective.ReprojectionClosure(obs, vis, m, n, d)
    kw = dict(iterations=20, error_threshold=-1.0, minimum_step=-1.0)
    out = BFGSSolver(**kw).eval()(x0, fn)
    ref = solver.bfgs_solve(x0, ref_fn, **kw)
    rel = (out.double() - ref.double()).norm(dim=-1) / ref.double().norm(dim=-1)
    assert out.device.type == "cpu" and (rel <= 1e-5).all(), rel


def test_cpu_fused_objective_gradient_through_the_solve():
    """create_graph on CPU tensors with a fused objective: d(sum w x_K)/dx0 through 3 iterations against the
    oracle's autograd of the same solve (float64)."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    x0, obs, vis = _cpu_scene(2, 2, 16, False, seed=8)
    x0, obs = x0.double(), obs.double()
    w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    kw = dict(iterations=3, error_threshold=-1.0, minimum_step=-1.0)
    xa = x0.clone().requires_grad_(True)
    (ga,) = torch.autograd.grad((BFGSSolver(**kw).eval()(xa, ReprojectionError(obs, vis, 2, 16)) * w).sum(), xa)
    xb = x0.clone().requires_grad_(True)
    (gb,) = torch.autograd.grad((solver.bfgs_solve(xb, objective.ReprojectionClosure(obs, vis, 2, 16), **kw) * w).sum(),
                                xb)
    assert torch.allclose(ga, gb, rtol=1e-8, atol=1e-10)


def _gradcheck(fn, *inputs):
    return torch.autograd.gradcheck(fn, inputs, eps=1e-6, atol=1e-7, rtol=1e-6)


def test_cpu_building_block_vjps_gradcheck():
    """The host VJPs (dava_cpu_*_backward, csrc/bfgs_host.hip) against finite differences in float64, for
    every building block the generic loop differentiates, including the branches where the reference's
    clamps bind (scale_initial_inverse_hessian, bfgs_solver.py:217-233: y.y < 1e-5, ratio < 1e-4) and the
    skipped update (InverseCurvature, utils/func_inverse_curvature.py:21-51: s.y <= 0 gives rho = 0, whose
    custom backward -rho^2 g is then 0 too)."""
    from deep_attention_visual_odometry_amd import native_ops

    gen = torch.Generator().manual_seed(11)
    n = 6

    def r(*shape, scale=1.0):
        return (torch.randn(*shape, dtype=torch.float64, generator=gen) * scale).requires_grad_(True)

    a = torch.randn(3, n, n, dtype=torch.float64, generator=gen)
    h = (a @ a.transpose(-1, -2) / n + torch.eye(n, dtype=torch.float64)).requires_grad_(True)
    s = r(3, n)
    y = (s.detach() + 0.3 * torch.randn(3, n, dtype=torch.float64, generator=gen)).requires_grad_(True)
    with torch.no_grad():
        y[1] = -s[1] * 0.7  # s.y < 0: the update is skipped for problem 1
    assert ((s * y).sum(-1) <= 0).tolist() == [False, True, False]
    assert _gradcheck(native_ops.update_inverse_hessian, h, s, y)
    assert _gradcheck(native_ops.scale_matrix, r(3, 1, 1).detach().abs().add(0.5).requires_grad_(True), h)
    assert _gradcheck(native_ops.search_direction, h, r(3, n))
    # initial scale: ordinary, y.y under the 1e-5 floor, ratio under the 1e-4 floor (s.y < 0)
    s2 = r(3, n)
    y2 = torch.stack([s2[0].detach() * 0.8 + 0.1, torch.full((n,), 1e-4, dtype=torch.float64),
                      -s2[2].detach()]).requires_grad_(True)
    yy = (y2 * y2).sum(-1)
    ratio = (s2 * y2).sum(-1) / yy.clamp(min=1e-5)
    assert yy[1] < 1e-5 and ratio[2] < 1e-4 and yy[0] > 1e-5 and ratio[0] > 1e-4
    assert _gradcheck(native_ops.initial_scale, s2, y2)
    # the clamped branches pass no gradient into what they clamp (torch's clamp backward)
    gs, gy = torch.autograd.grad(native_ops.initial_scale(s2, y2).sum(), (s2, y2))
    assert gs[2].abs().max() == 0 and gy[2].abs().max() == 0


def test_cpu_ops_refuse_non_contiguous_operands():
    """The host and device kernels read raw row-major pointers: a transposed or sliced view must be
    refused, not computed on the wrong layout."""
    b, n = 2, 5
    h = torch.eye(n, dtype=torch.float64).expand(b, n, n).contiguous()
    s = torch.randn(b, n, dtype=torch.float64)
    y = torch.randn(b, n, dtype=torch.float64)
    s_t = torch.randn(n, b, dtype=torch.float64).t()
    assert not s_t.is_contiguous()
    with pytest.raises(ValueError, match="contiguous"):
        torch.ops.dava.bfgs_update_inverse_hessian(h.transpose(1, 2), s, y)
    with pytest.raises(ValueError, match="contiguous"):
        torch.ops.dava.bfgs_search_direction(torch.randn(b, n, 2 * n, dtype=torch.float64)[:, :, :n], s)
    with pytest.raises(ValueError, match="contiguous"):
        torch.ops.dava.bfgs_initial_scale(s_t, y)
    with pytest.raises(ValueError, match="contiguous"):
        torch.ops.dava.wolfe_init(s_t, torch.zeros(b, dtype=torch.float64), y)
