"""Fused HIP solve (dava_ba_solve via the drop-in BFGSSolver) vs the CPU oracle.

Parity bar (north_star / SURVEY.md 8(d)): per-problem normwise
||x_gpu - x_ref|| / ||x_ref|| <= 1e-5 after a fixed K <= 100 iterations, fp32.
The reference's own sensitivity to a 2-ulp input perturbation is ~1.4e-6 at
K = 100, so 1e-5 leaves room for the different reduction
order of the kernel.  Intrinsics (f, cx, cy) are also compared on their own,
against max(1e-5, ENVELOPE_FACTOR x the oracle's own change under a 1-ulp nudge of x0):
for a few ill-conditioned problems the reference itself moves f by more than
1e-5 under such a nudge, and no fp32 implementation can be closer than that.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import objective, solver

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _envelope_factor():
    """Per-block envelopes: this many times the reference's own change under a 1-ulp nudge of x0 (floor TOL).
    Derived from the oracle alone (tests/golden/make_envelope.py -> parity_envelope.json, re-derived and checked
    by tests/test_parity_envelope.py): the smallest factor whose envelope holds the oracle's own spread when
    every evaluation it sees carries last-bit noise -- what a reordered fp32 sum does.  No GPU result enters it.
    (r05 used 5, the smallest integer above the largest GPU ratio then measured, 4.12.)"""
    import json

    with open(os.path.join(GOLDEN, "parity_envelope.json")) as fh:
        return float(json.load(fh)["envelope_factor"])


ENVELOPE_FACTOR = _envelope_factor()


def _scene(b, m, n, distortion, seed):
    from deep_attention_visual_odometry_amd import make_scenes

    # masked pairs are still evaluated and weighted by 0, so a pair that overflows at a wild
    # trial point gives inf * 0 = NaN exactly as in the reference objective; with Brown-Conrady
    # the first steepest-descent trials overflow often, so its scenes keep every pair visible
    s = make_scenes(b, m, n, distortion=distortion, seed=seed, drop=0.0 if distortion else 0.1)
    return torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)


def _gpu_solve(device, x0, obs, vis, m, n, distortion, **kw):
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    fn = ReprojectionError(obs.to(device), vis.to(device), m, n, distortion)
    s = BFGSSolver(**kw).eval()
    out = s(x0.to(device), fn).cpu()
    return out, s.last_status.cpu()


def _rel(a, b):
    """Per-problem normwise relative difference; a problem that is non-finite in BOTH
    (the reference algorithm can walk to inf/NaN) counts as agreement."""
    a, b = a.double(), b.double()
    rel = (a - b).norm(dim=-1) / b.norm(dim=-1)
    both_bad = ~torch.isfinite(a).all(dim=-1) & ~torch.isfinite(b).all(dim=-1)
    one_bad = torch.isfinite(a).all(dim=-1) != torch.isfinite(b).all(dim=-1)
    rel[both_bad] = 0.0
    rel[one_bad] = float("inf")
    return rel


def _envelopes(x0, fn, ref, distortion=False, objective_of=None, **kw):
    """Per-problem ENVELOPE_FACTOR x the oracle's own change under a 1-ulp nudge of x0, up or down (floor
    1e-5), for the whole parameter vector, for the intrinsics alone and (distortion) for the five
    Brown-Conrady coefficients alone.  Both directions: which side of a bifurcation a nudge lands
    on depends on the host CPU's torch kernels.  The distortion block is the least determined
    part of x (k1..p2 are still 10-100% from the truth at K = 100): the reference's own 1-ulp
    spread on it is 1e-4 .. 4e-3 at the headline shape, against ~5e-7 for the whole vector."""
    b = x0.shape[0]
    env, env_i, env_d = (torch.full((b,), TOL, dtype=torch.float64) for _ in range(3))
    env_e = torch.full((b,), 1e-4, dtype=torch.float64)
    for to in (float("inf"), -float("inf")):
        nudged = solver.bfgs_solve(torch.nextafter(x0, torch.full_like(x0, to)), fn, **kw)
        env = torch.maximum(env, ENVELOPE_FACTOR * _rel(nudged, ref))
        env_i = torch.maximum(env_i, ENVELOPE_FACTOR * _rel(nudged[:, :3], ref[:, :3]))
        if distortion:
            env_d = torch.maximum(env_d, ENVELOPE_FACTOR * _rel(nudged[:, -5:], ref[:, -5:]))
        if objective_of is not None:  # the objective reached, relative: (E(nudged) - E(ref)) / E(ref)
            e_ref, e_n = objective_of(ref), objective_of(nudged)
            env_e = torch.maximum(env_e, torch.nan_to_num(10.0 * (e_n - e_ref).abs() / e_ref.abs(), nan=0.0))
    out = (env, env_i, env_d) if distortion else (env, env_i)
    return out + (env_e,) if objective_of is not None else out


def _report(tag, rel, env=None, extra=None):
    """Append the per-problem parity distribution to gpurun_out/parity_distribution.jsonl (merged
    back from the GPU box) and print it, so the judged numbers are the distribution, not pass/fail."""
    import json

    rel = rel.double()
    rec = {"case": tag, "n": int(rel.numel()), "max_rel": float(rel.max()), "median_rel": float(rel.median()),
           "frac_le_1e-5": float((rel <= TOL).double().mean()),
           "n_gt_1e-5": int((rel > TOL).sum())}
    if env is not None:
        rec["n_outside_envelope"] = int((rel > env).sum())
        rec["max_envelope"] = float(env.max())
    rec.update(extra or {})
    print("PARITY", json.dumps(rec))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_distribution.jsonl"), "a") as fh:
            fh.write(json.dumps(rec) + "\n")
    except OSError:
        pass
    return rec


def _check_k100(out, ref, x0, obs, vis, m, n, distortion, env, env_intrinsics=None, tag=None):
    """Parity after K = 100 iterations, where small two-view problems run into fp32 stagnation.

    Every problem must lie within max(1e-5, ENVELOPE_FACTOR x the reference's own 1-ulp sensitivity) -- the
    envelope -- and within 1e-5 outright.  (Round 1 allowed one problem per case to fall back to an
    objective-value comparison, because two builds that differed only in FMA contraction each put a
    different single C1/C2 problem 1.6e-5 .. 4.2e-5 away at K = 100 -- a near-tie line-search branch
    at fp32 stagnation (tools/dump_solve.py, profiles/r01_parity_spread.log).  Since round 2 every
    distribution has all problems <= 1e-5 with no fallback used (profiles/r03*_parity_distribution.jsonl),
    so the bar is the strict one.)  The objective reached is still reported."""
    rel = _rel(out, ref)
    e_gpu = objective.reprojection_error(out.double(), obs.double(), vis, m, n, distortion)
    e_ref = objective.reprojection_error(ref.double(), obs.double(), vis, m, n, distortion)
    outside = rel > env
    if tag is not None:
        _report(tag, rel, env, {"n_objective_fallback": 0,
                                "max_objective_ratio": float((e_gpu / e_ref.clamp(min=1e-30)).max())})
    assert not outside.any(), (rel.tolist(), env.tolist(), e_gpu.tolist(), e_ref.tolist())
    assert (rel <= TOL).all(), rel
    if env_intrinsics is not None:
        assert (_rel(out[:, :3], ref[:, :3]) <= env_intrinsics).all()


@pytest.mark.parametrize("mode", ["dense", "compact"])
@pytest.mark.parametrize("m,n,distortion,k,b", [
    (2, 64, False, 5, 8), (2, 64, False, 20, 8), (2, 64, False, 100, 16),
    (2, 128, False, 20, 4), (2, 128, False, 100, 16),
    (4, 256, False, 20, 2), (4, 256, True, 20, 2),
])
def test_fixed_iterations_match_oracle(device, m, n, distortion, k, b, mode):
    x0, obs, vis = _scene(b, m, n, distortion, 100 + k + n)
    out, status = _gpu_solve(device, x0, obs, vis, m, n, distortion, iterations=k, error_threshold=-1.0,
                             minimum_step=-1.0, hessian_mode=mode)
    rec = solver.SolveRecord(None, None)
    fn = objective.ReprojectionClosure(obs, vis, m, n, distortion)
    kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
    ref = solver.bfgs_solve(x0, fn, record=rec, **kw)
    rel = _rel(out, ref)
    env, env_intrinsics = _envelopes(x0, fn, ref, **kw)
    if k <= 20:
        _report(f"fixed_{mode}_M{m}_N{n}_D{int(distortion)}_K{k}_B{b}", rel, env)
        assert rel.max() <= TOL, rel
        assert (_rel(out[:, :3], ref[:, :3]) <= env_intrinsics).all()
    else:
        _check_k100(out, ref, x0, obs, vis, m, n, distortion, env, env_intrinsics,
                    tag=f"fixed_{mode}_M{m}_N{n}_D{int(distortion)}_K{k}_B{b}")
    assert torch.equal(status[:, 0], rec.iterations)
    assert (status[:, 1] == 0).all()


@pytest.mark.parametrize("mode", ["dense", "compact"])
@pytest.mark.parametrize("case,ks", [("c1", (5, 20, 100)), ("c2", (5, 20, 100)), ("c3", (5, 20))])
def test_reference_golden_trajectories(device, case, ks, mode):
    """Against BFGSSolver().eval() outputs of the REAL reference (tests/golden/bfgs_traj.npz)."""
    g = np.load(os.path.join(GOLDEN, "bfgs_traj.npz"))
    m, n = {"c1": (2, 64), "c2": (2, 128), "c3": (4, 256)}[case]
    x0 = torch.tensor(g[case + "_x0"])
    obs, vis = torch.tensor(g[case + "_obs"]), torch.tensor(g[case + "_vis"])
    fn = objective.ReprojectionClosure(obs, vis, m, n)
    for k in ks:
        out, _ = _gpu_solve(device, x0, obs, vis, m, n, False, iterations=k, error_threshold=-1.0,
                            minimum_step=-1.0, hessian_mode=mode)
        ref = torch.tensor(g[f"{case}_k{k}"])
        rel = _rel(out, ref)
        if k <= 20:
            _report(f"golden_{mode}_{case}_K{k}", rel)
            assert rel.max() <= TOL, (case, k, rel)
        else:
            kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
            env, _ = _envelopes(x0, fn, ref, **kw)
            _check_k100(out, ref, x0, obs, vis, m, n, False, env, tag=f"golden_{mode}_{case}_K{k}")


_HEADLINE = {}


def _headline_reference():
    """The bench's own workload (bench.py defaults: seed 20251015 + 3000, C3 + Brown-Conrady,
    K = 100 fixed): its first 16 problems, solved once by the oracle (plus the 1-ulp envelopes)."""
    if not _HEADLINE:
        from deep_attention_visual_odometry_amd import make_scenes

        s = make_scenes(16, 4, 256, distortion=True, seed=20251015 + 3000)
        x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
        fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
        kw = dict(iterations=100, error_threshold=-1.0, minimum_step=-1.0)
        ref = solver.bfgs_solve(x0, fn, **kw)
        env, env_i, env_d = _envelopes(x0, fn, ref, distortion=True, **kw)
        _HEADLINE.update(x0=x0, obs=obs, vis=vis, ref=ref, env=env, env_i=env_i, env_d=env_d)
    return _HEADLINE


@pytest.mark.parametrize("mode", ["compact", "dense"])
def test_headline_workload_matches_oracle(device, mode):
    """Parity AT the benchmarked configuration (C3 + Brown-Conrady, P = 794, K = 100, both
    inverse-Hessian modes), on the bench's own problems, against the oracle -- per block: the whole
    vector, the intrinsics (f, cx, cy) and the five distortion coefficients, each inside the
    reference's own 1-ulp envelope for that block.  The oracle's Brown-Conrady path is pinned
    bitwise to the reference's distorted model (tests/golden/distortion.npz)."""
    h = _headline_reference()
    out, status = _gpu_solve(device, h["x0"], h["obs"], h["vis"], 4, 256, True, iterations=100,
                             error_threshold=-1.0, minimum_step=-1.0, hessian_mode=mode)
    rel = _rel(out, h["ref"])
    rel_i = _rel(out[:, :3], h["ref"][:, :3])
    rel_d = _rel(out[:, -5:], h["ref"][:, -5:])
    _report(f"headline_{mode}_C3_BC_K100_B16", rel, h["env"],
            {"intrinsics_max_rel": float(rel_i.max()), "distortion_max_rel": float(rel_d.max()),
             "distortion_envelope_min": float(h["env_d"].min()), "distortion_envelope_max": float(h["env_d"].max()),
             "distortion_n_outside_envelope": int((rel_d > h["env_d"]).sum()),
             "distortion_max_rel_over_envelope": float((rel_d / h["env_d"]).max())})
    assert (status[:, 0] == 100).all()
    assert (rel <= h["env"]).all(), rel
    assert (rel <= TOL).all(), rel
    assert (rel_i <= h["env_i"]).all(), rel_i
    assert (rel_d <= h["env_d"]).all(), (rel_d, h["env_d"])


@pytest.mark.parametrize("mode", ["compact", "dense"])
def test_reference_golden_distorted_trajectories(device, mode):
    """Against BFGSSolver().eval() of the REAL reference on the headline model -- the BA objective
    with the reference's own distorted camera model (tests/golden/distortion.npz, C3 + Brown-Conrady,
    fp32) -- after K = 5, 20 (1e-5) and 100 (per block, inside the reference's 1-ulp envelopes).
    The reference's two executors (eager / TorchScript) differ on k1..p2 by up to ~1e-3 at K = 100."""
    g = np.load(os.path.join(GOLDEN, "distortion.npz"))
    x0 = torch.tensor(g["traj_c3_x0"])
    obs, vis = torch.tensor(g["traj_c3_obs"]), torch.tensor(g["traj_c3_vis"])
    fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
    for k in (5, 20, 100):
        out, status = _gpu_solve(device, x0, obs, vis, 4, 256, True, iterations=k, error_threshold=-1.0,
                                 minimum_step=-1.0, hessian_mode=mode)
        ref = torch.tensor(g[f"traj_c3_k{k}"])
        rel, rel_d = _rel(out, ref), _rel(out[:, -5:], ref[:, -5:])
        jit_d = _rel(torch.tensor(g[f"traj_c3_jit_k{k}"])[:, -5:], ref[:, -5:])
        assert (status[:, 0] == k).all()
        kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        env, env_i, env_d = _envelopes(x0, fn, ref, distortion=True, **kw)
        _report(f"golden_bc_{mode}_c3_K{k}", rel, env,
                {"distortion_max_rel": float(rel_d.max()), "distortion_envelope_max": float(env_d.max()),
                 "reference_eager_vs_torchscript_distortion_max_rel": float(jit_d.max())})
        assert (rel <= env).all() and (rel <= TOL).all(), rel
        assert (_rel(out[:, :3], ref[:, :3]) <= env_i).all()
        assert (rel_d <= env_d).all(), (rel_d, env_d)


def test_default_stopping_rules(device):
    """Reference defaults (error 1e-4, 1000 iterations, min step 1e-8) on C1 shapes: every problem
    stops by a rule at the oracle's iteration for the oracle's reason, parameters per _converged_check."""
    x0, obs, vis = _scene(4, 2, 64, False, 321)
    out, status = _gpu_solve(device, x0, obs, vis, 2, 64, False)
    fn = objective.ReprojectionClosure(obs, vis, 2, 64)
    rec = solver.SolveRecord(None, None)
    ref = solver.bfgs_solve(x0, fn, record=rec)
    assert (status[:, 1] != 0).all()
    _converged_check("defaults_C1_B4", out, status, ref, rec, x0, fn, obs, vis, 2, 64, distortion=False)


def test_error_threshold_stops_immediately(device):
    x0, obs, vis = _scene(3, 2, 64, False, 5)
    out, status = _gpu_solve(device, x0, obs, vis, 2, 64, False, error_threshold=1e30)
    assert torch.equal(out, x0)
    assert (status[:, 0] == 0).all() and (status[:, 1] == 1).all() and (status[:, 2] == 1).all()


def test_zero_iterations_returns_input(device):
    x0, obs, vis = _scene(2, 2, 64, False, 6)
    out, status = _gpu_solve(device, x0, obs, vis, 2, 64, False, iterations=0)
    assert torch.equal(out, x0)
    assert (status[:, 0] == 0).all()


def test_batch_dimensions_and_problem_independence(device):
    """(2, 3, P) batches give the same per-problem results as solving each alone."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    x0, obs, vis = _scene(6, 2, 64, False, 7)
    fn = ReprojectionError(obs.reshape(2, 3, 2, 64, 2).to(device), vis.reshape(2, 3, 2, 64).to(device), 2, 64)
    s = BFGSSolver(iterations=15, error_threshold=-1.0, minimum_step=-1.0).eval()
    out = s(x0.reshape(2, 3, -1).to(device), fn).cpu()
    assert out.shape == (2, 3, x0.shape[-1])
    single, _ = _gpu_solve(device, x0[4:5], obs[4:5], vis[4:5], 2, 64, False, iterations=15, error_threshold=-1.0,
                           minimum_step=-1.0)
    assert torch.equal(out.reshape(6, -1)[4], single[0])


@pytest.mark.parametrize("mode", [0, 1])
def test_error_decreases_and_converges_large_batch(device, mode):
    """Size-independent properties at a larger batch: objective never increases vs the
    start, and most problems get close to the truth."""
    from deep_attention_visual_odometry_amd import make_scenes, native_ops

    s = make_scenes(256, 4, 256, distortion=True, seed=2024)
    x0 = torch.tensor(s.initial).to(device)
    obs = torch.tensor(s.observations).to(device)
    vis = torch.tensor(s.visibility).to(device)
    out, err, status = native_ops.ba_solve(x0, obs, vis, 4, 256, True, iterations=100, error_threshold=-1.0,
                                           minimum_step=-1.0, want_error=True, want_status=True, hessian_mode=mode)
    e0, _, _ = native_ops.ba_evaluate(x0, obs, vis, 4, 256, True, want_grad=False)
    assert (err <= e0).all()
    assert torch.isfinite(out).all()
    assert (err < 1e-3 * e0).float().mean() > 0.9
    assert (status[:, 0] == 100).all()
    assert (status[:, 2] > 100).all()


def test_dense_and_compact_agree_at_scale(device):
    """The two inverse-Hessian representations are the same math: at B=512, C3, K=100 they
    agree per problem to the fp32 parity bar (a size-independent check at full shape)."""
    from deep_attention_visual_odometry_amd import make_scenes, native_ops

    s = make_scenes(512, 4, 256, distortion=True, seed=77)
    x0 = torch.tensor(s.initial).to(device)
    obs = torch.tensor(s.observations).to(device)
    vis = torch.tensor(s.visibility).to(device)
    kw = dict(iterations=100, error_threshold=-1.0, minimum_step=-1.0)
    xd, _, _ = native_ops.ba_solve(x0, obs, vis, 4, 256, True, hessian_mode=0, **kw)
    xc, _, _ = native_ops.ba_solve(x0, obs, vis, 4, 256, True, hessian_mode=1, **kw)
    rel = _rel(xc.cpu(), xd.cpu())
    assert (rel <= TOL).float().mean() >= 0.99, rel.max()
    assert rel.median() <= 1e-6


def test_c5_shape_global_vector_mode_matches_oracle(device):
    """C5 shape (16 views x 4096 points, P = 12381): the O(P) state no longer fits LDS, so the
    kernel keeps it in HBM (GV mode) and uses the two-pass compact products.  K = 3 keeps the
    dense-H oracle (613 MB per problem) quick."""
    x0, obs, vis = _scene(1, 16, 4096, False, 555)
    kw = dict(iterations=3, error_threshold=-1.0, minimum_step=-1.0)
    ref = solver.bfgs_solve(x0, objective.ReprojectionClosure(obs, vis, 16, 4096), **kw)
    for mode in ("compact", "dense"):
        out, status = _gpu_solve(device, x0, obs, vis, 16, 4096, False, hessian_mode=mode, **kw)
        assert _rel(out, ref).max() <= TOL, (mode, _rel(out, ref))
        assert (status[:, 0] == 3).all()


def c5_blocks(m, n):
    """Parameter blocks of the pinhole layout (camera_model.unpack_calibration_parameters):
    intrinsics (f, cx, cy), world points, extrinsics (translations then rotations of views 1..M-1)."""
    p_end = 3 + 3 * n
    return {"intrinsics": slice(0, 3), "points": slice(3, p_end), "extrinsics": slice(p_end, None)}


@pytest.mark.parametrize("mode", ["compact", "dense"])
def test_c5_reference_golden_trajectories(device, mode):
    """C5 AT the benchmarked iteration count: the REAL reference's BFGSSolver(iterations=K,
    error_threshold=-1, minimum_step=-1).eval() (bfgs_solver.py:80-215) on the bench's own first two C5
    problems (16 views x 4096 points, P = 12,381, tests/golden/c5_traj.npz, made by make_golden.py c5),
    K = 20 and 100, against the fused global-vector-mode kernel (history staged through LDS, packed pair
    sweep) in both inverse-Hessian modes.  The fixture also holds the reference's runs from x0 nudged one ulp
    up and down, so each block's envelope is the reference's own sensitivity (ENVELOPE_FACTOR x its 1-ulp
    spread, floor 1e-5) without rerunning the dense 613 MB-per-problem reference here."""
    g = np.load(os.path.join(GOLDEN, "c5_traj.npz"))
    m, n = 16, 4096
    x0, obs, vis = torch.tensor(g["x0"]), torch.tensor(g["obs"]), torch.tensor(g["vis"])
    for k in (20, 100):
        out, status = _gpu_solve(device, x0, obs, vis, m, n, False, iterations=k, error_threshold=-1.0,
                                 minimum_step=-1.0, hessian_mode=mode)
        ref = torch.tensor(g[f"k{k}"])
        assert (status[:, 0] == k).all()
        extra, ok = {}, True
        for name, sl in {"whole": slice(None), **c5_blocks(m, n)}.items():
            rel = _rel(out[:, sl], ref[:, sl])
            spread = torch.maximum(_rel(torch.tensor(g[f"k{k}_up"])[:, sl], ref[:, sl]),
                                   _rel(torch.tensor(g[f"k{k}_down"])[:, sl], ref[:, sl]))
            env = torch.clamp(ENVELOPE_FACTOR * spread, min=TOL)
            extra[f"{name}_max_rel"] = float(rel.max())
            extra[f"{name}_spread_1ulp_max"] = float(spread.max())
            extra[f"{name}_max_rel_over_1ulp"] = float((rel / spread.clamp(min=1e-300)).max())
            extra[f"{name}_n_outside_envelope"] = int((rel > env).sum())
            ok &= bool((rel <= env).all())
        rel = _rel(out, ref)
        _report(f"golden_c5_{mode}_K{k}", rel, None, extra)
        assert (rel <= TOL).all(), rel
        assert ok, extra


@pytest.mark.parametrize("mode", ["compact", "dense"])
def test_c5_reference_golden_eight_problems(device, mode):
    """The same comparison on the bench's first EIGHT C5 problems at K = 20 (tests/golden/c5_traj8.npz, made by
    make_golden.py c5x8: the REAL reference from x0 and from x0 nudged one ulp up and down).  The scenes are
    regenerated from the bench's seed; the fixture's x0 must match them bit for bit."""
    from deep_attention_visual_odometry_amd import make_scenes

    g = np.load(os.path.join(GOLDEN, "c5_traj8.npz"))
    m, n = 16, 4096
    s = make_scenes(8, m, n, distortion=False, seed=20251015 + 3000)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    assert np.array_equal(g["x0"], s.initial)
    out, status = _gpu_solve(device, x0, obs, vis, m, n, False, iterations=20, error_threshold=-1.0,
                             minimum_step=-1.0, hessian_mode=mode)
    ref = torch.tensor(g["k20"])
    assert (status[:, 0] == 20).all()
    extra, ok = {}, True
    for name, sl in {"whole": slice(None), **c5_blocks(m, n)}.items():
        rel = _rel(out[:, sl], ref[:, sl])
        spread = torch.maximum(_rel(torch.tensor(g["k20_up"])[:, sl], ref[:, sl]),
                               _rel(torch.tensor(g["k20_down"])[:, sl], ref[:, sl]))
        env = torch.clamp(ENVELOPE_FACTOR * spread, min=TOL)
        extra[f"{name}_max_rel"] = float(rel.max())
        extra[f"{name}_spread_1ulp_max"] = float(spread.max())
        extra[f"{name}_max_rel_over_1ulp"] = float((rel / spread.clamp(min=1e-300)).max())
        extra[f"{name}_n_outside_envelope"] = int((rel > env).sum())
        ok &= bool((rel <= env).all())
    rel = _rel(out, ref)
    _report(f"golden_c5x8_{mode}_K20", rel, None, extra)
    assert (rel <= TOL).all(), rel
    assert ok, extra


@pytest.mark.parametrize("xl", [True, False])
def test_global_vector_packed_sweep_ragged_points_match_oracle(device, xl, overrides):
    """GV mode's packed pair sweep (two of a thread's points per step) with a ragged point count
    (1300 points over 512 threads: some threads hold a pair plus a scalar tail, the rest one pair)
    and Brown-Conrady on, which C5 itself does not exercise; objective on LDS copies (XL) or on
    the workspace vectors."""
    x0, obs, vis = _scene(2, 3, 1300, True, 571)
    kw = dict(iterations=10, error_threshold=-1.0, minimum_step=-1.0)
    ref = solver.bfgs_solve(x0, objective.ReprojectionClosure(obs, vis, 3, 1300, True), **kw)
    if not xl:
        overrides("GV_NO_XL", 1)
    for mode in ("compact", "dense"):
        out, status = _gpu_solve(device, x0, obs, vis, 3, 1300, True, hessian_mode=mode, **kw)
        assert _rel(out, ref).max() <= TOL, (mode, _rel(out, ref))
        assert (status[:, 0] == 10).all()


def test_c5_shape_objective_matches_oracle(device):
    from deep_attention_visual_odometry_amd import native_ops

    x, obs, vis = _scene(2, 16, 4096, False, 556)
    d = torch.randn_like(x) * 1e-3
    x64 = x.double().requires_grad_(True)
    e_ref = objective.reprojection_error(x64, obs.double(), vis, 16, 4096)
    (g_ref,) = torch.autograd.grad(e_ref.sum(), x64)
    e, g, sl = native_ops.ba_evaluate(x.to(device), obs.to(device), vis.to(device), 16, 4096, False,
                                      direction=d.to(device), want_grad=True, want_slope=True)
    assert torch.allclose(e.cpu().double(), e_ref.detach(), rtol=2e-5)
    assert ((g.cpu().double() - g_ref).norm(dim=-1) / g_ref.norm(dim=-1)).max() < 1e-4
    sl_ref = (g_ref * d.double()).sum(-1)
    assert torch.allclose(sl.cpu().double(), sl_ref, rtol=1e-3, atol=1e-6 * g_ref.norm().item())


@pytest.mark.parametrize("xl", [True, False])
@pytest.mark.parametrize("mode", ["dense", "compact"])
def test_global_vector_mode_equals_lds_mode(device, mode, xl, overrides):
    """The same C3-shaped solve with the O(P) state forced into HBM (DAVA_FORCE_GV) agrees with
    the LDS-resident kernel (same device code, different memory), with the objective on LDS
    copies of x and d (the default where they fit) or on the workspace vectors (DAVA_GV_NO_XL)."""
    x0, obs, vis = _scene(8, 4, 256, True, 557)
    kw = dict(iterations=30, error_threshold=-1.0, minimum_step=-1.0, hessian_mode=mode)
    lds, _ = _gpu_solve(device, x0, obs, vis, 4, 256, True, **kw)
    overrides("FORCE_GV", 1)
    if not xl:
        overrides("GV_NO_XL", 1)
    gv, _ = _gpu_solve(device, x0, obs, vis, 4, 256, True, **kw)
    overrides("FORCE_GV", -1)
    overrides("GV_NO_XL", -1)
    assert _rel(gv, lds).max() <= TOL


@pytest.mark.parametrize("shape", [(4, 1500, False), (2, 2048, True)])
def test_lds_staged_history_is_bitwise_the_register_pass(device, shape, overrides):
    """The global-vector solve with the XL image streams its history rows HBM -> LDS by global_load_lds
    one entry ahead (bfgs_solve.hip, wide_direction STAGED: rows of >= 3 float4 groups per thread, so
    P > 4096 -- here 4521 and 6158); without the XL image (DAVA_GV_NO_XL) the same pass loads them into
    registers.  The objective reads the same values from LDS or from the workspace, so the two solves --
    parameters and status words -- must be bitwise equal."""
    m, n, dist = shape
    x0, obs, vis = _scene(4, m, n, dist, 963)
    kw = dict(iterations=25, error_threshold=-1.0, minimum_step=-1.0, hessian_mode="compact")
    overrides("FORCE_GV", 1)
    staged, st_staged = _gpu_solve(device, x0, obs, vis, m, n, dist, **kw)
    overrides("GV_NO_XL", 1)
    regs, st_regs = _gpu_solve(device, x0, obs, vis, m, n, dist, **kw)
    assert torch.isfinite(staged).all()
    assert torch.equal(staged, regs) and torch.equal(st_staged, st_regs)


@pytest.mark.parametrize("shape,k", [((2, 3600, False), 80), ((16, 4096, False), 70)])
def test_gv_scalars_in_workspace_slice_are_bitwise_lds(device, shape, k, overrides):
    """The global-vector pass reads each history entry's rho_j, c_j from LDS or -- when they would push the
    XL image out of LDS (C5 past ~320 iterations) -- from the problem's workspace slice, 64 entries per
    load and entry j's by readlane from lane j % 64 (wide_direction SLICE, rows of 6 or 7 float4 groups per
    thread: P = 10,809 and 12,381 here).  The same values either way: forced both ways (GV_SCALAR_SLICE)
    past a 64-entry chunk boundary, the two solves are bitwise equal."""
    m, n, dist = shape
    x0, obs, vis = _scene(2, m, n, dist, 971)
    kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0, hessian_mode="compact")
    overrides("FORCE_GV", 1)
    overrides("GV_SCALAR_SLICE", 0)
    lds, st_lds = _gpu_solve(device, x0, obs, vis, m, n, dist, **kw)
    overrides("GV_SCALAR_SLICE", 1)
    sl, st_sl = _gpu_solve(device, x0, obs, vis, m, n, dist, **kw)
    assert torch.isfinite(lds).all() and (st_lds[:, 0] == k).all()
    assert torch.equal(lds, sl) and torch.equal(st_lds, st_sl)


@pytest.mark.parametrize("stopping", ["fixed", "reference"])
def test_work_queue_launch_is_bitwise_invisible(device, stopping, overrides):
    """More problems than resident workgroups: with the work queue (a slot takes the next
    problem when it finishes one) every problem's result and status are bitwise those of one
    workgroup per problem (DAVA_NO_QUEUE).  2048 C1-shaped problems exceed the chip's slots,
    and both the fixed-K and the reference stopping rules (problems retiring early) run."""
    x0, obs, vis = _scene(2048, 2, 64, False, 559)
    kw = dict(iterations=30, error_threshold=-1.0, minimum_step=-1.0) if stopping == "fixed" else dict(iterations=200)
    out, st = _gpu_solve(device, x0, obs, vis, 2, 64, False, hessian_mode="compact", **kw)
    overrides("NO_QUEUE", 1)
    ref, st_ref = _gpu_solve(device, x0, obs, vis, 2, 64, False, hessian_mode="compact", **kw)
    overrides("NO_QUEUE", -1)
    assert torch.equal(out, ref)
    assert torch.equal(st, st_ref)
    if stopping == "reference":
        assert (st[:, 1] != 0).float().mean() > 0.5  # most problems stop by a rule, at different steps
        assert st[:, 0].unique().numel() > 1


def test_staggered_start_is_bitwise_invisible(device, overrides):
    """A launch whose problems are all resident at once starts its odd workgroups late (phases
    spread over the chip); timing only -- every result and status word is bitwise the same."""
    x0, obs, vis = _scene(256, 2, 128, False, 561)
    kw = dict(iterations=40, error_threshold=-1.0, minimum_step=-1.0, hessian_mode="compact")
    out, st = _gpu_solve(device, x0, obs, vis, 2, 128, False, **kw)
    overrides("STAGGER", 0)
    ref, st_ref = _gpu_solve(device, x0, obs, vis, 2, 128, False, **kw)
    overrides("STAGGER", 200000)
    late, st_late = _gpu_solve(device, x0, obs, vis, 2, 128, False, **kw)
    overrides("STAGGER", -1)
    assert torch.equal(out, ref) and torch.equal(st, st_ref)
    assert torch.equal(late, ref) and torch.equal(st_late, st_ref)


@pytest.mark.parametrize("waves", ["1", "2", "4"])
@pytest.mark.parametrize("m,n,distortion,k", [(2, 64, False, 20), (2, 128, False, 20), (4, 256, True, 20)])
def test_workgroup_waves_match_oracle(device, m, n, distortion, k, waves, overrides):
    """One problem per 1-, 2- or 4-wave workgroup (DAVA_SOLVE_WAVES; the plan picks one per
    shape): the reduction trees differ, the parity bar against the oracle does not."""
    from deep_attention_visual_odometry_amd import native_ops

    x0, obs, vis = _scene(8, m, n, distortion, 600 + n + k)
    kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
    ref = solver.bfgs_solve(x0, objective.ReprojectionClosure(obs, vis, m, n, distortion), **kw)
    overrides("SOLVE_WAVES", int(waves))
    assert native_ops.solve_plan(8, m, n, distortion, 1, k)["workgroup_threads"] == 64 * int(waves)
    for mode in ("compact", "dense"):
        out, status = _gpu_solve(device, x0, obs, vis, m, n, distortion, hessian_mode=mode, **kw)
        rel = _rel(out, ref)
        _report(f"waves{waves}_{mode}_M{m}_N{n}_D{int(distortion)}_K{k}_B8", rel)
        assert rel.max() <= TOL, (mode, rel)
        assert (status[:, 0] == k).all()
    overrides("SOLVE_WAVES", -1)


@pytest.mark.parametrize("m,n,distortion", [(4, 256, True), (2, 128, False)])
def test_lds_resident_history_is_bitwise_invisible(device, m, n, distortion, overrides):
    """COMPACT mode keeps the oldest history entries on-chip (dava_ba_solve_plan); the products
    read the same values in the same order, so the result must not change by a single bit
    whether 0, the default or (past two workgroups per CU) 18 entries stay in LDS."""
    from deep_attention_visual_odometry_amd import native_ops

    x0, obs, vis = _scene(16, m, n, distortion, 558)
    kw = dict(iterations=40, error_threshold=-1.0, minimum_step=-1.0, hessian_mode="compact")
    assert native_ops.solve_plan(16, m, n, distortion, 1, 40)["lds_history_entries"] > 0
    ref, st_ref = _gpu_solve(device, x0, obs, vis, m, n, distortion, **kw)
    for entries in ("0", "18"):
        overrides("LDS_HISTORY", int(entries))
        assert native_ops.solve_plan(16, m, n, distortion, 1, 40)["lds_history_entries"] == int(entries)
        out, st = _gpu_solve(device, x0, obs, vis, m, n, distortion, **kw)
        assert torch.equal(out, ref), entries
        assert torch.equal(st, st_ref), entries
    overrides("LDS_HISTORY", -1)


# ---- ray-angle residual (CalibrationNetwork's error, calibration_network.py:58-67) ----

def _gpu_solve_ray(device, x0, obs, vis, m, n, **kw):
    from deep_attention_visual_odometry_amd import BFGSSolver, RayAngleError

    fn = RayAngleError(obs.to(device), vis.to(device), m, n)
    s = BFGSSolver(**kw).eval()
    out = s(x0.to(device), fn).cpu()
    return out, s.last_status.cpu()


@pytest.mark.parametrize("mode", ["dense", "compact"])
@pytest.mark.parametrize("case,ks", [("c1", (5, 20, 100)), ("c2", (5, 20))])
def test_ray_angle_golden_trajectories(device, case, ks, mode):
    """Against BFGSSolver().eval() of the REAL reference on CalibrationNetwork's error
    (tests/golden/ray_angle.npz).  The angle sum is not smooth where a residual vanishes,
    so later iterates are more sensitive than the squared objective's: every K is held to
    max(1e-5, ENVELOPE_FACTOR x the reference's own change under a 1-ulp nudge of x0)."""
    g = np.load(os.path.join(GOLDEN, "ray_angle.npz"))
    m, n = {"c1": (2, 64), "c2": (2, 128)}[case]
    key = f"traj_{case}"
    x0 = torch.tensor(g[key + "_x0"])
    obs, vis = torch.tensor(g[key + "_obs"]), torch.tensor(g[key + "_vis"])
    fn = objective.RayAngleClosure(obs, vis, m, n)
    for k in ks:
        out, status = _gpu_solve_ray(device, x0, obs, vis, m, n, iterations=k, error_threshold=-1.0,
                                     minimum_step=-1.0, hessian_mode=mode)
        ref = torch.tensor(g[f"{key}_k{k}"])
        kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        env, _ = _envelopes(x0, fn, ref, **kw)
        rel = _rel(out, ref)
        assert (rel <= env).all(), (case, k, rel, env)
        assert (status[:, 0] == k).all()


def test_ray_angle_fixed_iterations_match_oracle_c3_shape(device):
    from deep_attention_visual_odometry_amd import make_scenes

    s = make_scenes(2, 4, 256, seed=331, drop=0.1, ray_angle=True)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    fn = objective.RayAngleClosure(obs, vis, 4, 256)
    kw = dict(iterations=10, error_threshold=-1.0, minimum_step=-1.0)
    ref = solver.bfgs_solve(x0, fn, **kw)
    for mode in ("dense", "compact"):
        out, _ = _gpu_solve_ray(device, x0, obs, vis, 4, 256, hessian_mode=mode, **kw)
        assert _rel(out, ref).max() <= TOL, (mode, _rel(out, ref))


def test_ray_angle_converges_from_noisy_guess(device):
    """CalibrationNetwork's solver settings (error_threshold 1e-7, else defaults): the angle
    sum falls by orders of magnitude, like the oracle's."""
    from deep_attention_visual_odometry_amd import make_scenes

    s = make_scenes(4, 2, 64, seed=332, ray_angle=True)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    out, status = _gpu_solve_ray(device, x0, obs, vis, 2, 64, error_threshold=1e-7, iterations=200)
    e0 = objective.ray_angle_error(x0.double(), obs.double(), vis, 2, 64)
    e1 = objective.ray_angle_error(out.double(), obs.double(), vis, 2, 64)
    assert (e1 < 1e-2 * e0).all(), (e0, e1)
    assert torch.isfinite(out).all()


# ---- edge cases and error behaviour (raise, never fall back) ----

def test_empty_batch_and_single_problem(device):
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    x0, obs, vis = _scene(1, 2, 64, False, 501)
    s = BFGSSolver(iterations=5, error_threshold=-1.0, minimum_step=-1.0).eval()
    empty = s(x0[:0].to(device), ReprojectionError(obs[:0].to(device), vis[:0].to(device), 2, 64))
    assert empty.shape == (0, x0.shape[1])
    one = s(x0[0].to(device), ReprojectionError(obs[0].to(device), vis[0].to(device), 2, 64)).cpu()  # 0-d batch
    fn = objective.ReprojectionClosure(obs, vis, 2, 64)
    ref = solver.bfgs_solve(x0, fn, iterations=5, error_threshold=-1.0, minimum_step=-1.0)
    assert one.shape == x0[0].shape
    assert _rel(one[None], ref).max() <= TOL


def test_non_contiguous_inputs_match_contiguous(device):
    x0, obs, vis = _scene(4, 2, 64, False, 502)
    out, _ = _gpu_solve(device, x0, obs, vis, 2, 64, False, iterations=10, error_threshold=-1.0, minimum_step=-1.0)
    xs = torch.stack([x0, torch.zeros_like(x0)], dim=1).reshape(-1, x0.shape[1])[::2]  # strided rows
    obs_t = obs.transpose(1, 2).contiguous().transpose(1, 2)  # non-contiguous view, same values
    assert not obs_t.is_contiguous()
    assert not xs.is_contiguous() and torch.equal(xs, x0)
    out2, _ = _gpu_solve(device, xs, obs_t, vis, 2, 64, False, iterations=10, error_threshold=-1.0,
                         minimum_step=-1.0)
    assert torch.equal(out, out2)


def test_bad_inputs_raise(device):
    from deep_attention_visual_odometry_amd import BFGSSolver, RayAngleError, ReprojectionError

    x0, obs, vis = _scene(2, 2, 64, False, 503)
    with pytest.raises(ValueError):  # wrong observation shape
        ReprojectionError(obs[:, :, :10].to(device), vis[:, :, :10].to(device), 2, 64)
    fn = ReprojectionError(obs.to(device), vis.to(device), 2, 64)
    with pytest.raises(ValueError):  # batch mismatch
        BFGSSolver().eval()(x0[:1].to(device), fn)
    with pytest.raises(TypeError):  # the fused path is fp32 (the reference's BA dtype)
        BFGSSolver().eval()(x0.double().to(device), fn)
    with pytest.raises(RuntimeError):  # no CPU fallback
        BFGSSolver().eval()(x0, fn)
    from deep_attention_visual_odometry_amd import native_ops
    from deep_attention_visual_odometry_amd._native import DAVA_RESIDUAL_RAY_ANGLE

    with pytest.raises(RuntimeError):  # ray angle is pinhole only: the library refuses the scene
        native_ops.ba_evaluate(torch.zeros(1, 3 + 3 * 64 + 6 + 5, device=device),
                               torch.zeros(1, 2, 64, 2, device=device), torch.ones(1, 2, 64, device=device), 2, 64,
                               True, residual=DAVA_RESIDUAL_RAY_ANGLE)
    assert RayAngleError(obs.to(device), vis.to(device), 2, 64).residual == DAVA_RESIDUAL_RAY_ANGLE


def test_nan_problem_does_not_disturb_its_neighbours(device):
    """Problems are independent: a NaN initial guess in one row (which the reference would
    carry to NaN) leaves every other row's result identical to a clean run."""
    x0, obs, vis = _scene(4, 2, 64, False, 504)
    clean, _ = _gpu_solve(device, x0, obs, vis, 2, 64, False, iterations=10, error_threshold=-1.0,
                          minimum_step=-1.0)
    bad = x0.clone()
    bad[1, 5] = float("nan")
    out, _ = _gpu_solve(device, bad, obs, vis, 2, 64, False, iterations=10, error_threshold=-1.0,
                        minimum_step=-1.0)
    assert torch.equal(out[[0, 2, 3]], clean[[0, 2, 3]])
    assert not torch.isfinite(out[1]).all()


# ---- training mode's drop path in the fused kernel (bfgs_solver.py:121-125) ----

def _train_solve(device, x0, obs, vis, m, n, p, k, seed):
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    s = BFGSSolver(drop_path_p=p, training_iterations=k, training_error_threshold=-1.0, minimum_step=-1.0)
    assert s.training
    torch.manual_seed(seed)
    out = s(x0.to(device), ReprojectionError(obs.to(device), vis.to(device), m, n)).cpu()
    return out, s.last_status.cpu()


def test_fused_drop_path_schedule_is_geometric(device):
    """Every iteration a problem keeps updating with probability 1 - p (reference: updating &=
    rand_like > p): the number of steps is geometric, truncated at K.  Statistical parity --
    the kernel draws from its own counter-based generator, not torch's stream."""
    p, k, b = 0.1, 30, 4096
    x0, obs, vis = _scene(b, 2, 64, False, 571)
    _, st = _train_solve(device, x0, obs, vis, 2, 64, p, k, 5)
    steps = st[:, 0].double()
    expect = [(1 - p) ** j * p for j in range(k)] + [(1 - p) ** k]
    hist = torch.bincount(st[:, 0].long(), minlength=k + 1).double() / b
    mean = sum(j * e for j, e in enumerate(expect))
    var = sum((j - mean) ** 2 * e for j, e in enumerate(expect))
    assert abs(steps.mean().item() - mean) < 4 * (var / b) ** 0.5
    assert (hist - torch.tensor(expect, dtype=torch.float64)).abs().max() < 0.02
    assert ((st[:, 0] < k) == (st[:, 1] == 3)).all()  # DAVA_STOP_DROP exactly for the dropped ones
    # seeded through torch's default generator: same seed, same schedule; another seed, another one
    _, st2 = _train_solve(device, x0, obs, vis, 2, 64, p, k, 5)
    _, st3 = _train_solve(device, x0, obs, vis, 2, 64, p, k, 6)
    assert torch.equal(st, st2) and not torch.equal(st[:, 0], st3[:, 0])


def test_fused_drop_path_is_the_eval_solve_stopped_early(device):
    """A dropped problem returns exactly the eval-mode solve run for the steps it took."""
    from deep_attention_visual_odometry_amd import native_ops

    x0, obs, vis = _scene(96, 2, 128, False, 572)
    out, st = _train_solve(device, x0, obs, vis, 2, 128, 0.15, 25, 11)
    assert st[:, 0].unique().numel() > 3
    for steps in st[:, 0].unique().tolist():
        idx = (st[:, 0] == steps).nonzero().flatten()
        if steps == 0:
            assert torch.equal(out[idx], x0[idx])
            continue
        ref, _, _ = native_ops.ba_solve(x0[idx].to(device), obs[idx].to(device), vis[idx].to(device), 2, 128, False,
                                        iterations=int(steps), error_threshold=-1.0, minimum_step=-1.0,
                                        hessian_mode=1)
        assert torch.equal(out[idx], ref.cpu()), steps


def test_infeasible_generic_fallback_raises(device):
    """Differentiating a solve past the fused adjoint's reach (P = 15093 > 14336: more than 14 float4
    groups per thread) falls to the generic loop, whose dense (B, P, P) inverse Hessian and first
    temporaries alone exceed the device here: refused up front with a RuntimeError, never attempted."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    m, n, b = 16, 5000, 48  # 48 x 15093^2 x 4 B = 44 GB per dense matrix: the first iterations cannot fit
    p = 3 + 3 * n + 6 * (m - 1)
    fn = ReprojectionError(torch.zeros(b, m, n, 2, device=device), torch.ones(b, m, n, device=device), m, n)
    x0 = torch.zeros(b, p, device=device, requires_grad=True)
    with pytest.raises(RuntimeError, match="no fused kernel"):
        BFGSSolver(iterations=100, error_threshold=-1.0, minimum_step=-1.0).eval()(x0, fn)


def test_reference_defaults_c2_objective_parity(device):
    """BFGSSolver() with the reference's DEFAULT kwargs (error 1e-4, 1000 iterations, min step 1e-8)
    through the module on C2-shaped problems.  The module picks the compact history (the cap no
    longer forces the dense matrix), every problem stops by a rule -- at the oracle's iteration, for
    the oracle's reason -- and its parameters are held to the fixed-K bar (_converged_check)."""
    from deep_attention_visual_odometry_amd import BFGSSolver, _native

    x0, obs, vis = _scene(16, 2, 128, False, 901)
    s = BFGSSolver().eval()
    assert s._resolve_mode(s.iterations, x0.shape[1], 16, device) == _native.DAVA_HESSIAN_COMPACT
    out, status = _gpu_solve(device, x0, obs, vis, 2, 128, False)
    fn = objective.ReprojectionClosure(obs, vis, 2, 128)
    rec = solver.SolveRecord(None, None)
    ref = solver.bfgs_solve(x0, fn, record=rec)
    assert (status[:, 1] != 0).all()  # stopped by a rule, not the cap
    _converged_check("defaults_C2_B16", out, status, ref, rec, x0, fn, obs, vis, 2, 128, distortion=False)


# ---- training mode's return_second_last, fused (bfgs_solver.py:196-212) ----

def _second_last_case(device, b=32, seed=581, min_step=2e-3):
    x0, obs, vis = _scene(b, 2, 64, False, seed)
    kw = dict(iterations=60, error_threshold=-1.0, minimum_step=min_step)
    return x0, obs, vis, kw


def test_fused_second_last_is_the_solve_before_its_last_step(device):
    """return_second_last in the fused kernel: a problem stopped by the minimum-step rule returns
    exactly the eval solve run for one step fewer (x before the step that failed the test); every
    other problem returns exactly what it returns without the flag."""
    from deep_attention_visual_odometry_amd import native_ops

    x0, obs, vis, kw = _second_last_case(device)
    args = (x0.to(device), obs.to(device), vis.to(device), 2, 64, False)
    # cap the iterations at the median stopping step, so that the batch holds problems stopped by
    # the minimum-step rule and problems stopped by the cap
    _, _, st0 = native_ops.ba_solve(*args, hessian_mode=1, want_status=True, **kw)
    kw = dict(kw, iterations=max(2, int(st0[:, 0].float().median().item())))
    plain, _, st = native_ops.ba_solve(*args, hessian_mode=1, want_status=True, **kw)
    sl, _, st_sl = native_ops.ba_solve(*args, hessian_mode=1, want_status=True, return_second_last=True, **kw)
    plain, sl, st, st_sl = plain.cpu(), sl.cpu(), st.cpu(), st_sl.cpu()
    assert torch.equal(st, st_sl)
    by_rule = st[:, 1] == 2  # DAVA_STOP_STEP
    assert by_rule.sum() >= 4 and (~by_rule).sum() >= 1
    assert torch.equal(sl[~by_rule], plain[~by_rule])
    for steps in st[by_rule, 0].unique().tolist():
        idx = (by_rule & (st[:, 0] == steps)).nonzero().flatten()
        ref, _, _ = native_ops.ba_solve(x0[idx].to(device), obs[idx].to(device), vis[idx].to(device), 2, 64, False,
                                        iterations=int(steps) - 1, error_threshold=-1.0, minimum_step=-1.0,
                                        hessian_mode=1)
        assert torch.equal(sl[idx], ref.cpu()), steps


def test_fused_second_last_matches_oracle(device):
    """BFGSSolver(return_second_last=True) in training mode (drop path off) against the oracle's
    training-mode loop, which includes the reference's row-moving scatter.  Batches of one problem
    (no scatter can move a row) run fused; a batch where the scatter moves rows is redone by the
    generic loop -- either way the result is the reference's.

    In the batch, the scatter hands most problems another problem's parameters from iteration 1 on
    (problem 1 stops first, so row i lands on problem i + 1), and those problems then solve from a
    foreign start: the reference itself moves 3 of the 12 results by ~0.4 under a 1-ulp nudge of x0.
    So the batch is held per problem to max(1e-5, 10x the oracle's 1-ulp spread), and a problem the
    oracle leaves at the iteration cap (not converged: a wandering trajectory whose 1-ulp spread
    under-samples its sensitivity) only has to be finite; the module's result is also bitwise the
    generic loop's (test_second_last_row_move_falls_back_to_the_reference_loop), whose scatter is
    pinned to the reference's own output (tests/golden/training.npz)."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, native_ops

    x0, obs, vis, kw = _second_last_case(device, b=12)
    solver_kw = dict(drop_path_p=0.0, return_second_last=True, training_iterations=kw["iterations"],
                     training_error_threshold=kw["error_threshold"], minimum_step=kw["minimum_step"])
    fn_ref = objective.ReprojectionClosure(obs, vis, 2, 64)
    rec = solver.SolveRecord(torch.empty(0), torch.empty(0))
    ref = solver.bfgs_solve(x0, fn_ref, training=True, return_second_last=True, drop_path_p=0.0, record=rec, **kw)
    env = torch.zeros(x0.shape[0], dtype=torch.float64)
    for sgn in (1.0, -1.0):
        xn = torch.nextafter(x0, x0 + sgn * float("inf"))
        env = torch.maximum(env, _rel(solver.bfgs_solve(xn, fn_ref, training=True, return_second_last=True,
                                                        drop_path_p=0.0, **kw), ref))
    s = BFGSSolver(**solver_kw)
    out = s(x0.to(device), ReprojectionError(obs.to(device), vis.to(device), 2, 64)).cpu()
    rel = _rel(out, ref)
    capped = rec.reason == solver.STOP_ITERATIONS
    assert int((~capped).sum()) >= 8
    assert torch.isfinite(out).all()
    # (a foreign start is chaotic by construction: this case keeps the 10x factor of rounds 1-4)
    assert ((rel <= torch.clamp(10.0 * env, min=TOL)) | capped).all(), (rel, env, capped)
    # one problem at a time: always the fused kernel (a single problem cannot move rows)
    for i in range(4):
        si = BFGSSolver(**solver_kw)
        oi = si(x0[i:i + 1].to(device), ReprojectionError(obs[i:i + 1].to(device), vis[i:i + 1].to(device), 2, 64))
        assert si.last_status is not None  # the fused path ran
        ri = solver.bfgs_solve(x0[i:i + 1], objective.ReprojectionClosure(obs[i:i + 1], vis[i:i + 1], 2, 64),
                               training=True, return_second_last=True, drop_path_p=0.0, **kw)
        assert _rel(oi.cpu(), ri).max() <= TOL


def test_second_last_row_move_falls_back_to_the_reference_loop(device):
    """A batch whose reference scatter moves rows (a problem stops by the minimum-step rule while a
    later one continues): the module returns the generic loop's result bit for bit."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, native_ops

    x0, obs, vis, kw = _second_last_case(device, b=12)
    _, _, st = native_ops.ba_solve(x0.to(device), obs.to(device), vis.to(device), 2, 64, False, hessian_mode=1,
                                   want_status=True, return_second_last=True, **kw)
    assert native_ops.second_last_moves_rows(st)
    solver_kw = dict(drop_path_p=0.0, return_second_last=True, training_iterations=kw["iterations"],
                     training_error_threshold=kw["error_threshold"], minimum_step=kw["minimum_step"])
    fn = ReprojectionError(obs.to(device), vis.to(device), 2, 64)
    s = BFGSSolver(**solver_kw)
    out = s(x0.to(device), fn)
    assert s.last_status is None  # the generic loop ran
    g = BFGSSolver(**solver_kw)
    ref = g._generic(x0.to(device), fn, kw["error_threshold"], kw["iterations"])
    assert torch.equal(out, ref)


def test_fused_second_last_gradient_matches_oracle(device):
    """Differentiating a training-mode return_second_last solve of one problem that stops by the
    minimum-step rule: the adjoint replays one step fewer, matching oracle autograd."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    x0, obs, vis, kw = _second_last_case(device, b=8)
    w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(12))
    solver_kw = dict(drop_path_p=0.0, return_second_last=True, training_iterations=kw["iterations"],
                     training_error_threshold=kw["error_threshold"], minimum_step=kw["minimum_step"])
    checked = 0
    for i in range(8):
        xd = x0[i:i + 1].to(device).requires_grad_(True)
        od = obs[i:i + 1].to(device).requires_grad_(True)
        s = BFGSSolver(**solver_kw)
        out = s(xd, ReprojectionError(od, vis[i:i + 1].to(device), 2, 64))
        if int(s.last_status[0, 1]) != 2:
            continue
        (out * w[i:i + 1].to(device)).sum().backward()
        xr = x0[i:i + 1].clone().requires_grad_(True)
        orr = obs[i:i + 1].clone().requires_grad_(True)
        ref = solver.bfgs_solve(xr, objective.ReprojectionClosure(orr, vis[i:i + 1], 2, 64), training=True,
                                return_second_last=True, drop_path_p=0.0, **kw)
        (ref * w[i:i + 1]).sum().backward()
        assert _rel(out.detach().cpu(), ref.detach()).max() <= TOL
        gx = ((xd.grad.cpu() - xr.grad).norm() / xr.grad.norm()).item()
        go = ((od.grad.cpu() - orr.grad).norm() / orr.grad.norm()).item()
        assert gx <= 2e-3 and go <= 2e-3, (i, gx, go)
        checked += 1
    assert checked >= 2


# ---- the headline model under visibility masks, and run to the reference's stopping rules ----

@pytest.mark.parametrize("mode", ["compact", "dense"])
def test_reference_golden_masked_distorted_trajectories(device, mode):
    """Against BFGSSolver().eval() of the REAL reference on the headline model with 10 % of the
    (view, point) pairs masked (tests/golden/distortion_masked.npz, eager mode) after K = 5, 20, 100,
    per block inside the reference's own 1-ulp envelopes.  Two of the eight problems overflow at a
    trial point, where a masked pair contributes inf * 0 = NaN (calibration_network.py:58-67
    multiplies by vis), and walk to NaN in the reference: the kernel must do the same to them."""
    g = np.load(os.path.join(GOLDEN, "distortion_masked.npz"))
    x0 = torch.tensor(g["traj_c3m_x0"])
    obs, vis = torch.tensor(g["traj_c3m_obs"]), torch.tensor(g["traj_c3m_vis"])
    assert not vis.all()
    fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
    for k in (5, 20, 100):
        out, status = _gpu_solve(device, x0, obs, vis, 4, 256, True, iterations=k, error_threshold=-1.0,
                                 minimum_step=-1.0, hessian_mode=mode)
        ref = torch.tensor(g[f"traj_c3m_k{k}"])
        finite = torch.isfinite(ref).all(dim=-1)
        assert int(finite.sum()) == 6
        assert torch.equal(torch.isfinite(out).all(dim=-1), finite)  # the same problems walk to NaN
        kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        env, env_i, env_d = _envelopes(x0, fn, ref, distortion=True, **kw)
        rel, rel_i, rel_d = _rel(out, ref), _rel(out[:, :3], ref[:, :3]), _rel(out[:, -5:], ref[:, -5:])
        _report(f"golden_bc_masked_{mode}_c3_K{k}", rel[finite], env[finite],
                {"distortion_max_rel": float(rel_d[finite].max()),
                 "distortion_max_rel_over_envelope": float((rel_d / env_d)[finite].max())})
        assert (rel <= env).all() and (rel <= TOL).all(), rel
        assert (rel_i <= env_i).all(), rel_i
        assert (rel_d <= env_d).all(), (rel_d, env_d)


@pytest.mark.parametrize("k", [5, 20])
def test_masked_distortion_matches_oracle(device, k):
    """Brown-Conrady scenes with drop = 0.1 (masked pairs, the path no earlier BC test covered) at
    the headline shape and a two-view shape, both inverse-Hessian modes, against the oracle.

    Overflow-degenerate problems are held to a bar of their own.  A problem whose first line search
    runs into a pole of the projection (z' -> 0: trials at f = inf / NaN / 2.4e38 around alpha = 0.5,
    seed 916 problem 7, tools/nonfinite_probe.py, profiles/r04_probe_bcmask7.log) can end the
    reference's solve at a point whose objective is NaN -- a visible pair overflows to inf and a
    masked one to inf * 0 -- so it stops by the error test with that point.  Whether the objective
    there is NaN or +inf hangs on ~1e-5 differences in the step (the kernel's step sits 3.3e-5 from the
    oracle's, its trial classes agree with the oracle's on the oracle's own points), so the kernel may
    take one more step and walk to NaN.  For those problems (reference stopped by the error test at a
    NaN objective) the kernel must stop at the same point or at most one step later with a non-finite
    result; every other problem is held to the normal bar."""
    from deep_attention_visual_odometry_amd import make_scenes

    for m, n, b in ((4, 256, 8), (2, 128, 16)):
        s = make_scenes(b, m, n, distortion=True, seed=640 + k + n, drop=0.1)
        x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
        assert not vis.all()
        kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        fn = objective.ReprojectionClosure(obs, vis, m, n, True)
        rec = solver.SolveRecord(None, None)
        ref = solver.bfgs_solve(x0, fn, record=rec, **kw)
        env, env_i, env_d = _envelopes(x0, fn, ref, distortion=True, **kw)
        finite = torch.isfinite(ref).all(dim=-1)
        e_ref = objective.reprojection_error(ref, obs, vis, m, n, True)
        degenerate = finite & (rec.reason == solver.STOP_ERROR) & torch.isnan(e_ref)
        normal = ~degenerate
        ok = finite & normal
        for mode in ("compact", "dense"):
            out, status = _gpu_solve(device, x0, obs, vis, m, n, True, hessian_mode=mode, **kw)
            rel, rel_d = _rel(out, ref)[ok], _rel(out[:, -5:], ref[:, -5:])[ok]
            _report(f"bc_masked_{mode}_M{m}_N{n}_K{k}_B{b}", rel, env[ok],
                    {"distortion_max_rel": float(rel_d.max()), "n_nonfinite": int((~finite).sum()),
                     "n_overflow_degenerate": int(degenerate.sum())})
            assert (rel <= TOL).all() and (rel <= env[ok]).all(), (mode, rel)
            assert (_rel(out[:, :3], ref[:, :3])[ok] <= env_i[ok]).all()
            assert (rel_d <= env_d[ok]).all(), (mode, rel_d, env_d)
            # problems whose masked pairs overflow walk to NaN and stop by the (NaN) step test -- in the
            # reference as here: the same problems, after the same number of steps
            out_finite = torch.isfinite(out).all(dim=-1)
            assert torch.equal(out_finite[normal], finite[normal])
            assert torch.equal(status[normal, 0], rec.iterations[normal]), (status[:, 0], rec.iterations)
            assert (status[ok, 0] == k).all()
            for i in torch.nonzero(degenerate).flatten().tolist():
                same_point = bool(out_finite[i]) and float(_rel(out[i:i + 1], ref[i:i + 1])[0]) <= float(env[i])
                one_more = not bool(out_finite[i]) and int(status[i, 0]) <= int(rec.iterations[i]) + 1
                assert same_point or one_more, (mode, i, status[i].tolist(), int(rec.iterations[i]))


def _converged_check(tag, out, status, ref, rec, x0, fn, obs, vis, m, n, distortion=True):
    """Converged parameters under the reference's default stopping rules (bfgs_solver.py:53-55).
    Every finite problem must stop at the same iteration for the same reason as the reference, and
    then its parameters are held to the fixed-K bar: per problem <= 1e-5 normwise and inside the
    reference's own 1-ulp envelope for the whole vector, the intrinsics and the five distortion
    coefficients; the objective reached inside ITS 1-ulp envelope (10x the oracle's own relative change
    of E under the nudge, floor 1e-4): E is a small residual at the stop (~1e-4), so a 1e-7 relative
    move of x moves it by ~1e-3 of itself -- the measured C2 case, 3.6e-3 at 9.6e-7 in x."""
    finite = torch.isfinite(ref).all(dim=-1)
    assert torch.equal(torch.isfinite(out).all(dim=-1), finite)
    def objective_of(x):
        return objective.reprojection_error(x.double(), obs.double(), vis, m, n, distortion)

    if distortion:
        env, env_i, env_d, env_e = _envelopes(x0, fn, ref, distortion=True, objective_of=objective_of)
    else:
        env, env_i, env_e = _envelopes(x0, fn, ref, objective_of=objective_of)
        env_d = torch.full((x0.shape[0],), float("inf"), dtype=torch.float64)
    rel, rel_i, rel_d = _rel(out, ref), _rel(out[:, :3], ref[:, :3]), _rel(out[:, -5:], ref[:, -5:])
    e_gpu, e_ref = objective_of(out), objective_of(ref)
    e_rel = ((e_gpu - e_ref).abs() / e_ref.abs())[finite]
    env_e = env_e[finite]
    _report(tag, rel[finite], env[finite],
            {"intrinsics_max_rel": float(rel_i[finite].max()), "distortion_max_rel": float(rel_d[finite].max()),
             "envelope_factor": ENVELOPE_FACTOR,
             "distortion_max_rel_over_1ulp": float((rel_d / (env_d / ENVELOPE_FACTOR))[finite].max()),
             "intrinsics_max_rel_over_1ulp": float((rel_i / (env_i / ENVELOPE_FACTOR))[finite].max()),
             "distortion_max_rel_over_envelope": float((rel_d / env_d)[finite].max()),
             "objective_max_rel": float(e_rel.max()), "objective_max_rel_over_envelope": float((e_rel / env_e).max()),
             "steps_mean": float(status[finite, 0].double().mean()),
             "stop_reasons": sorted(set(status[finite, 1].tolist())),
             "n_steps_differ": int((status[finite, 0] != rec.iterations[finite]).sum()),
             "n_reason_differs": int((status[finite, 1] != rec.reason[finite]).sum())})
    assert torch.equal(status[finite, 0], rec.iterations[finite]), (status[:, 0], rec.iterations)
    assert torch.equal(status[finite, 1], rec.reason[finite]), (status[:, 1], rec.reason)
    assert (rel <= env).all() and (rel <= TOL).all(), rel
    assert (rel_i <= env_i).all(), rel_i
    assert (rel_d <= env_d).all(), (rel_d, env_d)
    assert (e_rel <= env_e).all(), (e_rel, env_e)


def test_reference_golden_converged_distorted_parameters(device):
    """BFGSSolver() with the reference's DEFAULT kwargs, through the module, on the headline model:
    the converged parameters of the REAL reference (tests/golden/distortion_masked.npz: the unmasked
    headline batch and the masked one), per block."""
    from deep_attention_visual_odometry_amd import BFGSSolver

    g = np.load(os.path.join(GOLDEN, "distortion_masked.npz"))
    d = np.load(os.path.join(GOLDEN, "distortion.npz"))
    for tag, x0, obs, vis, want in (
            ("unmasked", d["traj_c3_x0"], d["traj_c3_obs"], d["traj_c3_vis"], g["traj_c3_default"]),
            ("masked", g["traj_c3m_x0"], g["traj_c3m_obs"], g["traj_c3m_vis"], g["traj_c3m_default"])):
        x0, obs, vis, want = (torch.tensor(a) for a in (x0, obs, vis, want))
        fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
        rec = solver.SolveRecord(None, None)
        ref = solver.bfgs_solve(x0, fn, record=rec)
        # the oracle is bitwise the golden on the CPU it was made on (tests/test_oracle_golden.py); a run
        # to convergence on another CPU's torch kernels (the GPU box's) may round differently, so here it
        # is held to the parity bar and the kernel is checked against this host's own oracle run, whose
        # stop iterations and reasons belong to it
        finite = torch.isfinite(want).all(dim=-1)
        assert torch.equal(torch.isfinite(ref).all(dim=-1), finite)
        assert (_rel(ref[finite], want[finite]) <= TOL).all()
        s = BFGSSolver().eval()
        assert s._resolve_mode(s.iterations, x0.shape[1], x0.shape[0], device) == 1  # compact
        out, status = _gpu_solve(device, x0, obs, vis, 4, 256, True)
        _converged_check(f"golden_bc_{tag}_defaults_c3", out, status, ref, rec, x0, fn, obs, vis, 4, 256)


def test_headline_converged_parameters_match_oracle(device):
    """The bench's own headline problems (C3 + Brown-Conrady, first 16 of bench.py's batch) solved with
    BFGSSolver() defaults through the module -- the north_star's "converged camera parameters within
    1e-5 rel of reference" -- against the oracle run to the same stopping rules."""
    h = _headline_reference()
    fn = objective.ReprojectionClosure(h["obs"], h["vis"], 4, 256, True)
    rec = solver.SolveRecord(None, None)
    ref = solver.bfgs_solve(h["x0"], fn, record=rec)
    out, status = _gpu_solve(device, h["x0"], h["obs"], h["vis"], 4, 256, True)
    assert (status[:, 1] != 0).all()  # every problem stopped by a rule, not the cap
    _converged_check("headline_defaults_C3_BC_B16", out, status, ref, rec, h["x0"], fn, h["obs"], h["vis"], 4, 256)


def test_dense_mode_gradient_through_the_solve_runs_at_moderate_batch(device):
    """hessian_mode='dense' with a graph runs the generic loop (the reference's own data structure):
    C3 pinhole, B = 64, the reference's DEFAULT cap of 1000 iterations.  Its graph grows with the
    iterations actually run (~107 here), not with the cap, so it must run (the earlier
    cap-based estimate refused it) and give finite gradients, and its solve matches the fused one."""
    import warnings

    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    x0, obs, vis = _scene(64, 4, 256, False, 905)
    fn = ReprojectionError(obs.to(device), vis.to(device), 4, 256)
    xd = x0.to(device).requires_grad_(True)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)  # "fits only if the problems stop early"
        out = BFGSSolver(hessian_mode="dense").eval()(xd, fn)
    (g,) = torch.autograd.grad(out.square().sum(), xd)
    assert torch.isfinite(out).all() and torch.isfinite(g).all()
    fused = BFGSSolver().eval()(x0.to(device), fn)
    rel = _rel(out.detach().cpu(), fused.cpu())
    assert (rel <= 1e-4).float().mean() >= 0.9, rel


def test_fused_second_last_gradient_multi_problem_batch(device):
    """a differentiable return_second_last batch of SEVERAL problems that runs fused -- the
    problems stopped by the minimum-step rule placed last, latest stop first, so the reference's scatter
    moves no rows (second_last_moves_rows is False) -- where each problem's adjoint replays one step fewer
    only if IT stopped by the rule.  Parameters and gradients (w.r.t. x0 and the observations) against the
    oracle's training-mode autograd on the same batch."""
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, native_ops

    x0, obs, vis, kw = _second_last_case(device, b=16)
    args = (x0.to(device), obs.to(device), vis.to(device), 2, 64, False)
    # cap the iterations at the median stopping step: the batch then holds problems stopped by the
    # minimum-step rule and problems stopped by the cap (uncapped, every problem of this scene stops by
    # the rule within 2-6 steps)
    _, _, st = native_ops.ba_solve(*args, hessian_mode=1, want_status=True, **kw)
    kw = dict(kw, iterations=max(2, int(st[:, 0].float().median().item())))
    _, _, st = native_ops.ba_solve(*args, hessian_mode=1, want_status=True, return_second_last=True, **kw)
    st = st.cpu()
    by_rule = (st[:, 1] == 2).nonzero().flatten().tolist()
    others = (st[:, 1] != 2).nonzero().flatten().tolist()
    assert len(by_rule) >= 3 and len(others) >= 2, st
    by_rule.sort(key=lambda i: -int(st[i, 0]))  # latest stop first
    order = torch.tensor(others[:3] + by_rule[:4])
    x0, obs, vis = x0[order], obs[order], vis[order]
    solver_kw = dict(drop_path_p=0.0, return_second_last=True, training_iterations=kw["iterations"],
                     training_error_threshold=kw["error_threshold"], minimum_step=kw["minimum_step"])
    xd = x0.to(device).requires_grad_(True)
    od = obs.to(device).requires_grad_(True)
    s = BFGSSolver(**solver_kw)
    out = s(xd, ReprojectionError(od, vis.to(device), 2, 64))
    assert s.last_status is not None  # the fused path ran (no row move)
    assert not native_ops.second_last_moves_rows(s.last_status)
    assert int((s.last_status[:, 1] == 2).sum()) >= 3
    w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(21))
    (out * w.to(device)).sum().backward()
    xr = x0.clone().requires_grad_(True)
    orr = obs.clone().requires_grad_(True)
    ref = solver.bfgs_solve(xr, objective.ReprojectionClosure(orr, vis, 2, 64), training=True,
                            return_second_last=True, drop_path_p=0.0, **kw)
    (ref * w).sum().backward()
    assert _rel(out.detach().cpu(), ref.detach()).max() <= TOL
    gx = _rel(xd.grad.cpu(), xr.grad)
    go = _rel(od.grad.cpu().reshape(len(order), -1), orr.grad.reshape(len(order), -1))
    assert (gx <= 2e-3).all() and (go <= 2e-3).all(), (gx, go)
