"""Diagnostic (GPU box): one problem's first iterations on the fused kernel vs the CPU oracle --
x_k, E(x_k), |g(x_k)| per iteration and the line search's step -- to find where they part.
usage: python tools/problem_probe.py [--problem 4801] [--batch 8192] [--seed 7] [--iterations 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", type=int, default=4801)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--iterations", type=int, default=3)
    ap.add_argument("--drop", type=float, default=0.0)
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import make_scenes, native_ops
    from oracle import objective, solver

    dev = torch.device("cuda", 0)
    s = make_scenes(args.batch, 4, 256, distortion=True, seed=args.seed, drop=args.drop)
    b = args.problem
    x0 = torch.tensor(s.initial[b:b + 1])
    obs = torch.tensor(s.observations[b:b + 1])
    vis = torch.tensor(s.visibility[b:b + 1])
    fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
    traj = []
    solver.bfgs_solve(x0, fn, iterations=args.iterations, error_threshold=-1.0, minimum_step=-1.0, trajectory=traj)
    for k in range(1, args.iterations + 1):
        xg, _, st = native_ops.ba_solve(x0.to(dev), obs.to(dev), vis.to(dev), 4, 256, True, iterations=k,
                                        error_threshold=-1.0, minimum_step=-1.0, hessian_mode=1, want_status=True)
        xg = xg.cpu()
        xr = traj[k - 1]
        e_g, g_g, _ = native_ops.ba_evaluate(xg.to(dev), obs.to(dev), vis.to(dev), 4, 256, True)
        x64 = xr.double().requires_grad_(True)
        e_r = objective.reprojection_error(x64, obs.double(), vis, 4, 256, True)
        (g_r,) = torch.autograd.grad(e_r.sum(), x64)
        e_r32 = objective.reprojection_error(xr, obs, vis, 4, 256, True)
        print(json.dumps({"k": k, "status": st.cpu().tolist()[0],
                          "x_rel": float(((xg.double() - xr.double()).norm() / xr.double().norm())),
                          "x_gpu_finite": bool(torch.isfinite(xg).all()),
                          "E_gpu": float(e_g.cpu()[0]), "E_oracle_f32": float(e_r32[0]), "E_oracle_f64": float(e_r[0]),
                          "|g_gpu|": float(g_g.cpu().norm()), "|g_oracle_f64|": float(g_r.norm()),
                          "min_z_hint": float(xr[0, 3 + 2:3 + 3 * 256:3].abs().min())}), flush=True)


def trials(problem=4801, batch=8192, seed=7):
    """First line search of the problem: f and phi' at x0 + alpha d0 (d0 = -g0) on the GPU
    (ba_evaluate, trial point formed in-kernel) and the oracle (fp32, autograd), alpha = 2^-4 .. 2^6."""
    from deep_attention_visual_odometry_amd import make_scenes, native_ops
    from oracle import objective

    dev = torch.device("cuda", 0)
    s = make_scenes(batch, 4, 256, distortion=True, seed=seed, drop=0.0)
    x0 = torch.tensor(s.initial[problem:problem + 1])
    obs = torch.tensor(s.observations[problem:problem + 1])
    vis = torch.tensor(s.visibility[problem:problem + 1])
    xr = x0.clone().requires_grad_(True)
    e0 = objective.reprojection_error(xr, obs, vis, 4, 256, True)
    (g0,) = torch.autograd.grad(e0.sum(), xr)
    d = -1.0 * g0
    for e in range(-4, 7):
        al = 2.0 ** e
        a = torch.tensor([al], requires_grad=True)
        xt = x0 + a * d
        ft = objective.reprojection_error(xt, obs, vis, 4, 256, True)
        (sl,) = torch.autograd.grad(ft.sum(), a)
        eg, _, slg = native_ops.ba_evaluate(x0.to(dev), obs.to(dev), vis.to(dev), 4, 256, True, direction=d.to(dev),
                                            alpha=torch.tensor([al], device=dev), want_grad=True, want_slope=True)
        print(json.dumps({"alpha": al, "f_oracle": float(ft[0]), "f_gpu": float(eg.cpu()[0]),
                          "slope_oracle": float(sl[0]), "slope_gpu": float(slg.cpu()[0])}), flush=True)


if __name__ == "__main__":
    trials() if os.environ.get("PROBE_TRIALS") else main()
