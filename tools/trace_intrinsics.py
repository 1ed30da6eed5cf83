"""Trace the bench's per-block parity outlier back to where the fused solve and the oracle part (GPU box).

The bench line's parity block (bench.py cpu_baseline) compares the fused solve with the CPU oracle on the
bench's own first problems; its intrinsics block (f, cx, cy) sat at up to 2.41x the oracle's own change
under a 1-ulp nudge of x0 (BENCH_r04).  This tool finds that problem and follows it:

1. all `--problems` bench problems (C3 + Brown-Conrady, seed 20251015 + 3000, K = 100): the GPU solve, the
   oracle, and the oracle from x0 nudged one ulp up / down; per problem the intrinsics distance and spread;
2. for the worst problem (largest intrinsics distance / spread), every iteration k = 1 .. K: the fused solve
   stopped at k against the oracle's trajectory, and the nudged oracles' trajectories against it, per block;
3. at x0: the gradient from the kernel (ba_evaluate) and from the oracle's fp32 autograd against an fp64
   autograd of the same objective, per block -- how far each fp32 reduction order lies from the exact sum.

usage: python tools/trace_intrinsics.py [--problems 48] [--iterations 100]  -> JSON lines on stdout
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402

from deep_attention_visual_odometry_amd import make_scenes, native_ops  # noqa: E402
from oracle import objective, solver  # noqa: E402

M, N = 4, 256


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm(dim=-1) / b.norm(dim=-1))


def blocks():
    p_end = 3 + 3 * N
    t_end = p_end + 3 * (M - 1)
    return {"whole": slice(None), "intrinsics": slice(0, 3), "points": slice(3, p_end),
            "translations": slice(p_end, t_end), "rotations": slice(t_end, t_end + 3 * (M - 1)),
            "distortion": slice(-5, None)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=48)
    ap.add_argument("--iterations", type=int, default=100)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    K = args.iterations
    s = make_scenes(args.problems, M, N, distortion=True, seed=20251015 + 3000)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    fn = objective.ReprojectionClosure(obs, vis, M, N, True)
    kw = dict(iterations=K, error_threshold=-1.0, minimum_step=-1.0)
    gpu, _, _ = native_ops.ba_solve(x0.to(dev), obs.to(dev), vis.to(dev), M, N, True, hessian_mode=1, **kw)
    gpu = gpu.cpu()
    traj = []
    ref = solver.bfgs_solve(x0, fn, trajectory=traj, **kw)
    nudged = {}
    for tag, to in (("up", float("inf")), ("down", -float("inf"))):
        t = []
        solver.bfgs_solve(torch.nextafter(x0, torch.full_like(x0, to)), fn, trajectory=t, **kw)
        nudged[tag] = t
    B = blocks()
    per = {}
    for name, sl in B.items():
        d = rel(gpu[:, sl], ref[:, sl])
        sp = torch.maximum(rel(nudged["up"][-1][:, sl], ref[:, sl]), rel(nudged["down"][-1][:, sl], ref[:, sl]))
        per[name] = (d, sp)
        r = d / sp.clamp(min=1e-300)
        print(json.dumps({"step": "per-problem", "block": name, "max_rel": float(d.max()),
                          "max_rel_over_1ulp": float(r.max()), "argmax": int(r.argmax()),
                          "median_rel_over_1ulp": float(r.median()),
                          "ratios_sorted_top5": sorted([round(float(v), 3) for v in r], reverse=True)[:5]}),
              flush=True)
    d, sp = per["intrinsics"]
    worst = int((d / sp.clamp(min=1e-300)).argmax())
    print(json.dumps({"step": "worst", "problem": worst, "intrinsics_rel": float(d[worst]),
                      "intrinsics_spread": float(sp[worst])}), flush=True)
    # 2. per-iteration divergence of the worst problem
    xw, ow, vw = x0[worst:worst + 1], obs[worst:worst + 1], vis[worst:worst + 1]
    for k in range(1, K + 1):
        xk, _, _ = native_ops.ba_solve(xw.to(dev), ow.to(dev), vw.to(dev), M, N, True, hessian_mode=1,
                                       iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        xk = xk.cpu()
        rec = {"step": "iteration", "k": k}
        for name in ("whole", "intrinsics", "translations", "distortion"):
            sl = B[name]
            o = traj[k - 1][worst:worst + 1, sl]
            rec[name] = float(rel(xk[:, sl], o)[0])
            rec[name + "_nudge"] = max(float(rel(nudged[t][k - 1][worst:worst + 1, sl], o)[0]) for t in ("up", "down"))
        print(json.dumps(rec), flush=True)
    # 3. the gradient at x0: kernel and oracle fp32 vs fp64, per block
    x64 = xw.double().requires_grad_(True)
    e64 = objective.reprojection_error(x64, ow.double(), vw, M, N, True)
    (g64,) = torch.autograd.grad(e64.sum(), x64)
    x32 = xw.clone().requires_grad_(True)
    e32 = objective.reprojection_error(x32, ow, vw, M, N, True)
    (g32,) = torch.autograd.grad(e32.sum(), x32)
    _, gk, _ = native_ops.ba_evaluate(xw.to(dev), ow.to(dev), vw.to(dev), M, N, True, want_grad=True)
    gk = gk.cpu()
    rec = {"step": "gradient_at_x0"}
    for name, sl in B.items():
        rec[name] = {"kernel_vs_fp64": float(rel(gk[:, sl], g64[:, sl])[0]),
                     "oracle_fp32_vs_fp64": float(rel(g32[:, sl], g64[:, sl])[0]),
                     "kernel_vs_oracle": float(rel(gk[:, sl], g32[:, sl])[0])}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
