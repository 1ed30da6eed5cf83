"""Diagnostic (GPU box): where does the fused solve of an overflowing problem part from the oracle?

Every line-search trial the oracle makes in the first --iterations iterations is logged (alpha,
f(alpha), phi'(alpha) = autograd w.r.t. alpha); the kernel evaluates the same trial point
(ba_evaluate at the oracle's x_k, d_k, alpha) and the finite / +-Inf / NaN class of its f, its
forward-mode slope and the reverse-mode d . grad are compared with the oracle's.  Then the fused
solve itself runs K = 1 .. --iterations and K = 100 against the oracle.
usage: python tools/nonfinite_probe.py [--problem 4801] [--seed 7] [--iterations 3]
       python tools/nonfinite_probe.py --batch 8 --problem 7 --seed 916 --drop 0.1 --iterations 3
       (--batch > 0: generate that batch and take row --problem of it)
"""
import argparse
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def cls(v: float) -> str:
    return "nan" if math.isnan(v) else ("+inf" if v == math.inf else ("-inf" if v == -math.inf else "fin"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", type=int, default=4801)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--iterations", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--drop", type=float, default=0.0)
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import make_scenes, native_ops
    from oracle import objective, solver

    dev = torch.device("cuda", 0)
    if args.batch > 0:
        s = make_scenes(args.batch, 4, 256, distortion=True, seed=args.seed, drop=args.drop)
        r = slice(args.problem, args.problem + 1)
        x0, obs, vis = (torch.tensor(a)[r] for a in (s.initial, s.observations, s.visibility))
    else:
        s = make_scenes(1, 4, 256, distortion=True, seed=args.seed, first_index=args.problem, drop=args.drop)
        x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
    log, traj = [], []
    solver.bfgs_solve(x0, fn, iterations=args.iterations, error_threshold=-1.0, minimum_step=-1.0,
                      trial_log=log, trajectory=traj)
    od, vd = obs.to(dev), vis.to(dev)
    mismatches = 0
    for k, call in enumerate(log):
        xk, dk = call["x"].to(dev), call["direction"].to(dev)
        for t, tr in enumerate(call["trials"]):
            al = float(tr["alpha"][0])
            f_o, s_o = float(tr["f"][0]), float(tr["dphi"][0])
            e, g, sl = native_ops.ba_evaluate(xk, od, vd, 4, 256, True, direction=dk,
                                              alpha=torch.tensor([al], device=dev), want_grad=True, want_slope=True)
            f_g, s_fwd = float(e.cpu()[0]), float(sl.cpu()[0])
            s_dot = float((g * dk).sum(dim=-1).cpu()[0])
            rec = {"k": k, "trial": t, "alpha": al, "f": [cls(f_o), cls(f_g)],
                   "slope_oracle": cls(s_o), "slope_fwd": cls(s_fwd), "slope_dot": cls(s_dot),
                   "f_oracle": f_o, "f_gpu": f_g}
            bad = cls(f_o) != cls(f_g) or cls(s_o) != cls(s_dot if not (math.isfinite(f_g) and math.isfinite(s_fwd))
                                                         else s_fwd)
            rec["class_mismatch_with_rule"] = bad
            rec["fwd_class_mismatch"] = cls(s_o) != cls(s_fwd)
            mismatches += bad
            print(json.dumps(rec), flush=True)
    print(json.dumps({"trials_logged": sum(len(c["trials"]) for c in log), "class_mismatches_with_rule": mismatches}))
    for k in list(range(1, args.iterations + 1)) + [100]:
        ref = traj[k - 1] if k <= len(traj) else solver.bfgs_solve(x0, fn, iterations=k, error_threshold=-1.0,
                                                                   minimum_step=-1.0)
        xg, _, st = native_ops.ba_solve(x0.to(dev), od, vd, 4, 256, True, iterations=k, error_threshold=-1.0,
                                        minimum_step=-1.0, hessian_mode=1, want_status=True)
        xg = xg.cpu()
        rel = float((xg.double() - ref.double()).norm() / ref.double().norm())
        print(json.dumps({"K": k, "gpu_finite": bool(torch.isfinite(xg).all()),
                          "oracle_finite": bool(torch.isfinite(ref).all()), "rel": rel,
                          "status": st.cpu().tolist()[0]}), flush=True)


if __name__ == "__main__":
    main()
