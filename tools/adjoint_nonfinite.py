"""Diagnostic (GPU box): which problems of a C3 K = 100 batch get a non-finite gradient through
the fused solve's adjoint, and what the generic loop (the reference's ops one by one, graph kept
by torch) and the CPU oracle (the reference's arithmetic, fp32 autograd) give for the same
problems.  usage: python tools/adjoint_nonfinite.py [--batch 8192] [--iterations 100] [--oracle 2]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def grads(dev, x0, obs, vis, truth, k, generic=False):
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    if generic:
        os.environ["DAVA_GENERIC_BACKWARD"] = "1"
    try:
        xd = x0.to(dev).requires_grad_(True)
        od = obs.to(dev).requires_grad_(True)
        out = BFGSSolver(iterations=k, error_threshold=-1.0, minimum_step=-1.0).eval()(
            xd, ReprojectionError(od, vis.to(dev), 4, 256, True))
        (out - truth.to(dev)).square().sum().backward()
        return out.detach().cpu(), xd.grad.cpu(), od.grad.cpu()
    finally:
        os.environ.pop("DAVA_GENERIC_BACKWARD", None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--oracle", type=int, default=2, help="bad problems to re-run on the CPU oracle")
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import make_scenes
    from oracle import objective, solver

    dev = torch.device("cuda", 0)
    s = make_scenes(args.batch, 4, 256, distortion=True, seed=7, drop=0.0)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    truth = torch.tensor(s.truth, dtype=torch.float32)
    k = args.iterations
    _, gx, go = grads(dev, x0, obs, vis, truth, k)
    bad = (~torch.isfinite(gx).all(-1) | ~torch.isfinite(go.flatten(1)).all(-1)).nonzero().flatten()
    print(json.dumps({"batch": args.batch, "K": k, "nonfinite_problems": int(bad.numel()),
                      "indices": bad[:16].tolist()}), flush=True)
    if bad.numel() == 0:
        return
    idx = bad[:8]
    _, gx_g, go_g = grads(dev, x0[idx], obs[idx], vis[idx], truth[idx], k, generic=True)
    _, gx_f, go_f = grads(dev, x0[idx], obs[idx], vis[idx], truth[idx], k)
    for j, b in enumerate(idx.tolist()):
        rec = {"problem": b, "fused_finite": bool(torch.isfinite(gx_f[j]).all() and torch.isfinite(go_f[j]).all()),
               "generic_finite": bool(torch.isfinite(gx_g[j]).all() and torch.isfinite(go_g[j]).all()),
               "fused_max_abs": float(gx_f[j].abs().nan_to_num(float("inf")).max()),
               "generic_max_abs": float(gx_g[j].abs().nan_to_num(float("inf")).max())}
        if j < args.oracle:
            xr = x0[b:b + 1].clone().requires_grad_(True)
            orr = obs[b:b + 1].clone().requires_grad_(True)
            out = solver.bfgs_solve(xr, objective.ReprojectionClosure(orr, vis[b:b + 1], 4, 256, True), iterations=k,
                                    error_threshold=-1.0, minimum_step=-1.0)
            (out - truth[b:b + 1]).square().sum().backward()
            rec["oracle_finite"] = bool(torch.isfinite(xr.grad).all() and torch.isfinite(orr.grad).all())
            rec["oracle_max_abs"] = float(xr.grad.abs().nan_to_num(float("inf")).max())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
