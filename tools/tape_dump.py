"""Diagnostic (GPU box): record one problem's fused solve and print its tape's per-iteration scalars
(alpha_k, rho_j, c_j, gamma, |s|, |y|, s.y) and where the adjoint's running state stops being finite.
usage: python tools/tape_dump.py [--problem 4801] [--batch 8192] [--iterations 100]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", type=int, default=4801)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--iterations", type=int, default=100)
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import make_scenes, native_ops

    dev = torch.device("cuda", 0)
    s = make_scenes(args.batch, 4, 256, distortion=True, seed=7, drop=0.0)
    b = args.problem
    x0 = torch.tensor(s.initial[b:b + 1], device=dev)
    obs = torch.tensor(s.observations[b:b + 1], device=dev)
    vis = torch.tensor(s.visibility[b:b + 1], device=dev).to(torch.uint8)
    k = args.iterations
    x, status, tape = torch.ops.dava.ba_solve_record(x0, obs, vis, 4, 256, True, 1e-4, 0.9, -1.0, k, -1.0, 1000, True,
                                                     0)
    p = x0.shape[1]
    pv = (p + 3) // 4 * 4
    kcap = max(k - 1, 1)
    t = (3 * k + 1 + 3) // 4 * 4
    f = tape.view(torch.float32).cpu().numpy()
    hist = f[: 2 * kcap * pv].reshape(2, kcap, pv)
    xs = f[2 * kcap * pv: 2 * kcap * pv + k * pv].reshape(k, pv)
    gs = f[2 * kcap * pv + k * pv: 2 * kcap * pv + 2 * k * pv].reshape(k, pv)
    sc = f[2 * kcap * pv + 2 * k * pv: 2 * kcap * pv + 2 * k * pv + t]
    print(json.dumps({"status": status.cpu().tolist()[0], "gamma": float(sc[3 * k])}))
    for j in range(k):
        rec = {"k": j, "alpha": float(sc[j]), "|g|": float(np.linalg.norm(gs[j, :p])),
               "|x|": float(np.linalg.norm(xs[j, :p]))}
        if j < k - 1:
            sj, wj = hist[0, j, :p], hist[1, j, :p]
            y = gs[j + 1, :p] - gs[j, :p] if j + 1 < k else None
            rec.update({"rho": float(sc[k + j]), "c": float(sc[2 * k + j]), "|s|": float(np.linalg.norm(sj)),
                        "|w|": float(np.linalg.norm(wj))})
            if y is not None:
                rec.update({"|y|": float(np.linalg.norm(y)), "s.y": float(np.dot(sj.astype(np.float64), y))})
        print(json.dumps(rec))
    xd = x0.clone().requires_grad_(True)
    od = obs.clone().requires_grad_(True)
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError

    out = BFGSSolver(iterations=k, error_threshold=-1.0, minimum_step=-1.0).eval()(
        xd, ReprojectionError(od, vis, 4, 256, True))
    truth = torch.tensor(s.truth[b:b + 1], device=dev, dtype=torch.float32)
    (out - truth).square().sum().backward()
    print(json.dumps({"grad_finite": bool(torch.isfinite(xd.grad).all()), "grad_max": float(xd.grad.abs().max())}))


if __name__ == "__main__":
    main()
