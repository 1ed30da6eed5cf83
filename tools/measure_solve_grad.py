"""Diagnostic (GPU box): time and peak device memory of differentiating THROUGH a solve on the
BA objective (the reference's create_graph mode, bfgs_solver.py:85,134,213-215), i.e. the generic
loop with a dense (B, P, P) inverse Hessian per iteration kept in the autograd graph, at C2 and C3
shapes for a few batch sizes and iteration counts.  One JSON line per case on stdout.

usage: python tools/measure_solve_grad.py [--cases c2:64:20,c3:16:20]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def run(shape, b, k, dev):
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, make_scenes

    m, n, dist = {"c2": (2, 128, False), "c3": (4, 256, True)}[shape]
    s = make_scenes(b, m, n, distortion=dist, seed=7)
    obs = torch.tensor(s.observations, device=dev).requires_grad_(True)
    vis = torch.tensor(s.visibility, device=dev)
    x0 = torch.tensor(s.initial, device=dev).requires_grad_(True)
    fn = ReprojectionError(obs, vis, m, n, dist)
    solver = BFGSSolver(iterations=k, error_threshold=-1.0, minimum_step=-1.0).eval()
    torch.cuda.synchronize(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    t0 = time.perf_counter()
    x = solver(x0, fn)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    fwd_peak = torch.cuda.max_memory_allocated(dev) - base
    loss = (x - torch.tensor(s.truth, device=dev, dtype=torch.float32)).square().sum()
    gx, gobs = torch.autograd.grad(loss, (x0, obs))
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    peak = torch.cuda.max_memory_allocated(dev) - base
    p = x0.shape[1]
    return {"shape": shape, "B": b, "K": k, "P": p, "forward_s": round(t1 - t0, 3), "backward_s": round(t2 - t1, 3),
            "forward_peak_GB": round(fwd_peak / 1e9, 3), "peak_GB": round(peak / 1e9, 3),
            "dense_H_GB_per_iteration": round(b * p * p * 4 / 1e9, 3),
            "grad_finite": bool(torch.isfinite(gx).all() and torch.isfinite(gobs).all())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c2:16:10,c2:64:10,c2:64:20,c3:4:10,c3:16:10,c3:16:20")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for case in args.cases.split(","):
        shape, b, k = case.split(":")
        print(json.dumps(run(shape, int(b), int(k), dev)), flush=True)


if __name__ == "__main__":
    main()
