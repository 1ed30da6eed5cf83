"""Differentiating THROUGH a BA solve (the reference's create_graph mode, bfgs_solver.py:85,134,213-215):
time and peak device memory of the two paths, one JSON line per case.

  fused    the recording solve (one launch, tape in HBM) + the adjoint kernel (one launch),
           csrc/bfgs_adjoint.hip -- the default for ReprojectionError / RayAngleError closures
  generic  the per-iteration loop with a dense (B, P, P) inverse Hessian per iteration kept in the
           autograd graph (HIP VJP kernels per op) -- the GENERIC_BACKWARD override

Forward and backward are timed separately (HIP events on torch's current stream, after one
warm-up); "problems_per_s" is B / (forward + backward).  The adjoint's algorithmic HBM bytes
(reads of the a_j / g_j rows and history rows per reverse step, tape rows, row updates) give its
bandwidth.  usage: python tools/measure_solve_grad.py [--cases c3:8192:100:fused,c2:64:20:generic]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402

SHAPES = {"c1": (2, 64, False), "c2": (2, 128, False), "c3": (4, 256, True)}


def adjoint_bytes(p: int, n: int) -> float:
    """Per problem, n reverse steps: step k reads rows a_j, g_j for j = k .. n-1 (2 (n-k) rows) and
    history rows s_j, w_j for j < k-1 (2 (k-1) rows), reads x_k, g_k, g_{k-1}, s_{k-1}, w_{k-1} and
    the old a_k, writes a_k twice and a_{k-1} once: 8 rows of Pv floats."""
    pv = (p + 3) // 4 * 4
    rows = sum(2 * (n - k) + 2 * max(k - 1, 0) + 8 for k in range(1, n)) + 4
    return 4.0 * pv * rows


def run(shape, b, k, path, dev, repeats=2):
    from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, make_scenes

    m, n, dist = SHAPES[shape]
    s = make_scenes(b, m, n, distortion=dist, seed=7, drop=0.0 if dist else 0.1)
    truth = torch.tensor(s.truth, device=dev, dtype=torch.float32)
    from deep_attention_visual_odometry_amd import _native

    _native.set_debug_override("GENERIC_BACKWARD", 1 if path == "generic" else -1)
    solver = BFGSSolver(iterations=k, error_threshold=-1.0, minimum_step=-1.0).eval()
    times = []
    for rep in range(repeats + 1):  # the first round is the warm-up
        obs = torch.tensor(s.observations, device=dev).requires_grad_(True)
        vis = torch.tensor(s.visibility, device=dev)
        x0 = torch.tensor(s.initial, device=dev).requires_grad_(True)
        fn = ReprojectionError(obs, vis, m, n, dist)
        torch.cuda.synchronize(dev)
        torch.cuda.reset_peak_memory_stats(dev)
        base = torch.cuda.memory_allocated(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        x = solver(x0, fn)
        ev[1].record()
        loss = (x - truth).square().sum()
        gx, gobs = torch.autograd.grad(loss, (x0, obs))
        ev[2].record()
        torch.cuda.synchronize(dev)
        peak = torch.cuda.max_memory_allocated(dev) - base
        if rep > 0:
            times.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
    _native.set_debug_override("GENERIC_BACKWARD", -1)
    fwd = min(t[0] for t in times)
    bwd = min(t[1] for t in times)
    p = x0.shape[1]
    out = {"shape": shape, "B": b, "K": k, "P": p, "path": path, "forward_ms": round(fwd, 3),
           "backward_ms": round(bwd, 3), "problems_per_s": round(b / ((fwd + bwd) * 1e-3), 1),
           "peak_GB": round(peak / 1e9, 3), "dense_H_GB_per_iteration": round(b * p * p * 4 / 1e9, 3),
           "grad_finite": bool(torch.isfinite(gx).all() and torch.isfinite(gobs).all())}
    if path == "fused":
        by = b * adjoint_bytes(p, k)
        out["adjoint_algorithmic_GB"] = round(by / 1e9, 2)
        out["adjoint_GBps_incl_hvp"] = round(by / (bwd * 1e-3) / 1e9, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c2:64:20:generic,c2:64:20:fused,c3:16:20:generic,c3:16:20:fused,"
                                       "c2:1024:100:fused,c3:8192:100:fused")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for case in args.cases.split(","):
        shape, b, k, path = case.split(":")
        try:
            print(json.dumps(run(shape, int(b), int(k), path, dev)), flush=True)
        except torch.cuda.OutOfMemoryError as e:  # the generic loop's dense H graph at scale
            print(json.dumps({"shape": shape, "B": int(b), "K": int(k), "path": path, "error": "out of memory",
                              "detail": str(e)[:200]}), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
