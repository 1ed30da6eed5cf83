"""Diagnostic (GPU box): what the observation cotangent costs the fused adjoint -- solve + gradient at C5
(B = 256, K = 100) with the observations requiring grad (the HVP read-modify-writes their cotangent every
reverse step) and without (no observation cotangent at all).  Prints the backward time of each.
usage: python tools/adjoint_obs_cost.py [--batch 256] [--views 16] [--points 4096] [--k 100]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402

from deep_attention_visual_odometry_amd import make_scenes, native_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--views", type=int, default=16)
    ap.add_argument("--points", type=int, default=4096)
    ap.add_argument("--k", type=int, default=100)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    s = make_scenes(args.batch, args.views, args.points, distortion=False, seed=20251015 + 3000)
    x0, obs, vis = (torch.tensor(t, device=dev) for t in (s.initial, s.observations, s.visibility))
    kw = dict(iterations=args.k, error_threshold=-1.0, minimum_step=-1.0)
    w = torch.randn_like(x0)
    for rep in range(3):
        for obs_grad in (True, False):
            xg = x0.clone().requires_grad_(True)
            og = obs.clone().requires_grad_(obs_grad)
            x, _ = native_ops.ba_solve_differentiable(xg, og, vis, args.views, args.points, False, **kw)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g = torch.autograd.grad((w * x).sum(), [xg, og] if obs_grad else [xg])
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            print(f"rep {rep} obs_grad={obs_grad}: backward {ms:.2f} ms, finite {bool(torch.isfinite(g[0]).all())}",
                  flush=True)


if __name__ == "__main__":
    main()
