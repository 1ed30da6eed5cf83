"""Diagnostic (GPU box): per-problem work distribution of the bench configurations.

A workgroup-per-problem launch takes as long as its slowest problems, so the tail of
line-search trials / objective evaluations per problem matters as much as the mean.
usage: python tools/status_stats.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402

from deep_attention_visual_odometry_amd import make_scenes, native_ops  # noqa: E402

CONFIGS = {"C2": (1024, 2, 128, False, 20251015 + 3000), "C3": (2048, 4, 256, True, 20251015 + 3000)}


def main():
    dev = torch.device("cuda", 0)
    for tag, (b, m, n, dist, seed) in CONFIGS.items():
        s = make_scenes(b, m, n, distortion=dist, seed=seed)
        x0 = torch.tensor(s.initial, device=dev)
        obs = torch.tensor(s.observations, device=dev)
        vis = torch.tensor(s.visibility, device=dev)
        _, _, st = native_ops.ba_solve(x0, obs, vis, m, n, dist, iterations=100, error_threshold=-1.0,
                                       minimum_step=-1.0, hessian_mode=1, want_status=True)
        st = st.cpu().double()
        for col, name in ((2, "evals"), (3, "trials")):
            v = st[:, col]
            q = torch.quantile(v, torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=torch.float64))
            print(f"{tag} {name}/problem: mean {v.mean():.1f} p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} "
                  f"max {q[3]:.0f}")


if __name__ == "__main__":
    main()
