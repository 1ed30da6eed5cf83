"""Diagnostic (GPU box): dump fused-solve outputs of a few fixed cases for bitwise comparison
of kernel variants (select the library / knobs through the environment).

usage: python tools/dump_solve.py OUT.npz
       python tools/dump_solve.py --compare A.npz B.npz
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import numpy as np  # noqa: E402


def dump(path):
    import torch

    from deep_attention_visual_odometry_amd import make_scenes, native_ops

    dev = torch.device("cuda", 0)
    out = {}
    g = np.load(os.path.join(REPO, "tests", "golden", "bfgs_traj.npz"))
    for case, (m, n) in (("c1", (2, 64)), ("c2", (2, 128))):
        x0 = torch.tensor(g[case + "_x0"], device=dev)
        obs = torch.tensor(g[case + "_obs"], device=dev)
        vis = torch.tensor(g[case + "_vis"], device=dev)
        for mode in (0, 1):
            for k in (20, 100):
                x, _, _ = native_ops.ba_solve(x0, obs, vis, m, n, False, iterations=k, error_threshold=-1.0,
                                              minimum_step=-1.0, hessian_mode=mode)
                out[f"{case}_m{mode}_k{k}"] = x.cpu().numpy()
    s = make_scenes(64, 2, 128, seed=4243)
    x0, obs, vis = (torch.tensor(a, device=dev) for a in (s.initial, s.observations, s.visibility))
    for k in (20, 100):
        x, _, _ = native_ops.ba_solve(x0, obs, vis, 2, 128, False, iterations=k, error_threshold=-1.0,
                                      minimum_step=-1.0, hessian_mode=1)
        out[f"c2b64_k{k}"] = x.cpu().numpy()
    s = make_scenes(64, 4, 256, distortion=True, seed=4242)
    x0 = torch.tensor(s.initial, device=dev)
    obs = torch.tensor(s.observations, device=dev)
    vis = torch.tensor(s.visibility, device=dev)
    for k in (1, 2, 5, 20):
        x, _, _ = native_ops.ba_solve(x0, obs, vis, 4, 256, True, iterations=k, error_threshold=-1.0,
                                      minimum_step=-1.0, hessian_mode=1)
        out[f"c3_k{k}"] = x.cpu().numpy()
    e, gr, sl = native_ops.ba_evaluate(x0, obs, vis, 4, 256, True, direction=x0 * 1e-3, want_grad=True,
                                       want_slope=True)
    out["c3_eval_grad"] = gr.cpu().numpy()
    np.savez(path, **out)


def compare(a, b):
    """Prints one line per case; exit status 1 unless every case is bitwise identical."""
    za, zb = np.load(a), np.load(b)
    all_same = True
    for k in za.files:
        x, y = za[k].astype(np.float64), zb[k].astype(np.float64)
        same = np.array_equal(za[k], zb[k])
        all_same &= same
        rel = np.linalg.norm(x - y, axis=-1) / np.linalg.norm(y, axis=-1)
        print(f"{k:16s} bitwise={same} max_rel={rel.max():.2e}")
    return all_same


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    else:
        dump(sys.argv[1])
