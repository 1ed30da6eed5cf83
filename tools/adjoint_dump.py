"""Diagnostic (GPU box): the fused adjoint's gradients for a few fixed cases, saved to (or compared
between) .npz files -- the bitwise check of an adjoint A/B (run once per library via DAVA_LIB).
usage: python tools/adjoint_dump.py OUT.npz  |  python tools/adjoint_dump.py --compare A.npz B.npz
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import numpy as np  # noqa: E402


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = 0
        for k in sorted(a.files):
            same = np.array_equal(a[k], b[k], equal_nan=True)
            bad += not same
            print(f"{k:24s} bitwise={same}")
        sys.exit(1 if bad else 0)
    import torch

    from deep_attention_visual_odometry_amd import make_scenes

    dev = torch.device("cuda", 0)
    out = {}
    for name, (b, m, n, dist, k, ray) in {"c2_k30": (16, 2, 128, False, 30, False),
                                          "c3_k40": (16, 4, 256, True, 40, False),
                                          "c2ray_k20": (8, 2, 128, False, 20, True)}.items():
        s = make_scenes(b, m, n, distortion=dist, seed=77, drop=0.1, ray_angle=ray)
        x0 = torch.tensor(s.initial, device=dev)
        obs = torch.tensor(s.observations, device=dev)
        vis = torch.tensor(s.visibility, device=dev).to(torch.uint8)
        w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(k)).to(dev)
        x, status, tape = torch.ops.dava.ba_solve_record(x0, obs, vis, m, n, dist, 1e-4, 0.9, -1.0, k, -1.0, 1000,
                                                         True, 1 if ray else 0)
        gx, gobs = torch.ops.dava.ba_solve_backward(w, tape, status, obs, vis, m, n, dist, k, 1 if ray else 0, True)
        out[name + "_gx"] = gx.cpu().numpy()
        out[name + "_gobs"] = gobs.cpu().numpy()
    np.savez(sys.argv[1], **out)


if __name__ == "__main__":
    main()
