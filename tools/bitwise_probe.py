"""Diagnostic (GPU box): is the fused solve bitwise reproducible, and bitwise invariant under the
launch knobs that must not change results (LDS-resident history entries, work queue)?

Each case runs in a fresh subprocess (the knobs are read at launch from the environment) and the
outputs are compared bitwise.  usage: python tools/bitwise_probe.py [--lib PATH] [--shape c3|c2]
"""
import argparse
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [%(repo)r, %(repo)r + "/deep-attention-visual-odometry_amd"]
from deep_attention_visual_odometry_amd import make_scenes, native_ops
m, n, dist = %(shape)s
s = make_scenes(16, m, n, distortion=dist, seed=558, drop=0.0 if dist else 0.1)
dev = torch.device("cuda", 0)
x0, obs, vis = (torch.tensor(a, device=dev) for a in (s.initial, s.observations, s.visibility))
x, _, st = native_ops.ba_solve(x0, obs, vis, m, n, dist, iterations=%(k)d, error_threshold=-1.0, minimum_step=-1.0,
                               hessian_mode=1, want_status=True)
np.save(%(out)r, x.cpu().numpy())
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--shape", default="c3")
    ap.add_argument("--k", type=int, default=40)
    args = ap.parse_args()
    shape = {"c3": "(4, 256, True)", "c2": "(2, 128, False)"}[args.shape]
    cases = [("default", {}), ("default_again", {}), ("lds0", {"DAVA_LDS_HISTORY": "0"}),
             ("lds18", {"DAVA_LDS_HISTORY": "18"}), ("lds3", {"DAVA_LDS_HISTORY": "3"}),
             ("noqueue", {"DAVA_NO_QUEUE": "1"})]
    import numpy as np

    tmp = tempfile.mkdtemp()
    res = {}
    for name, env in cases:
        out = os.path.join(tmp, name + ".npy")
        e = dict(os.environ, DAVA_DEBUG_OVERRIDES="1", **env)  # the binding reads DAVA_<NAME> once, at load
        if args.lib:
            e["DAVA_LIB"] = args.lib
        code = CHILD % {"repo": REPO, "shape": shape, "k": args.k, "out": out}
        subprocess.run([sys.executable, "-c", code], env=e, check=True, timeout=300)
        res[name] = np.load(out)
    ref = res["default"]
    for name, x in res.items():
        diff = np.abs(x.astype(np.float64) - ref).max()
        rows = int((x != ref).any(axis=1).sum())
        print(f"{args.shape} {name:14s} bitwise={np.array_equal(x, ref)} rows_differing={rows} max_abs={diff:.3e}")


if __name__ == "__main__":
    main()
