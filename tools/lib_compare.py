"""Diagnostic (GPU box): the fused solve of a whole batch under two builds of the library (DAVA_LIB),
each in a fresh subprocess, compared problem by problem: bitwise-equal rows, rows that differ, and
rows that are non-finite in either.  A change meant to touch only overflowing problems (e.g. the
non-finite trial-slope rule) must leave every finite row bitwise unchanged.
usage: python tools/lib_compare.py LIB_A LIB_B [--seed 7] [--batch 8192] [--k 100] [--mode 0|1]
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
s = make_scenes(%(batch)d, %(m)d, %(n)d, distortion=%(dist)r, seed=%(seed)d, ray_angle=%(ray)r)
dev = torch.device("cuda", 0)
x0, obs, vis = (torch.tensor(a, device=dev) for a in (s.initial, s.observations, s.visibility))
x, _, st = native_ops.ba_solve(x0, obs, vis, %(m)d, %(n)d, %(dist)r, iterations=%(k)d, error_threshold=-1.0,
                               minimum_step=-1.0, hessian_mode=%(mode)d, want_status=True, residual=%(res)d)
np.savez(%(out)r, x=x.cpu().numpy(), st=st.cpu().numpy())
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib_a")
    ap.add_argument("lib_b")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--points", type=int, default=256)
    ap.add_argument("--no-distortion", action="store_true")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--mode", type=int, default=1, help="0 = DENSE, 1 = COMPACT")
    ap.add_argument("--residual", choices=["reprojection", "ray_angle"], default="reprojection")
    args = ap.parse_args()
    import numpy as np

    tmp = tempfile.mkdtemp()
    res = {}
    for tag, lib in (("a", args.lib_a), ("b", args.lib_b)):
        out = os.path.join(tmp, tag + ".npz")
        code = CHILD % dict(repo=REPO, batch=args.batch, m=args.views, n=args.points, dist=not args.no_distortion,
                            seed=args.seed, k=args.k, out=out, mode=args.mode,
                    ray=args.residual == "ray_angle", res=1 if args.residual == "ray_angle" else 0)
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, DAVA_DEBUG_OVERRIDES="1", DAVA_LIB=os.path.abspath(lib)),
                       check=True, timeout=300)
        res[tag] = np.load(out)
    xa, xb = res["a"]["x"], res["b"]["x"]
    fa, fb = np.isfinite(xa).all(axis=1), np.isfinite(xb).all(axis=1)
    same = (xa.view(np.uint32) == xb.view(np.uint32)).all(axis=1)
    print(f"seed={args.seed} batch={args.batch} K={args.k}: bitwise-equal rows {int(same.sum())}/{len(same)}; "
          f"differing rows {np.flatnonzero(~same).tolist()[:20]}; non-finite rows a={np.flatnonzero(~fa).tolist()} "
          f"b={np.flatnonzero(~fb).tolist()}; finite-in-both rows differing {int((~same & fa & fb).sum())}")
    for i in np.flatnonzero(~same)[:10]:
        print(f"  row {i}: status a={res['a']['st'][i].tolist()} b={res['b']['st'][i].tolist()}")


if __name__ == "__main__":
    main()
