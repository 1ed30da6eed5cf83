"""The Jacobian sweep on its own (north_star: "rocprof reports achieved HBM GB/s for the Jacobian sweep").

One objective evaluation of the whole batch -- E, the reverse-mode gradient J^T r and the forward-mode
slope d . grad E at the trial point x + alpha d, exactly the pass the fused solve runs per line-search
trial (ba_evaluate_kernel<GRAD, SLOPE, TRIAL>, csrc/bfgs_solve.hip) -- launched alone through
dava_ba_evaluate, timed with HIP events on the launch stream.  This is the reference's
error_function(x) + torch.autograd.grad (bfgs_solver.py:131-135) for a batch.

Algorithmic bytes per problem: observations 8 MN + visibility MN + x, d and grad 3 x 4P + E, slope, alpha
12 B.  Arithmetic: counted by rocprofv3 (SQ_INSTS_VALU_FLOPS_FP32, tools/profile_eval.sh) -- the pass is
VALU work per (view, point) pair, so the VALU peak is its roofline, not HBM.

usage (GPU box): python tools/eval_sweep.py [--config C3|C5|both] [--reps R]  -> one JSON line per config
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {"C3": (8192, 4, 256, True), "C5": (256, 16, 4096, False)}
HBM_PEAK_GBS = 8000.0
VALU_FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table (vector FP32, packed FMA)


def scenes(b, m, n, distortion):
    from deep_attention_visual_odometry_amd import make_scenes

    cache = f"/tmp/dava_scenes_{20251015 + 3000}_0_{b}_{m}_{n}_{int(distortion)}_0.npz"  # bench.py's cache
    if os.path.exists(cache):
        z = np.load(cache)
        return z["initial"], z["observations"], z["visibility"]
    s = make_scenes(b, m, n, distortion=distortion, seed=20251015 + 3000)
    np.savez(cache, initial=s.initial, observations=s.observations, visibility=s.visibility)
    return s.initial, s.observations, s.visibility


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="both", choices=["C3", "C5", "both"])
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import native_ops

    dev = torch.device("cuda", 0)
    for name in (["C3", "C5"] if args.config == "both" else [args.config]):
        b, m, n, dist = CONFIGS[name]
        x0, obs, vis = (torch.tensor(a).to(dev) for a in scenes(b, m, n, dist))
        p = x0.shape[1]
        d = (torch.randn(x0.shape, generator=torch.Generator().manual_seed(3)) * 1e-3).to(dev)
        alpha = torch.full((b,), 0.5, device=dev)

        def run():
            return native_ops.ba_evaluate(x0, obs, vis, m, n, dist, direction=d, alpha=alpha, want_grad=True,
                                          want_slope=True)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            err, grad, slope = run()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        mn = m * n
        algo = b * (9.0 * mn + 12.0 * p + 12.0)
        gbs = algo / (ms * 1e-3) / 1e9
        print(json.dumps({
            "kernel": "ba_evaluate_kernel<GRAD,SLOPE,TRIAL>", "config": name, "batch": b, "views": m, "points": n,
            "distortion": dist, "num_parameters": p, "pairs_per_launch": b * mn, "avg_launch_ms": round(ms, 4),
            "algorithmic_bytes_per_launch": algo, "achieved_GBps": round(gbs, 1),
            "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), "pairs_per_ns": round(b * mn / (ms * 1e6), 2),
            "finite": bool(torch.isfinite(err).all() and torch.isfinite(grad).all() and torch.isfinite(slope).all()),
            "byte_model": "per problem: obs 8MN + vis MN + x, d, grad 4P each + E, slope, alpha",
        }), flush=True)


if __name__ == "__main__":
    main()
