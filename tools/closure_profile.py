"""Diagnostic (GPU box): where the drop-in's generic loop spends its time when called as CalibrationNetwork calls it
(bench.py --entry closure: the torch ray-angle closure), C3 shape, B = 256, K = ITERS (default 10): torch.profiler's
top operators by device time and by host time, plus the wall clock per iteration and the host syncs.
usage: python tools/closure_profile.py [--batch 256] [--iters 10] [--dense]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--points", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dense", action="store_true")
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import BFGSSolver, _native, make_scenes
    from deep_attention_visual_odometry_amd.geometry import closure_ops

    if args.dense:
        _native.set_debug_override("GENERIC_DENSE", 1)
    dev = torch.device("cuda", 0)
    s = make_scenes(args.batch, args.views, args.points, distortion=False, seed=20254015, ray_angle=True)
    x0 = torch.tensor(s.initial, device=dev)
    obs = torch.tensor(s.observations, device=dev)
    vis = torch.tensor(s.visibility, device=dev)
    closure = closure_ops.calibration_network_error(obs, vis.to(obs.dtype), args.views, args.points)
    solver = BFGSSolver(iterations=args.iters, error_threshold=-1.0, minimum_step=-1.0).eval()
    solver(x0, closure)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    solver(x0, closure)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    print(f"wall {wall * 1e3:.1f} ms for {args.iters} iterations ({wall * 1e3 / args.iters:.2f} ms / iteration), "
          f"B = {args.batch}, {'dense' if args.dense else 'compact'}", flush=True)
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        solver(x0, closure)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by="self_cuda_time_total", row_limit=25, max_name_column_width=60))
    print(ka.table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=60))


if __name__ == "__main__":
    main()
