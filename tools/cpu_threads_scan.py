"""Diagnostic (GPU box host): CPU-oracle throughput vs torch thread count on a short C3 sample, to
choose the cpu_baseline thread count (SURVEY 8(d) asks for os.cpu_count(); a box's CPU share may be
far smaller than the machine's count).  usage: python tools/cpu_threads_scan.py [--k 10] [--n 16]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--threads", default="")
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import make_scenes
    from oracle import objective, solver

    s = make_scenes(args.n, 4, 256, distortion=True, seed=20251015 + 3000)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    fn = objective.ReprojectionClosure(obs, vis, 4, 256, True)
    counts = [int(t) for t in args.threads.split(",") if t] or sorted({8, 16, 32, 64, os.cpu_count() or 1})
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    for t in counts:
        torch.set_num_threads(t)
        solver.bfgs_solve(x0[:2], fn.__class__(obs[:2], vis[:2], 4, 256, True), iterations=2, error_threshold=-1.0,
                          minimum_step=-1.0)
        t0 = time.perf_counter()
        solver.bfgs_solve(x0, fn, iterations=args.k, error_threshold=-1.0, minimum_step=-1.0)
        sec = time.perf_counter() - t0
        print(json.dumps({"threads": t, "seconds": round(sec, 3), "problem_iterations_per_s": args.n * args.k / sec,
                          "cpu_count": os.cpu_count(), "affinity": affinity,
                          "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}), flush=True)


if __name__ == "__main__":
    main()
