"""Benchmark: BA problems/sec for the fused MI355X BFGS solve (BASELINE.json metric).

One "step" = one fused solve (``dava_ba_solve``) of this rank's batch of
synthetic problems: C3 = B=8192 per GPU, 4 views x 256 points, pinhole +
Brown-Conrady (P = 794), K = 100 fixed BFGS iterations (error_threshold =
minimum_step = -1, as SURVEY.md 8(d) prescribes for the throughput metric),
strong Wolfe line search, fp32.  With N GPUs each rank solves its own 8192
problems (weak scaling, problems generated per rank from (seed, global
index), no input scatter) and the converged parameters are joined by ONE
RCCL all-gather (config C4 at N = 8: 65536 problems).

Prints ONE JSON line on rank 0 with the metric plus:
  roofline     -- the solve kernel's algorithmic HBM bytes per launch over its
                  HIP-event-timed average launch duration vs 8 TB/s; `traffic`
                  comes from the committed rocprofv3 PMC summary when one for
                  this configuration exists (profiles/), else null.
  cpu_baseline -- the CPU oracle (PyTorch-CPU restatement of the reference,
                  bitwise-equal to it) on a bounded sample of the same workload,
                  rank 0 at N = 1 only.
Launch: python bench.py [--gpus N --steps K --warmup W]
        (N > 1 via torch.distributed.run, one rank per GPU, RCCL backend).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--batch", type=int, default=8192, help="problems per GPU")
    p.add_argument("--views", type=int, default=4)
    p.add_argument("--points", type=int, default=256)
    p.add_argument("--no-distortion", action="store_true")
    p.add_argument("--iterations", type=int, default=100)
    p.add_argument("--mode", choices=["dense", "compact"], default="compact")
    p.add_argument("--residual", choices=["reprojection", "ray_angle"], default="reprojection",
                   help="ray_angle: CalibrationNetwork's error (pinhole only; not the headline metric)")
    p.add_argument("--seed", type=int, default=20251015 + 3000)
    p.add_argument("--error-threshold", type=float, default=-1.0,
                   help=">= 0: stop problems by the reference's rules (e.g. 1e-4 with --minimum-step 1e-8 "
                        "--iterations 1000); not the headline metric, roofline then null")
    p.add_argument("--minimum-step", type=float, default=-1.0)
    p.add_argument("--cpu-sample", type=int, default=32, help="problems timed on the CPU oracle (0 = skip)")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return p.parse_args()


def dense_algorithmic_bytes(p: int, mn: int, iters: int) -> float:
    """Minimum HBM bytes of the dense deferred-update algorithm for one problem:
    iterations k >= 3 read + write H (8 P^2), k = 2 only writes it (4 P^2, H_0 = gamma I is
    synthesised), k = 0, 1 touch no matrix; scene (obs 8 B + vis 1 B per pair) and x0 read
    once, x written once."""
    h = 0.0
    if iters >= 3:
        h = 4.0 * p * p + 8.0 * p * p * (iters - 3)
    return h + 9.0 * mn + 8.0 * p


def compact_algorithmic_bytes(p: int, mn: int, iters: int, lds_entries: int = 0) -> float:
    """Minimum HBM bytes of the compact-history algorithm for one problem (Pv = P rounded
    up to 4 floats): iteration k >= 2 reads the k-1 history rows of S and W once
    (8 (k-1) Pv; the single-pass kernels -- fused per wave for P <= 1024, workgroup-wide
    in global-vector mode for P <= 14336 -- do exactly this, the two-pass fallback for
    mid-size LDS-mode rows reads them twice and is charged the minimum all the same);
    iterations k = 1 .. K-1 append one S and one W row = 8 Pv; scene and x0 read once,
    x written once.  The oldest `lds_entries` entries (dava_ba_solve_plan) never leave the
    CU: they are neither written to nor read from HBM."""
    pv = (p + 3) // 4 * 4
    reads = 8.0 * pv * sum(max(k - 1 - lds_entries, 0) for k in range(2, iters))
    writes = 8.0 * pv * max(iters - 1 - lds_entries, 0)
    return reads + writes + 9.0 * mn + 8.0 * p


def cpu_baseline(args, x0, obs, vis, p):
    from oracle import objective, solver

    n = min(args.cpu_sample, x0.shape[0])
    if args.residual == "ray_angle":
        fn = objective.RayAngleClosure(obs[:n], vis[:n], args.views, args.points)
    else:
        fn = objective.ReprojectionClosure(obs[:n], vis[:n], args.views, args.points, not args.no_distortion)
    threads = torch.get_num_threads()
    t = time.perf_counter()
    solver.bfgs_solve(x0[:n], fn, iterations=args.iterations, error_threshold=args.error_threshold,
                      minimum_step=args.minimum_step)
    dt = time.perf_counter() - t
    return {
        "value": n / dt,
        "unit": "problems/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} problems of the same workload (first {n} of rank 0's batch), K={args.iterations}, "
                  f"oracle = PyTorch-CPU restatement bitwise-equal to the reference, {threads} torch threads, "
                  f"{dt:.1f} s",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from deep_attention_visual_odometry_amd import make_scenes, native_ops
    from deep_attention_visual_odometry_amd import _native
    from deep_attention_visual_odometry_amd.sharding import gather_rows, shard_range

    distortion = not args.no_distortion
    ray = args.residual == "ray_angle"
    if ray and distortion:
        raise SystemExit("--residual ray_angle is pinhole only: add --no-distortion")
    residual = _native.DAVA_RESIDUAL_RAY_ANGLE if ray else _native.DAVA_RESIDUAL_SQUARED_REPROJECTION
    b = args.batch
    first = shard_range(world * b, world, rank).start  # this rank's slab of the global batch
    cache = f"/tmp/dava_scenes_{args.seed}_{first}_{b}_{args.views}_{args.points}_{int(distortion)}_{int(ray)}.npz"
    if os.path.exists(cache):  # generation is ~1 ms/problem on the host; cache it for repeated runs
        z = np.load(cache)
        scenes = type("S", (), {k: z[k] for k in ("initial", "observations", "visibility")})
    else:
        scenes = make_scenes(b, args.views, args.points, distortion=distortion, seed=args.seed,
                             first_index=first, ray_angle=ray)
        np.savez(cache, initial=scenes.initial, observations=scenes.observations, visibility=scenes.visibility)
    x0_cpu = torch.tensor(scenes.initial)
    obs_cpu = torch.tensor(scenes.observations)
    vis_cpu = torch.tensor(scenes.visibility)
    x0 = x0_cpu.to(dev)
    obs = obs_cpu.to(dev)
    vis = vis_cpu.to(dev, dtype=torch.uint8)
    p = x0.shape[1]
    mn = args.views * args.points
    mode = _native.DAVA_HESSIAN_DENSE if args.mode == "dense" else _native.DAVA_HESSIAN_COMPACT
    ws_bytes = native_ops.solve_workspace_bytes(b, args.views, args.points, distortion, mode, args.iterations)
    workspace = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    kernel_ms = []

    def step(timed: bool):
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        x, _, status = native_ops.ba_solve(x0, obs, vis, args.views, args.points, distortion,
                                           iterations=args.iterations, error_threshold=args.error_threshold,
                                           minimum_step=args.minimum_step,
                                           hessian_mode=mode, want_status=True, workspace=workspace,
                                           residual=residual)
        if timed:
            e1.record(stream)
            kernel_ms.append((e0, e1))
        if world > 1:  # the one collective: converged parameters + status of every problem
            gather_rows(x, world * b)
            gather_rows(status, world * b)
        return x, status

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x, status = step(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    launch_ms = float(np.mean([a.elapsed_time(b_) for a, b_ in kernel_ms]))
    st = status.cpu()
    evals = st[:, 2].double().mean().item() / max(args.iterations, 1)
    trials = st[:, 3].double().mean().item() / max(args.iterations, 1)
    finite = bool(torch.isfinite(x).all().item())

    if rank == 0:
        fixed_k = args.error_threshold < 0 and args.minimum_step < 0  # every problem runs exactly K iterations
        headline = fixed_k and (b, args.views, args.points, distortion, ray, args.iterations) == (8192, 4, 256, True, False, 100)
        value = world * b * args.steps / elapsed
        plan = native_ops.solve_plan(b, args.views, args.points, distortion, mode, args.iterations, residual)
        if args.mode == "dense":
            algo = b * dense_algorithmic_bytes(p, mn, args.iterations)
        else:
            algo = b * compact_algorithmic_bytes(p, mn, args.iterations, plan["lds_history_entries"])
        roofline = None
        if algo is not None and fixed_k:
            achieved = algo / (launch_ms * 1e-3) / 1e9
            traffic = None
            try:
                with open(args.traffic_json) as fh:
                    tj = json.load(fh)
                key = f"{args.mode}_B{b}_M{args.views}_N{args.points}_D{int(distortion)}_K{args.iterations}"
                if ray:
                    key += "_ray"
                if plan["lds_history_entries"]:
                    key += f"_L{plan['lds_history_entries']}"
                if key in tj:
                    traffic = tj[key]["hbm_bytes_per_launch"]
            except (OSError, ValueError, KeyError):
                traffic = None
            roofline = {"kernel": "bfgs_ba_solve_kernel", "bound": "hbm", "achieved": round(achieved, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "algorithmic_bytes_per_launch": algo,
                        "avg_launch_ms": round(launch_ms, 3)}
        cpu = cpu_baseline(args, x0_cpu, obs_cpu, vis_cpu, p) if (world == 1 and args.cpu_sample > 0) else None
        line = {
            "metric": f"BA problems/sec (B={b} per GPU, {args.views} views x {args.points} pts"
                      f"{', Brown-Conrady' if distortion else ''}{', ray-angle residual' if ray else ''}, "
                      f"K={args.iterations} BFGS iterations{'' if fixed_k else ' max, reference stopping rules'})",
            "value": round(value, 2),
            "unit": "problems/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded look-at scenes, noise-free observations, x0 = truth + noise)",
            "config": {
                "workload": (("C3" if world == 1 else f"C4-style dp{world}") if headline else "custom") +
                            f": batch={b} per GPU, {args.views} views x {args.points} pts, "
                            f"{'pinhole+Brown-Conrady' if distortion else 'pinhole'}"
                            f"{' ray-angle residual' if ray else ''}, P={p}, "
                            f"K={args.iterations} {'fixed iterations' if fixed_k else f'iterations max, error <= {args.error_threshold}, step <= {args.minimum_step}'}"
                            f", strong Wolfe (c1=1e-4, c2=0.9)",
                "global_batch": world * b,
                "num_parameters": p,
                "iterations": args.iterations,
                "hessian_mode": args.mode,
                "parallelism": f"dp{world} (problem sharding, one RCCL all-gather of x)",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "diagnostics": {"objective_evals_per_iteration": round(evals, 3),
                            "line_search_trials_per_iteration": round(trials, 3),
                            "mean_steps_per_problem": round(st[:, 0].double().mean().item(), 2),
                            "all_finite": finite, "plan": plan},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
