"""Benchmark: BA problems/sec for the fused MI355X BFGS solve (BASELINE.json metric).

One "step" = one fused solve (``dava_ba_solve``) of this rank's batch of
synthetic problems: C3 = B=8192 per GPU, 4 views x 256 points, pinhole +
Brown-Conrady (P = 794), K = 100 fixed BFGS iterations (error_threshold =
minimum_step = -1, as SURVEY.md 8(d) prescribes for the throughput metric),
strong Wolfe line search, fp32.  With N GPUs each rank solves its own 8192
problems (weak scaling, problems generated per rank from (seed, global
index), no input scatter) and ONE RCCL all-gather of a packed (B, P + 4)
buffer (parameters + the 4 status words, bit-cast) joins them on every rank
(config C4 at N = 8: 65536 problems).

Prints ONE JSON line on rank 0 with the metric plus:
  roofline     -- the solve kernel's algorithmic HBM bytes per launch (compact
                  byte model, stated in `byte_model`; the dense 8P^2 model's
                  equivalent rate beside it) over its HIP-event-timed average
                  launch duration vs 8 TB/s; `traffic` is the rocprofv3 PMC
                  figure for this exact configuration from the committed summary
                  (profiles/pmc_traffic.json, source tag in `traffic_source`),
                  else null.
  cpu_baseline -- the CPU oracle (PyTorch-CPU restatement of the reference,
                  bitwise-equal to it) on a bounded sample of the same workload:
                  1 warm-up, then 3 timed runs on 3 disjoint slices, median rate;
                  rank 0 at N = 1 only.
  parity       -- the GPU result for those same sampled problems against the
                  oracle's: per-problem normwise relative error distribution.
Launch: python bench.py [--gpus N --steps K --warmup W]
        N > 1 without WORLD_SIZE in the environment: this process starts N ranks
        itself (python -m torch.distributed.run, one rank per GPU, RCCL backend)
        before touching the GPU and exits with their status.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
HBM_COPY_GBS = 6290.0  # measured float4 copy (MI355X_MICROARCH.md chip table: 79% of spec)
PARITY_BAR = 1e-5  # north_star: converged params within 1e-5 rel of the reference
# per-block envelopes: max(1e-5, this x the oracle's own 1-ulp change); derived from the oracle alone
# (tests/golden/make_envelope.py -> parity_envelope.json; the GPU tests read the same file)
with open(os.path.join(REPO, "tests", "golden", "parity_envelope.json")) as _fh:
    ENVELOPE_FACTOR = float(json.load(_fh)["envelope_factor"])


def parse(argv=None):
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
    p.add_argument("--parity-envelope", type=int, default=16,
                   help="problems of the first CPU slice whose per-block 1-ulp envelopes are computed (0 = skip)")
    p.add_argument("--cpu-sample", type=int, default=16,
                   help="problems per timed CPU-oracle run (3 runs on disjoint slices; 0 = skip)")
    p.add_argument("--no-converged-parity", dest="converged_parity", action="store_false",
                   help="skip parity.converged (the cpu_baseline problems solved by the reference's stopping rules on "
                        "both sides; ~1 min of CPU)")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    p.add_argument("--entry", choices=["op", "module", "closure"], default="op",
                   help="module: time the drop-in BFGSSolver(...).eval()(x0, ReprojectionError) call itself "
                        "(its own Hessian-mode choice and workspace allocation) instead of the op with a reused "
                        "workspace; closure: the drop-in called as the reference's CalibrationNetwork calls it, with "
                        "its torch error closure (networks/calibration_network.py:58-67, ray angle, pinhole), which "
                        "runs the generic loop -- not the headline metric")
    p.add_argument("--differentiate", action="store_true",
                   help="time the solve AND its gradient (recording solve + adjoint kernel, d(w.x)/d(x0, obs)) -- "
                        "the reference's create_graph mode; not the headline metric")
    p.add_argument("--no-live-counters", action="store_true",
                   help="skip the rocprofv3 FETCH_SIZE / WRITE_SIZE child passes and the history-stream ceiling run "
                        "that follow the timed region at N = 1 (roofline.traffic then comes from the committed summary)")
    p.add_argument("--sustain-seconds", type=float, default=10.0,
                   help="after the timed region, keep solving the same batch for about this long (same step, no "
                        "collective) and report the sustained rate beside the timed one (clocks and power at "
                        "steady state; a phase long enough for a GPU-busy sampler to see).  0 = skip")
    p.add_argument("--launch-test", action="store_true",
                   help="multi-rank LAUNCH plumbing check on CPU (gloo, identity stub instead of the solve); "
                        "prints a line marked as a launch test, never a measurement")
    return p.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """Start args.gpus ranks of this script via torch.distributed.run and return their exit code.
    Runs in a parent that has not touched the GPU (no HIP call happens before this point), and
    starts the ranks as child processes -- nothing is exec'd in place."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    return subprocess.call(cmd, env=env)


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


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _rel(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    a, b = a.double(), b.double()
    return (a - b).norm(dim=-1) / b.norm(dim=-1)


def cpu_baseline(args, x0, obs, vis, x_gpu):
    """The CPU oracle on 3 disjoint slices of args.cpu_sample problems each (after one short
    warm-up solve), median rate; plus the parity of the GPU result on the same problems."""
    from oracle import objective, solver

    n = min(args.cpu_sample, x0.shape[0] // 3)
    if n <= 0:
        return None, None

    def closure(lo, hi):
        if args.residual == "ray_angle":
            return objective.RayAngleClosure(obs[lo:hi], vis[lo:hi], args.views, args.points)
        return objective.ReprojectionClosure(obs[lo:hi], vis[lo:hi], args.views, args.points,
                                             not args.no_distortion)

    kw = dict(iterations=args.iterations, error_threshold=args.error_threshold, minimum_step=args.minimum_step)
    threads = torch.get_num_threads()  # the box's CPU share (OMP_NUM_THREADS), not the machine's count
    solver.bfgs_solve(x0[:2], closure(0, 2), iterations=3, error_threshold=-1.0, minimum_step=-1.0)  # warm-up
    secs, refs = [], []
    for r in range(3):
        lo, hi = r * n, (r + 1) * n
        t = time.perf_counter()
        refs.append(solver.bfgs_solve(x0[lo:hi], closure(lo, hi), **kw))
        secs.append(time.perf_counter() - t)
    rate = statistics.median(n / s for s in secs)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    cpu = {
        "value": rate,
        "unit": "problems/s",
        "cores": threads,
        "kind": "port",
        "sample": f"3 timed runs of {n} problems each (problems 0..{3 * n - 1} of rank 0's batch, disjoint "
                  f"slices), same workload K={args.iterations}, after a 2-problem warm-up; median rate. "
                  f"Oracle = PyTorch-CPU restatement bitwise-equal to the reference; {threads} torch threads "
                  f"(the box's CPU share; os.cpu_count()={os.cpu_count()}, affinity={affinity}); "
                  f"run seconds {[round(s, 2) for s in secs]}; the full batch of {x0.shape[0]} would take "
                  f"~{x0.shape[0] / rate:.0f} s at this rate",
        "cpu_model": _cpu_model(),
    }
    ref = torch.cat(refs)
    gpu = x_gpu[: 3 * n].detach().cpu()
    rel = _rel(gpu, ref)
    rel_i = _rel(gpu[:, :3], ref[:, :3])
    parity = {
        "n": int(ref.shape[0]),
        "bar": PARITY_BAR,
        "max_rel": float(rel.max()),
        "median_rel": float(rel.median()),
        "frac_le_bar": float((rel <= PARITY_BAR).double().mean()),
        "intrinsics_max_rel": float(rel_i.max()),
        "metric": "per-problem ||x_gpu - x_oracle|| / ||x_oracle||, fp64 norms, same problems as cpu_baseline",
    }
    if not args.no_distortion and args.parity_envelope > 0:
        # per-block envelopes on the first slice: ENVELOPE_FACTOR x the oracle's own change under a 1-ulp nudge of x0
        # (up and down), floor 1e-5 -- the reference's sensitivity, the bar no fp32 solver can beat
        m = min(args.parity_envelope, n)
        spread = {k: torch.zeros((m,), dtype=torch.float64) for k in ("x", "i", "d")}  # the 1x 1-ulp spread
        for to in (float("inf"), -float("inf")):
            nudged = solver.bfgs_solve(torch.nextafter(x0[:m], torch.full_like(x0[:m], to)), closure(0, m), **kw)
            for key, sl in (("x", slice(None)), ("i", slice(0, 3)), ("d", slice(-5, None))):
                spread[key] = torch.maximum(spread[key], _rel(nudged[:, sl], ref[:m, sl]))
        noise = ulp_noise_spread(solver, x0[:m], closure(0, m), kw, ref[:m])
        parity["over_per_evaluation_ulp_noise"] = {
            k: {"max": float((r[:m] / noise[key].clamp(min=1e-300)).max()),
                "median": float((r[:m] / noise[key].clamp(min=1e-300)).median()),
                "spread_max": float(noise[key][torch.isfinite(noise[key])].max()) if torch.isfinite(noise[key]).any()
                else None,
                "n_noise_runs_nonfinite": int((~torch.isfinite(noise[key])).sum())}
            for k, key, r in (("whole", "x", rel), ("intrinsics", "i", rel_i),
                              ("distortion", "d", _rel(gpu[:, -5:], ref[:, -5:])))}
        parity["over_per_evaluation_ulp_noise"]["note"] = (
            "the GPU's distance from the oracle over the oracle's own spread when EVERY objective value and iterate "
            "gradient it sees moves by -1/0/+1 ulp at random (max over 2 seeds; oracle.solver ulp_noise) -- the "
            "perturbation a reordered fp32 sum makes in every evaluation, where the x0 nudge perturbs the start only")
        env = {k: torch.clamp(ENVELOPE_FACTOR * v, min=PARITY_BAR) for k, v in spread.items()}
        rel_d = _rel(gpu[:, -5:], ref[:, -5:])

        def over(r, k):  # the GPU's distance in units of the reference's own 1-ulp spread (floor: 1 ulp of it)
            q = r[:m] / torch.clamp(spread[k], min=1e-300)
            return {"max": float(q.max()), "median": float(q.median())}

        parity.update({
            "whole_max_rel_over_1ulp": over(rel, "x"),
            "intrinsics_max_rel_over_1ulp": over(rel_i, "i"),
            "distortion_max_rel_over_1ulp": over(rel_d, "d"),
            "distortion_spread_1ulp_max": float(spread["d"].max()),
            "distortion_max_rel": float(rel_d.max()),
            "distortion_frac_le_bar": float((rel_d <= PARITY_BAR).double().mean()),
            "envelope_problems": m,
            "envelope_n_outside": {"whole": int((rel[:m] > env["x"]).sum()),
                                   "intrinsics": int((rel_i[:m] > env["i"]).sum()),
                                   "distortion": int((rel_d[:m] > env["d"]).sum())},
            "distortion_envelope_max": float(env["d"].max()),
            "distortion_envelope_min": float(env["d"].min()),
            "distortion_max_rel_over_envelope": float((rel_d[:m] / env["d"]).max()),
            "envelope_factor": ENVELOPE_FACTOR,
            "envelope_factor_source": "tests/golden/parity_envelope.json: the smallest factor whose envelope holds "
                                      "the ORACLE's own spread under per-evaluation ulp noise (tests/golden/"
                                      "make_envelope.py; no GPU result enters it; tests/test_parity_envelope.py "
                                      "re-derives it and checks the tests and this file use it)",
            "note": ("per-block envelopes = max(1e-5, envelope_factor x the oracle's own change under a 1-ulp nudge of x0); "
                     "*_over_1ulp = the GPU's distance / that change (1x, no floor): <= 1 means no farther from the "
                     "oracle than the reference is from itself under a 1-ulp nudge; the "
                     "oracle's Brown-Conrady path is bitwise the reference's distorted_camera_model._full_forward_model "
                     "(tests/golden/distortion.npz), whose own eager and TorchScript runs differ on k1..p2 by up to "
                     "~1e-3 at K=100"),
        })
    if args.converged_parity and args.residual == "reprojection" and args.error_threshold < 0:
        parity["converged"] = converged_parity(args, x0[: 3 * n], obs[: 3 * n], vis[: 3 * n],
                                               closure, args.parity_envelope, x_gpu.device)
    return cpu, parity


BLOCKS = (("x", slice(None)), ("i", slice(0, 3)), ("d", slice(-5, None)))


def ulp_noise_spread(solver, x0, closure, kw, ref, seeds=(1, 2)):
    """Per problem and block, the oracle's largest distance from its own result `ref` when every evaluation it
    sees carries random 1-ulp noise (oracle.solver.bfgs_solve ulp_noise), over `seeds`."""
    out = {k: torch.zeros((x0.shape[0],), dtype=torch.float64) for k, _ in BLOCKS}
    for seed in seeds:
        noisy = solver.bfgs_solve(x0, closure, ulp_noise=torch.Generator().manual_seed(seed), **kw)
        for key, sl in BLOCKS:
            r = _rel(noisy[:, sl], ref[:, sl])
            # a noisy run that walks to inf / NaN (a wild trial under Brown-Conrady): an unbounded spread, so that
            # problem drops out of the ratios (GPU distance / inf = 0) instead of turning them into NaN
            out[key] = torch.maximum(out[key], torch.where(torch.isfinite(r), r, torch.full_like(r, float("inf"))))
    return out


def converged_parity(args, x0, obs, vis, closure, n_env, dev):
    """north_star's 'converged camera parameters ... within 1e-5 rel': the reference's stopping rules
    (error 1e-4, 1000 iterations, step 1e-8: bfgs_solver.py:53-55) on the cpu_baseline problems, the fused solve
    against the oracle run the same way.  Per camera parameter (f, cx, cy, k1..p2): max |rel| and the fraction of
    problems within 1e-5; per block: the GPU's distance over the oracle's own spread (1-ulp nudge of x0 up/down,
    and per-evaluation ulp noise) on the first n_env problems, and the stop iterations / reasons compared."""
    from deep_attention_visual_odometry_amd import _native, native_ops
    from oracle import solver

    kw = dict(iterations=1000, error_threshold=1e-4, minimum_step=1e-8)
    n = x0.shape[0]
    x_g, _, st = native_ops.ba_solve(x0.to(dev), obs[:n].to(dev), vis[:n].to(dev, dtype=torch.uint8), args.views,
                                     args.points, not args.no_distortion, hessian_mode=_native.DAVA_HESSIAN_COMPACT,
                                     want_status=True, **kw)
    x_g, st = x_g.cpu(), st.cpu()
    rec = solver.SolveRecord(iterations=None, reason=None)
    ref = torch.cat([solver.bfgs_solve(x0[lo:lo + 16], closure(lo, min(lo + 16, n)), record=(rec if lo == 0 else None),
                                       **kw) for lo in range(0, n, 16)])
    names = ["f", "cx", "cy"] + (["k1", "k2", "k3", "p1", "p2"] if not args.no_distortion else [])
    cols = list(range(3)) + (list(range(x0.shape[1] - 5, x0.shape[1])) if not args.no_distortion else [])
    per = {}
    for name, c in zip(names, cols):
        r = ((x_g[:, c] - ref[:, c]).abs().double() / ref[:, c].abs().double().clamp(min=1e-30))
        per[name] = {"max_rel": float(r.max()), "frac_le_1e-5": float((r <= PARITY_BAR).double().mean())}
    m = min(n_env, n, 16)
    spread = {k: torch.zeros((m,), dtype=torch.float64) for k, _ in BLOCKS}
    for to in (float("inf"), -float("inf")):
        nudged = solver.bfgs_solve(torch.nextafter(x0[:m], torch.full_like(x0[:m], to)), closure(0, m), **kw)
        for key, sl in BLOCKS:
            spread[key] = torch.maximum(spread[key], _rel(nudged[:, sl], ref[:m, sl]))
    noise = ulp_noise_spread(solver, x0[:m], closure(0, m), kw, ref[:m])
    blocks = {}
    for name, key, sl in (("whole", "x", slice(None)), ("intrinsics", "i", slice(0, 3)), ("distortion", "d", slice(-5, None))):
        if key == "d" and args.no_distortion:
            continue
        r = _rel(x_g[:, sl], ref[:, sl])
        blocks[name] = {"max_rel": float(r.max()), "frac_le_1e-5": float((r <= PARITY_BAR).double().mean()),
                        "over_1ulp_nudge_max": float((r[:m] / spread[key].clamp(min=1e-300)).max()),
                        "over_ulp_noise_max": float((r[:m] / noise[key].clamp(min=1e-300)).max()),
                        "nudge_spread_max": float(spread[key].max()),
                        "noise_spread_max": float(noise[key][torch.isfinite(noise[key])].max())
                        if torch.isfinite(noise[key]).any() else None,
                        "n_noise_runs_nonfinite": int((~torch.isfinite(noise[key])).sum())}
    return {"n": n, "rules": "error_threshold 1e-4, iterations 1000, minimum_step 1e-8 (bfgs_solver.py:53-55)",
            "per_parameter": per, "blocks": blocks, "envelope_problems": m,
            "same_stop_iteration": float((st[:16, 0] == rec.iterations.to(st.dtype)).double().mean()),
            "same_stop_reason": float((st[:16, 1] == rec.reason.to(st.dtype)).double().mean()),
            "mean_iterations": float(st[:, 0].double().mean())}


def _scenes(args, b, first, distortion, ray):
    from deep_attention_visual_odometry_amd import make_scenes

    cache = f"/tmp/dava_scenes_{args.seed}_{first}_{b}_{args.views}_{args.points}_{int(distortion)}_{int(ray)}.npz"
    if os.path.exists(cache):  # generation is ~1 ms/problem on the host; cache it for repeated runs
        z = np.load(cache)
        return z["initial"], z["observations"], z["visibility"]
    s = make_scenes(b, args.views, args.points, distortion=distortion, seed=args.seed, first_index=first,
                    ray_angle=ray)
    try:
        np.savez(cache, initial=s.initial, observations=s.observations, visibility=s.visibility)
    except OSError:
        pass
    return s.initial, s.observations, s.visibility


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; measuring {world} ranks", file=sys.stderr)
    launch_test = args.launch_test
    if launch_test:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)

    from deep_attention_visual_odometry_amd.sharding import gather_packed, shard_range

    distortion = not args.no_distortion
    ray = args.residual == "ray_angle"
    if ray and distortion:
        raise SystemExit("--residual ray_angle is pinhole only: add --no-distortion")
    b = args.batch
    first = shard_range(world * b, world, rank).start  # this rank's slab of the global batch
    x0_np, obs_np, vis_np = _scenes(args, b, first, distortion, ray)
    x0_cpu = torch.tensor(x0_np)
    obs_cpu = torch.tensor(obs_np)
    vis_cpu = torch.tensor(vis_np)
    x0 = x0_cpu.to(dev)
    obs = obs_cpu.to(dev)
    vis = vis_cpu.to(dev, dtype=torch.uint8)
    p = x0.shape[1]
    mn = args.views * args.points

    if launch_test:
        def solve():  # identity stub: exercises ranks, slabs and the packed gather only
            return x0.clone(), torch.zeros((b, 4), dtype=torch.int32)

        def sync():
            pass
        plan = None
    else:
        from deep_attention_visual_odometry_amd import _native, native_ops

        residual = _native.DAVA_RESIDUAL_RAY_ANGLE if ray else _native.DAVA_RESIDUAL_SQUARED_REPROJECTION
        mode = _native.DAVA_HESSIAN_DENSE if args.mode == "dense" else _native.DAVA_HESSIAN_COMPACT
        ws_bytes = (native_ops.solve_workspace_bytes(b, args.views, args.points, distortion, mode, args.iterations)
                    if args.entry == "op" else 0)  # the module allocates its own
        workspace = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        plan = native_ops.solve_plan(b, args.views, args.points, distortion, mode, args.iterations, residual)

        def solve():
            x, _, status = native_ops.ba_solve(x0, obs, vis, args.views, args.points, distortion,
                                               iterations=args.iterations, error_threshold=args.error_threshold,
                                               minimum_step=args.minimum_step, hessian_mode=mode,
                                               want_status=True, workspace=workspace, residual=residual)
            return x, status

        if args.entry == "module":  # the drop-in module exactly as a caller uses it
            from deep_attention_visual_odometry_amd import BFGSSolver, RayAngleError, ReprojectionError

            fn = (RayAngleError(obs, vis, args.views, args.points) if ray else
                  ReprojectionError(obs, vis, args.views, args.points, distortion))
            module = BFGSSolver(error_threshold=args.error_threshold, iterations=args.iterations,
                                minimum_step=args.minimum_step).eval()
            chosen = module._resolve_mode(args.iterations, p, b, dev)
            plan = native_ops.solve_plan(b, args.views, args.points, distortion, chosen, args.iterations, residual)
            plan["module_hessian_mode"] = "dense" if chosen == _native.DAVA_HESSIAN_DENSE else "compact"
            args.mode = plan["module_hessian_mode"]

            def solve():  # noqa: F811
                x = module(x0, fn)
                return x, module.last_status

        if args.entry == "closure":  # the reference's unchanged caller: a torch closure, the generic loop
            if not ray or distortion:
                raise SystemExit("--entry closure is CalibrationNetwork's ray-angle error: add --residual ray_angle "
                                 "--no-distortion")
            from deep_attention_visual_odometry_amd import BFGSSolver
            from deep_attention_visual_odometry_amd.geometry import calibration_network_error

            fn = calibration_network_error(obs, vis.to(obs.dtype), args.views, args.points)
            module = BFGSSolver(error_threshold=args.error_threshold, iterations=args.iterations,
                                minimum_step=args.minimum_step).eval()

            def solve():  # noqa: F811
                return module(x0, fn), torch.zeros((b, 4), dtype=torch.int32, device=dev)

        if args.differentiate:  # recording solve + adjoint, each timed with its own events
            cot = torch.randn(x0.shape, generator=torch.Generator().manual_seed(1)).to(dev)
            phase_ms = []

            def solve():  # noqa: F811
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                x, status, tape = torch.ops.dava.ba_solve_record(
                    x0, obs, vis, args.views, args.points, distortion, 1e-4, 0.9, args.error_threshold,
                    args.iterations, args.minimum_step, 1000, True, residual)
                ev[1].record()
                gx, gobs = torch.ops.dava.ba_solve_backward(cot, tape, status, obs, vis, args.views, args.points,
                                                            distortion, args.iterations, residual, True)
                ev[2].record()
                phase_ms.append(ev)
                solve.grads = (gx, gobs)
                return x, status

        def sync():
            torch.cuda.synchronize(dev)

    # HIP events on the stream the solve is launched on (native_ops launches on torch's current stream); at
    # N > 1 a third event after the all-gather (the current stream waits for RCCL's stream there) splits each
    # step into the rank's own solve and the collective
    stream = None if launch_test else torch.cuda.current_stream(dev)
    kernel_ms, gather_ms = [], []

    def step(timed: bool):
        if timed and stream is not None:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(stream)
        t_solve = time.perf_counter()
        x, status = solve()
        if timed and stream is not None:
            ev[1].record(stream)
            kernel_ms.append((ev[0], ev[1]))
        t_gather = time.perf_counter()
        gathered = gather_packed(x, status, world * b) if world > 1 else None  # the one collective
        if timed:
            if stream is not None:
                ev[2].record(stream)
                gather_ms.append((ev[1], ev[2]))
            else:  # launch test on CPU: host clocks
                t_end = time.perf_counter()
                kernel_ms.append((t_gather - t_solve) * 1e3)
                gather_ms.append((t_end - t_gather) * 1e3)
        return x, status, gathered

    for _ in range(args.warmup):
        step(False)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    if not launch_test:
        torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x, status, gathered = step(True)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ranks = per_rank_phases(kernel_ms, gather_ms, world, dev) if world > 1 else None
    peak_bytes = None if launch_test else int(torch.cuda.max_memory_allocated(dev))
    sustained = None
    if args.sustain_seconds > 0 and not launch_test and not args.differentiate and args.entry != "closure":
        sustained = sustain(args, solve, sync, elapsed / args.steps, world, b, dev)

    if gathered is not None:  # diagnostics over the whole global batch
        x_all, st = gathered[0].cpu(), gathered[1].cpu()
    else:
        x_all, st = x.cpu(), status.cpu()
    finite = bool(torch.isfinite(x_all).all().item())

    if rank == 0:
        value = world * b * args.steps / elapsed
        base = {"metric": None, "value": round(value, 2), "unit": "problems/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None}
        if launch_test:
            base.update({"metric": "LAUNCH TEST (identity stub on CPU, gloo) -- not a measurement",
                         "config": {"global_batch": world * b, "gathered_rows": int(x_all.shape[0]),
                                    "gathered_matches_inputs": bool(torch.equal(
                                        x_all[first: first + b], x0_cpu)) if world == 1 else None,
                                    "parallelism": f"dp{world}"}})
            if world > 1:  # rank 0 regenerates every slab and checks global problem order
                want = [torch.tensor(_scenes(args, shard_range(world * b, world, r).size,
                                             shard_range(world * b, world, r).start, distortion, ray)[0])
                        for r in range(world)]
                base["config"]["gathered_matches_inputs"] = bool(torch.equal(x_all, torch.cat(want)))
                base["per_rank"] = ranks
                base["spot_check"] = {"rows": min(4, b), "identity_stub_rows_equal_inputs": bool(
                    torch.equal(x_all[: min(4, b)], x0_cpu[: min(4, b)]))}
            print(json.dumps(base), flush=True)
        elif args.differentiate:
            print(json.dumps(differentiate_line(args, base, world, b, p, distortion, ray, phase_ms[-args.steps:],
                                                st, finite, solve.grads)), flush=True)
        elif args.entry == "closure":
            print(json.dumps(closure_line(args, base, world, b, p, x0, obs, vis, x, module, peak_bytes, finite)),
                  flush=True)
        else:
            line = measurement_line(args, base, world, b, p, mn, distortion, ray, plan, kernel_ms, st, finite, x0_cpu,
                                    obs_cpu, vis_cpu, x)
            if sustained is not None:
                sustained["ratio_to_value"] = round(sustained["value"] / value, 4)
                line["sustained"] = sustained
            if world > 1:
                line["per_rank"] = ranks
                line["spot_check"] = spot_check(args, x0_cpu, obs_cpu, vis_cpu, x_all, distortion, ray)
            print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def sustain(args, solve, sync, step_s, world, b, dev):
    """The same solve, back to back for about --sustain-seconds after the timed region (no collective: each
    rank's own slab), bracketed like the timed region (sync + barrier, max over ranks).  The step count is
    fixed from the timed region's step time, so every rank runs the same number."""
    n = max(1, int(round(args.sustain_seconds / max(step_s, 1e-6))))
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        solve()
    sync()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = tt.item()
    return {"seconds": round(t, 3), "steps": n, "value": round(world * b * n / t, 2), "unit": "problems/s",
            "note": "the timed step repeated back to back after the timed region (rank-local solves, no gather); "
                    "steady-state clocks and power, not the headline value"}


def _config_argv(args):
    """This configuration's flags, for a child bench process that must run the same workload."""
    out = ["--batch", str(args.batch), "--views", str(args.views), "--points", str(args.points),
           "--iterations", str(args.iterations), "--mode", args.mode, "--residual", args.residual,
           "--seed", str(args.seed), "--error-threshold", str(args.error_threshold),
           "--minimum-step", str(args.minimum_step)]
    return out + (["--no-distortion"] if args.no_distortion else [])


def _child_argv(args):
    """The command line of a counter-pass child: ONE launch of this configuration, no warm-up, no CPU oracle, no
    counter passes or sustained phase of its own (a 10 s phase under rocprofv3 --pmc would profile ~300 launches)."""
    return [sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "0", "--cpu-sample", "0",
            "--no-live-counters", "--sustain-seconds", "0"] + _config_argv(args)


def live_traffic(args, kernel="bfgs_ba_solve_kernel"):
    """HBM (fabric) bytes per launch of the solve kernel, measured in THIS run: two rocprofv3 --pmc passes
    (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass) over a child bench process that runs one launch of
    the same configuration, started after the timed region (a child process; nothing here is exec'd).
    Corrected as MI355X_MICROARCH.md's HBM section prescribes: read = 2 x FETCH_SIZE (gfx950 tallies a
    16 B/lane streaming read at half its bytes), write = WRITE_SIZE, KiB -> bytes.  None (with the reason)
    if rocprofv3 is unavailable or a pass fails."""
    import csv
    import shutil
    import tempfile

    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if prof is None:
        return None, "rocprofv3 not found"
    vals = {}
    with tempfile.TemporaryDirectory(prefix="dava_pmc_", dir="/tmp") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "-d", out, "-o", "p", "--output-format", "csv", "--"] + _child_argv(args)
            env = dict(os.environ, TMPDIR="/tmp")
            try:
                r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=180)
            except subprocess.TimeoutExpired:
                return None, f"{counter} pass timed out"
            if r.returncode != 0:
                return None, f"{counter} pass exited {r.returncode}: {r.stderr[-300:]}"
            rows = []
            for root, _, files in os.walk(out):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        with open(os.path.join(root, f)) as fh:
                            rows += [row for row in csv.DictReader(fh)
                                     if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter]
            if not rows:
                return None, f"{counter}: no {kernel} rows in the counter output"
            vals[counter] = sum(float(row["Counter_Value"]) for row in rows) / len(rows)
    return 2.0 * 1024.0 * vals["FETCH_SIZE"] + 1024.0 * vals["WRITE_SIZE"], vals


def live_ceiling(p):
    """The headline's history stream alone (tools/micro/solve_pass_stream P ceiling: the solve's own LDS-mode
    history pass over C3's rows, B = 8192, 6 LDS-resident entries, every resident problem streaming all the
    time), run as a child process after the timed region: the rate this access pattern reaches with no
    objective evaluation beside it.  Returns (ms, GB/s of history rows) or None."""
    exe = os.path.join(REPO, "tools", "micro", "solve_pass_stream")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe, str(p), "ceiling"], capture_output=True, text=True, timeout=120)
    except subprocess.TimeoutExpired:
        return None
    for line in r.stdout.splitlines():
        if "B= 8192" in line and "ms" in line:
            ms = float(line.split(":")[-1].split("ms")[0])
            gbs = float(line.split("ms")[1].split("GB/s")[0])
            return ms, gbs
    return None


GOLDEN_C5 = os.path.join(REPO, "tests", "golden", "c5_traj.npz")


def golden_parity(args, x0_cpu, x):
    """C5 (16 views x 4096 points): the CPU oracle is the reference's dense P x P algorithm, ~5 min per
    problem at K = 100, so the line compares instead with the REAL reference's own results for its first
    two problems (tests/golden/c5_traj.npz: bench.py's default seed, K = 20 and 100, with the runs from x0
    nudged one ulp up and down, whose spread is the reference's own sensitivity).  None for other configs."""
    if (args.views, args.points, args.no_distortion, args.residual) != (16, 4096, True, "reprojection") \
            or not os.path.exists(GOLDEN_C5):
        return None
    g = np.load(GOLDEN_C5)
    key = f"k{args.iterations}"
    n = g["x0"].shape[0]
    if key not in g.files or not np.array_equal(g["x0"], x0_cpu[:n].numpy()):
        return None
    ref = torch.tensor(g[key])
    gpu = x[:n].detach().cpu()
    p_end = 3 + 3 * args.points
    out = {"n": n, "bar": PARITY_BAR, "reference": f"tests/golden/c5_traj.npz[{key}] (the real reference, "
           "BFGSSolver(iterations=K, error_threshold=-1, minimum_step=-1).eval(), bfgs_solver.py:80-215)"}
    for name, sl in (("whole", slice(None)), ("intrinsics", slice(0, 3)), ("points", slice(3, p_end)),
                     ("extrinsics", slice(p_end, None))):
        rel = _rel(gpu[:, sl], ref[:, sl])
        spread = torch.maximum(_rel(torch.tensor(g[key + "_up"])[:, sl], ref[:, sl]),
                               _rel(torch.tensor(g[key + "_down"])[:, sl], ref[:, sl]))
        out[name] = {"max_rel": float(rel.max()), "spread_1ulp_max": float(spread.max()),
                     "max_rel_over_1ulp": float((rel / spread.clamp(min=1e-300)).max())}
    out["max_rel"] = out["whole"]["max_rel"]
    out["frac_le_bar"] = float((_rel(gpu, ref) <= PARITY_BAR).double().mean())
    return out


def per_rank_phases(kernel_ms, gather_ms, world, dev):
    """Each rank's mean solve and all-gather time per timed step, collected on every rank (after the timed
    region): the rank-to-rank spread of the solve and the collective's share of the step, which the single
    max-over-ranks wall clock cannot show."""
    def mean_ms(pairs):
        if not pairs:
            return 0.0
        if isinstance(pairs[0], float):
            return float(np.mean(pairs))
        return float(np.mean([a.elapsed_time(b_) for a, b_ in pairs]))

    mine = torch.tensor([mean_ms(kernel_ms), mean_ms(gather_ms)], dtype=torch.float64,
                        device=dev if dev.type == "cuda" else "cpu")
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    solve = [round(float(t[0]), 3) for t in every]
    gather = [round(float(t[1]), 3) for t in every]
    return {"solve_ms": solve, "all_gather_ms": gather,
            "solve_ms_max_over_min": round(max(solve) / max(min(solve), 1e-9), 4),
            "note": "per rank, mean over the timed steps: the rank's own fused solve (HIP events on its launch "
                    "stream) and the packed all-gather after it (event after the collective on the same stream)"}


def spot_check(args, x0_cpu, obs_cpu, vis_cpu, x_all, distortion, ray, rows=4):
    """At N > 1 (no cpu_baseline there): rank 0 solves the first `rows` problems of its own slab with the CPU
    oracle and compares them with the GATHERED result's rows -- after the timed region, so it costs nothing
    measured, and it proves the rows that came back through RCCL are the solved ones in global order."""
    from oracle import objective, solver

    n = min(rows, x0_cpu.shape[0])
    fn = (objective.RayAngleClosure(obs_cpu[:n], vis_cpu[:n], args.views, args.points) if ray else
          objective.ReprojectionClosure(obs_cpu[:n], vis_cpu[:n], args.views, args.points, distortion))
    t = time.perf_counter()
    ref = solver.bfgs_solve(x0_cpu[:n], fn, iterations=args.iterations, error_threshold=args.error_threshold,
                            minimum_step=args.minimum_step)
    rel = _rel(x_all[:n], ref)
    return {"rows": n, "max_rel": float(rel.max()), "frac_le_bar": float((rel <= PARITY_BAR).double().mean()),
            "bar": PARITY_BAR, "oracle_seconds": round(time.perf_counter() - t, 2),
            "note": "rank 0's first rows of the gathered global batch vs the CPU oracle, outside the timed region"}


def adjoint_algorithmic_bytes(p: int, n: int, lds_entries: int = 0) -> float:
    """Minimum HBM bytes of the adjoint kernel for one problem of n steps (csrc/bfgs_adjoint.hip):
    reverse step k reads rows (a_j, g_j), j = k .. n-1, and history rows (s_j, w_j), j < k-1, once each,
    plus x_k, g_k, g_{k-1}, s_{k-1}, w_{k-1} and the final a_k write: Pv floats per row.  The oldest
    `lds_entries` history entries are read once per problem into LDS and never again."""
    pv = (p + 3) // 4 * 4
    lh = min(lds_entries, max(n - 1, 0))
    rows = sum(2 * (n - k) + 2 * max(k - 1 - lh, 0) + 6 for k in range(1, n)) + 2 + 2 * lh
    return 4.0 * pv * rows


def differentiate_line(args, line, world, b, p, distortion, ray, phase_ms, st, finite, grads):
    fwd = float(np.mean([e[0].elapsed_time(e[1]) for e in phase_ms]))
    bwd = float(np.mean([e[1].elapsed_time(e[2]) for e in phase_ms]))
    from deep_attention_visual_odometry_amd import native_ops

    lds_entries = native_ops.adjoint_lds_entries(b, args.views, args.points, distortion, args.iterations,
                                                 1 if ray else 0)
    # the byte model is per recorded step: sum it over each problem's own step count (status word 0), so
    # problems stopped early by --error-threshold / --minimum-step / the drop path are charged what they ran
    counts = torch.bincount(st[:b, 0].long().clamp(min=0)).tolist()
    algo = float(sum(c * adjoint_algorithmic_bytes(p, n, lds_entries) for n, c in enumerate(counts) if c))
    achieved = algo / (bwd * 1e-3) / 1e9
    gx, gobs = grads
    line.update({
        "metric": f"BA problems/sec THROUGH the solve and its gradient (B={b} per GPU, {args.views} views x "
                  f"{args.points} pts{', Brown-Conrady' if distortion else ''}{', ray-angle residual' if ray else ''}, "
                  f"K={args.iterations}; d(w . x_K)/d(x0, observations))",
        "dtype": "f32",
        "data": "synthetic (seeded look-at scenes, x0 = truth + noise), fixed random cotangent w",
        "config": {"workload": f"differentiate: batch={b} per GPU, {args.views}x{args.points}, P={p}, K={args.iterations} "
                               f"fixed iterations, recording solve + adjoint",
                   "global_batch": world * b, "num_parameters": p, "iterations": args.iterations,
                   "parallelism": f"dp{world}"},
        "phases_ms": {"recording_solve": round(fwd, 3), "adjoint": round(bwd, 3)},
        "roofline": {"kernel": "bfgs_ba_adjoint_kernel", "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "byte_model": "adjoint: per reverse step k, rows (a_j, g_j) j >= k and history rows (s_j, w_j) "
                                   "j < k-1 read once + 6 tape/workspace rows; the oldest lds_entries history "
                                   "entries are read once per problem; its dual-number HVP is on top",
                     "lds_entries": lds_entries,
                     "algorithmic_bytes_per_launch": algo, "avg_launch_ms": round(bwd, 3)},
        "cpu_baseline": None,
        "parity": {"note": "gradient parity vs oracle autograd / the reference's goldens: tests/test_gpu_solve_grad.py"},
        "diagnostics": {"all_finite": finite and bool(torch.isfinite(gx).all()) and bool(torch.isfinite(gobs).all()),
                        "mean_steps_per_problem": round(st[:, 0].double().mean().item(), 2)},
    })
    return line


def closure_line(args, line, world, b, p, x0, obs, vis, x, module, peak_bytes, finite):
    """--entry closure: the drop-in BFGSSolver called with the reference's own torch closure (generic loop)."""
    from deep_attention_visual_odometry_amd import _native, native_ops

    hist = getattr(module, "last_generic_history", None)
    # the same problems through the fused kernel (RayAngleError): how far the generic loop's result is from it
    x_f, _, _ = native_ops.ba_solve(x0, obs, vis, args.views, args.points, False, iterations=args.iterations,
                                    error_threshold=args.error_threshold, minimum_step=args.minimum_step,
                                    hessian_mode=_native.DAVA_HESSIAN_COMPACT,
                                    residual=_native.DAVA_RESIDUAL_RAY_ANGLE)
    rel = _rel(x.detach().cpu(), x_f.cpu())
    line.update({
        "metric": f"BA problems/sec through the drop-in BFGSSolver called as CalibrationNetwork calls it: its torch "
                  f"error closure (networks/calibration_network.py:58-67, ray angle), B={b}, {args.views} views x "
                  f"{args.points} pts, K={args.iterations} -- the generic loop, not the headline metric",
        "dtype": "f32",
        "data": "synthetic (seeded look-at scenes, noise-free observations, x0 = truth + noise)",
        "config": {"workload": f"closure: batch={b}, {args.views}x{args.points}, P={p}, K={args.iterations}"
                               f"{' fixed iterations' if args.error_threshold < 0 else ' max, reference stopping rules'}",
                   "global_batch": world * b, "num_parameters": p, "iterations": args.iterations,
                   "parallelism": f"dp{world}"},
        "generic_inverse_hessian": "compact history (dava_bfgs_compact_direction)" if hist is not None else
                                   "dense (B, P, P), the reference's data structure",
        "peak_memory_bytes": peak_bytes,
        "history_bytes": hist.nbytes() if hist is not None else None,
        "roofline": None,
        "cpu_baseline": None,
        "parity": {"vs_fused_ray_angle_solve_max_rel": float(rel.max()), "median_rel": float(rel.median()),
                   "note": "the fused RayAngleError solve of the same problems (its parity with the oracle: "
                           "tests/test_gpu_solver.py); the closure's own parity with the oracle: tests/test_gpu_generic.py"},
        "diagnostics": {"all_finite": finite},
    })
    return line


def status_percentiles(st):
    """Per-problem distribution of the status words (steps, objective evaluations, line-search trials): a launch of
    one workgroup per problem lasts as long as its slowest problems, so the tail matters beside the mean."""
    out = {}
    for col, name in ((0, "steps"), (2, "evaluations"), (3, "trials")):
        v = st[:, col].double()
        q = torch.quantile(v, torch.tensor([0.5, 0.9, 0.99], dtype=torch.float64)).tolist()
        out[name] = {"mean": round(v.mean().item(), 2), "p50": q[0], "p90": q[1], "p99": q[2], "max": v.max().item()}
    return out


def measurement_line(args, line, world, b, p, mn, distortion, ray, plan, kernel_ms, st, finite, x0_cpu, obs_cpu,
                     vis_cpu, x):
    fixed_k = args.error_threshold < 0 and args.minimum_step < 0  # every problem runs exactly K iterations
    headline = fixed_k and (b, args.views, args.points, distortion, ray, args.iterations) == (8192, 4, 256, True,
                                                                                               False, 100)
    launch_ms = float(np.mean([a.elapsed_time(b_) for a, b_ in kernel_ms]))
    evals = st[:, 2].double().mean().item() / max(args.iterations, 1)
    trials = st[:, 3].double().mean().item() / max(args.iterations, 1)
    dense_bytes = b * dense_algorithmic_bytes(p, mn, args.iterations)
    if args.mode == "dense":
        algo, model = dense_bytes, "dense: 8 P^2 per problem-iteration (read + write of H, k >= 3) + scene + x"
    else:
        algo = b * compact_algorithmic_bytes(p, mn, args.iterations, plan["lds_history_entries"])
        model = (f"compact: 8 (k-1) Pv per problem-iteration (one read of each HBM history row) + 8 Pv appends, "
                 f"the oldest {plan['lds_history_entries']} entries LDS-resident (0 bytes) + scene + x")
    scene_once = None
    if plan and plan.get("global_vectors"):
        # global-vector mode (C5): the scene (9 MN B per problem: 590 KB at C5) does not fit on-chip beside the
        # O(P) image, so every objective evaluation reads it again -- SURVEY 8(d): "Scene data is counted once
        # per solve if staged in LDS/L2. Report both the 'minimal' count (scene once) and the per-evaluation
        # count."  The per-evaluation count (evaluations from status word 2) is the algorithmic figure here; the
        # minimal count is kept beside it.
        scene_once = algo
        algo = algo - b * 9.0 * mn + float(st[:b, 2].double().sum()) * 9.0 * mn
        model += ("; global-vector mode: the scene is not staged on-chip, so it is counted per objective "
                  "evaluation (9 MN B x the evaluations in status word 2), SURVEY 8(d)")
    roofline = None
    if fixed_k:
        achieved = algo / (launch_ms * 1e-3) / 1e9
        traffic, source = None, None
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
                source = (f"cached: profiles/pmc_traffic.json[{key}] (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, "
                          f"tag {tj[key].get('tag')}, {tj[key].get('date', 'round 1')}), not measured in this run")
        except (OSError, ValueError, KeyError):
            traffic = None
        roofline = {"kernel": "bfgs_ba_solve_kernel", "bound": "hbm", "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_source": source, "byte_model": model,
                    "algorithmic_bytes_per_launch": algo, "avg_launch_ms": round(launch_ms, 3),
                    "frac_of_measured_copy_ceiling": round(achieved / HBM_COPY_GBS, 4),
                    "bytes_note": ("achieved and traffic count bytes that miss L2 (the fabric side: HBM plus the "
                                   "256 MiB Infinity Cache, whose hits FETCH_SIZE includes, MI355X_MICROARCH.md HBM "
                                   "section); the history the resident problems re-read every iteration can be "
                                   "IC-resident, so achieved may exceed the 6.29 TB/s measured HBM copy ceiling")}
        if scene_once is not None:
            roofline["scene_once_model"] = {
                "bytes_per_launch": scene_once, "GBps": round(scene_once / (launch_ms * 1e-3) / 1e9, 1),
                "frac": round(scene_once / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "note": "SURVEY 8(d)'s 'minimal' count: the scene read once per solve, as if it stayed on-chip"}
        if args.mode != "dense":
            roofline["dense_model_equivalent"] = {
                "bytes_per_launch": dense_bytes,
                "GBps": round(dense_bytes / (launch_ms * 1e-3) / 1e9, 1),
                "note": "the reference's dense P x P inverse Hessian would have to move these bytes; the compact "
                        "history is exact BFGS (same rank-2 terms, different rounding), so this is an "
                        "algorithmic saving, not skipped work"}
    cpu, parity = (cpu_baseline(args, x0_cpu, obs_cpu, vis_cpu, x) if (world == 1 and args.cpu_sample > 0)
                   else (None, None))
    if parity is None and fixed_k:
        parity = golden_parity(args, x0_cpu, x)
    if roofline is not None and world == 1 and not args.no_live_counters:
        measured, detail = live_traffic(args)
        if measured is not None:
            roofline["traffic"] = measured
            roofline["traffic_source"] = ("measured in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE "
                                          "passes (child processes, one launch of this configuration each, after "
                                          "the timed region); read = 2 x FETCH_SIZE, write = WRITE_SIZE "
                                          f"(KiB: {detail})")
            roofline["traffic_over_algorithmic"] = round(measured / algo, 4)
        else:
            roofline["traffic_live_failed"] = detail
        if headline and args.mode == "compact":
            ceil = live_ceiling(p)
            if ceil is not None:
                roofline["measured_ceiling"] = {
                    "ms": ceil[0], "GBps_history_reads": ceil[1],
                    "frac_of_measured_ceiling": round(ceil[0] / launch_ms, 4),
                    "source": "tools/micro/solve_pass_stream 794 ceiling (best of 8 launches), run in this session after the timed "
                              "region: the solve's own history pass over the same rows (B = 8192, 6 LDS-resident "
                              "entries, 512 problems resident), nothing else on the CU; frac = its time / the "
                              "solve's launch time"}
    line.update({
        "metric": f"BA problems/sec (B={b} per GPU, {args.views} views x {args.points} pts"
                  f"{', Brown-Conrady' if distortion else ''}{', ray-angle residual' if ray else ''}, "
                  f"K={args.iterations} BFGS iterations{'' if fixed_k else ' max, reference stopping rules'})",
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
            "parallelism": f"dp{world} (problem sharding, one RCCL all-gather of packed x + status)",
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity": parity,
        "diagnostics": {"objective_evals_per_iteration": round(evals, 3),
                        "line_search_trials_per_iteration": round(trials, 3),
                        "mean_steps_per_problem": round(st[:, 0].double().mean().item(), 2),
                        "per_problem": status_percentiles(st),
                        "problems_in_diagnostics": int(st.shape[0]),
                        "all_finite": finite, "plan": plan},
    })
    return line


if __name__ == "__main__":
    main()
