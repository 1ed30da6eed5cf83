"""BASELINE configuration C4 -- the 8-GPU global batch (B = 65536, 4 views x 256 points, pinhole +
Brown-Conrady, fp32, K = 100) -- on the HIP path of one GPU.

SURVEY.md 8(e): the problems are independent, so the 8 ranks each generate and solve a contiguous slab
(`sharding.shard_range`) and one all-gather joins the results.  Here the 8 slabs are generated the way
the ranks would generate them (`make_scenes(first_index=shard.start)`, one process per slab), the whole
global batch is solved by ONE fused launch (bfgs_solver.py:80-215 semantics), and:
  * slab generation is the global generation (windows across every slab boundary, and rows checked
    against a direct generation of their global index);
  * every problem is finite, ran its 100 steps, and ends below its starting objective;
  * two problems of each slab match the oracle at K = 100 (per problem <= 1e-5 and inside the
    reference's own 1-ulp envelope, per block);
  * solving a slab on its own is bitwise the global launch's rows (sharding changes nothing);
  * `sharding.gather_packed` runs on the device under an `nccl` (RCCL) process group of world size 1
    and returns the parameters and status words bit for bit.
"""
import concurrent.futures as cf
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

from conftest import SRC

pytestmark = pytest.mark.gpu

GLOBAL_B, WORLD, M, N, K = 65536, 8, 4, 256, 100
SEED = 20251015 + 4000
TOL = 1e-5


def _slab(rank):
    """One rank's slab, generated in a fresh process exactly as that rank would."""
    import sys

    if SRC not in sys.path:
        sys.path.insert(0, SRC)
    from deep_attention_visual_odometry_amd import make_scenes
    from deep_attention_visual_odometry_amd.sharding import shard_range

    sh = shard_range(GLOBAL_B, WORLD, rank)
    s = make_scenes(sh.size, M, N, distortion=True, seed=SEED, first_index=sh.start)
    return rank, s.initial, s.observations, s.visibility.astype(np.uint8)


_C4 = {}


def _global_batch():
    if not _C4:
        x0 = np.empty((GLOBAL_B, 3 + 3 * N + 6 * (M - 1) + 5), np.float32)
        obs = np.empty((GLOBAL_B, M, N, 2), np.float32)
        vis = np.empty((GLOBAL_B, M, N), np.uint8)
        from deep_attention_visual_odometry_amd.sharding import shard_range

        # child processes are started fresh (spawn), never forked from this GPU process
        with cf.ProcessPoolExecutor(max_workers=WORLD, mp_context=mp.get_context("spawn")) as pool:
            for rank, a, b, c in pool.map(_slab, range(WORLD)):
                sh = shard_range(GLOBAL_B, WORLD, rank)
                x0[sh.start:sh.stop], obs[sh.start:sh.stop], vis[sh.start:sh.stop] = a, b, c
        _C4.update(x0=x0, obs=obs, vis=vis)
    return _C4


def test_c4_slabs_are_the_global_generation():
    from deep_attention_visual_odometry_amd import make_scenes
    from deep_attention_visual_odometry_amd.sharding import shard_range

    g = _global_batch()
    for rank in range(1, WORLD):  # a window across every slab boundary, generated in one call
        start = shard_range(GLOBAL_B, WORLD, rank).start - 2
        w = make_scenes(4, M, N, distortion=True, seed=SEED, first_index=start)
        assert np.array_equal(w.initial, g["x0"][start:start + 4])
        assert np.array_equal(w.observations, g["obs"][start:start + 4])
        assert np.array_equal(w.visibility.astype(np.uint8), g["vis"][start:start + 4])
    for i in (0, 12345, GLOBAL_B - 1):
        one = make_scenes(1, M, N, distortion=True, seed=SEED, first_index=i)
        assert np.array_equal(one.initial[0], g["x0"][i])


def _spot_rows():
    from deep_attention_visual_odometry_amd.sharding import shard_range

    rows = []
    for rank in range(WORLD):
        sh = shard_range(GLOBAL_B, WORLD, rank)
        rows += [sh.start + 17 * rank % sh.size, sh.stop - 1 - rank]
    return rows


def test_c4_global_batch_on_one_gpu(device):
    from oracle import objective, solver
    from test_gpu_solver import _envelopes, _rel, _report

    from deep_attention_visual_odometry_amd import native_ops
    from deep_attention_visual_odometry_amd.sharding import shard_range

    g = _global_batch()
    x0 = torch.from_numpy(g["x0"]).to(device)
    obs = torch.from_numpy(g["obs"]).to(device)
    vis = torch.from_numpy(g["vis"]).to(device)
    kw = dict(iterations=K, error_threshold=-1.0, minimum_step=-1.0)
    x, err, status = native_ops.ba_solve(x0, obs, vis, M, N, True, hessian_mode=1, want_error=True,
                                         want_status=True, **kw)
    e0, _, _ = native_ops.ba_evaluate(x0, obs, vis, M, N, True, want_grad=False)
    assert torch.isfinite(x).all() and torch.isfinite(err).all()
    assert (status[:, 0] == K).all() and (status[:, 1] == 0).all()
    assert (err <= e0).all()

    # a slab solved on its own (what one rank runs) is bitwise the global launch's rows
    for rank in (0, WORLD - 1):
        sh = shard_range(GLOBAL_B, WORLD, rank)
        xs, _, ss = native_ops.ba_solve(x0[sh.start:sh.stop], obs[sh.start:sh.stop], vis[sh.start:sh.stop], M, N,
                                        True, hessian_mode=1, want_status=True, **kw)
        assert torch.equal(xs, x[sh.start:sh.stop]) and torch.equal(ss, status[sh.start:sh.stop])

    # two problems of every slab against the oracle (the reference algorithm, bitwise pinned)
    rows = _spot_rows()
    xr = torch.from_numpy(g["x0"][rows])
    ob, vb = torch.from_numpy(g["obs"][rows]), torch.from_numpy(g["vis"][rows]).bool()
    fn = objective.ReprojectionClosure(ob, vb, M, N, True)
    ref = solver.bfgs_solve(xr, fn, **kw)
    env, env_i, env_d = _envelopes(xr, fn, ref, distortion=True, **kw)
    out = x[rows].cpu()
    rel, rel_i, rel_d = _rel(out, ref), _rel(out[:, :3], ref[:, :3]), _rel(out[:, -5:], ref[:, -5:])
    _report("c4_B65536_one_gpu_spot16", rel, env,
            {"intrinsics_max_rel": float(rel_i.max()), "distortion_max_rel": float(rel_d.max()),
             "distortion_max_rel_over_envelope": float((rel_d / env_d).max())})
    assert (rel <= TOL).all() and (rel <= env).all(), rel
    assert (rel_i <= env_i).all(), rel_i
    assert (rel_d <= env_d).all(), (rel_d, env_d)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c4_gather_packed_under_rccl(device):
    """The all-gather of bench.py --gpus N (sharding.gather_packed) on the device, nccl backend (RCCL),
    world size 1: the packed (B, P + 4) buffer -- parameters plus bit-cast status words -- comes back
    bit for bit, NaN payloads and negative status words included."""
    import torch.distributed as dist

    from deep_attention_visual_odometry_amd.sharding import gather_packed

    p = 3 + 3 * N + 6 * (M - 1) + 5
    gen = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(GLOBAL_B, p, generator=gen).to(device)
    x[5, 7] = float("nan")
    status = torch.randint(-5, 1 << 20, (GLOBAL_B, 4), generator=gen, dtype=torch.int32).to(device)
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=device)
    try:
        assert dist.get_backend() == "nccl"
        xg, sg = gather_packed(x, status, GLOBAL_B)
        torch.cuda.synchronize(device)
        assert xg.device == x.device and xg.dtype == torch.float32 and sg.dtype == torch.int32
        assert torch.equal(xg.view(torch.int32), x.view(torch.int32))  # bitwise, NaN included
        assert torch.equal(sg, status)
    finally:
        if own:
            dist.destroy_process_group()
