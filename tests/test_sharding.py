"""Multi-process (gloo, world_size 2) tests of the problem-sharding path on CPU.

The per-rank solve is the CPU oracle here (the GPU solve is covered by the
-m gpu tests); what is under test is the partitioning, the per-rank scene
generation (no scatter) and the single all-gather that reassembles results
in global problem order.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deep_attention_visual_odometry_amd.sharding import gather_rows, shard_range, solve_sharded


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, global_batch, results):
    import sys

    sys.path[:0] = [os.environ["DAVA_TEST_REPO"], os.path.join(os.environ["DAVA_TEST_REPO"],
                                                               "deep-attention-visual-odometry_amd")]
    from deep_attention_visual_odometry_amd import make_scenes
    from oracle import objective, solver

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)

    def solve_slab(shard):
        s = make_scenes(shard.size, 2, 16, seed=5, first_index=shard.start)
        fn = objective.ReprojectionClosure(torch.tensor(s.observations), torch.tensor(s.visibility), 2, 16)
        rec = solver.SolveRecord(None, None)
        x = solver.bfgs_solve(torch.tensor(s.initial), fn, iterations=5, error_threshold=-1.0, minimum_step=-1.0,
                              record=rec)
        status = torch.stack([rec.iterations, rec.reason, torch.zeros_like(rec.iterations),
                              torch.full_like(rec.iterations, shard.start)], dim=-1).to(torch.int32)
        return x, status

    x, status = solve_sharded(solve_slab, global_batch)
    if rank == 0:
        results.put((x, status))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("global_batch", [6, 7])
def test_two_rank_solve_matches_single_process(global_batch):
    from deep_attention_visual_odometry_amd import make_scenes
    from oracle import objective, solver

    os.environ["DAVA_TEST_REPO"] = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, global_batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    x, status = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    s = make_scenes(global_batch, 2, 16, seed=5)
    fn = objective.ReprojectionClosure(torch.tensor(s.observations), torch.tensor(s.visibility), 2, 16)
    ref = solver.bfgs_solve(torch.tensor(s.initial), fn, iterations=5, error_threshold=-1.0, minimum_step=-1.0)
    assert x.shape == ref.shape
    assert torch.allclose(x, ref, rtol=1e-6, atol=1e-6)
    assert (status[:, 0] == 5).all()
    first = [shard_range(global_batch, 2, r).start for r in range(2)]
    assert status[:, 3].tolist() == [first[0]] * shard_range(global_batch, 2, 0).size + \
        [first[1]] * shard_range(global_batch, 2, 1).size


def test_shard_ranges_cover_batch_exactly():
    for b in (0, 1, 7, 8192, 65536, 65537):
        for w in (1, 2, 3, 8):
            shards = [shard_range(b, w, r) for r in range(w)]
            assert shards[0].start == 0 and shards[-1].stop == b
            assert all(shards[i].stop == shards[i + 1].start for i in range(w - 1))
            assert max(s.size for s in shards) - min(s.size for s in shards) <= 1
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)


def test_scene_slabs_equal_global_generation():
    """A rank generating only its slab gets exactly the rows of the global batch (no scatter needed)."""
    from deep_attention_visual_odometry_amd import make_scenes

    full = make_scenes(10, 2, 16, seed=9)
    part = make_scenes(4, 2, 16, seed=9, first_index=3)
    assert (part.initial == full.initial[3:7]).all()
    assert (part.observations == full.observations[3:7]).all()


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts two ranks itself (torch.distributed.run
    children, spawned before any device call) and rank 0 reports the global job.  --launch-test swaps
    the solve for an identity stub on CPU/gloo, so this checks the launch, the per-rank slabs and the
    single packed all-gather (rank 0 regenerates every slab and compares the gathered rows)."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--launch-test",
                          "--batch", "5", "--views", "2", "--points", "8", "--steps", "2", "--warmup", "1",
                          "--seed", "77"], capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 10
    assert line["config"]["gathered_rows"] == 10
    assert line["config"]["gathered_matches_inputs"] is True
    # the N > 1 line splits each rank's step into its own solve and the all-gather, and rank 0 spot-checks
    # rows of the gathered batch (against the identity stub's inputs here, the oracle on the GPU)
    ranks = line["per_rank"]
    assert len(ranks["solve_ms"]) == 2 and len(ranks["all_gather_ms"]) == 2
    assert all(t >= 0 for t in ranks["solve_ms"] + ranks["all_gather_ms"])
    assert line["spot_check"]["identity_stub_rows_equal_inputs"] is True


def test_packed_gather_round_trips_status_bits():
    """x and the int32 status words share one float32 buffer; bit patterns that are NaNs or
    denormals as floats must come back unchanged."""
    from deep_attention_visual_odometry_amd.sharding import gather_packed

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        x = torch.randn(3, 5)
        status = torch.tensor([[0, 1, -1, 0x7FC00001], [2, 7, 123456, 1], [2147483647, -2147483648, 5, 3]],
                              dtype=torch.int32)
        gx, gs = gather_packed(x, status, 3)
        assert torch.equal(gx, x) and torch.equal(gs, status)
    finally:
        dist.destroy_process_group()
