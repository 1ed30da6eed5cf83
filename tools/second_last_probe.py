"""Diagnostic (GPU box): return_second_last on the test case of tests/test_gpu_solver.py
(_second_last_case, b=12): which problems the reference scatter moves, and per problem the
distance of the fused solve, the generic loop and the oracle (with and without the scatter)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]
from deep_attention_visual_odometry_amd import BFGSSolver, ReprojectionError, make_scenes, native_ops  # noqa: E402
from oracle import objective, solver  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm(dim=-1) / b.norm(dim=-1)).tolist()


def main():
    dev = torch.device("cuda", 0)
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    s = make_scenes(b, 2, 64, distortion=False, seed=581, drop=0.1)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    kw = dict(iterations=60, error_threshold=-1.0, minimum_step=2e-3)
    fused, _, st = native_ops.ba_solve(x0.to(dev), obs.to(dev), vis.to(dev), 2, 64, False, hessian_mode=1,
                                       want_status=True, return_second_last=True, **kw)
    print("status (steps, reason):", st[:, :2].cpu().tolist())
    print("moves rows:", native_ops.second_last_moves_rows(st))
    fn = ReprojectionError(obs.to(dev), vis.to(dev), 2, 64)
    g = BFGSSolver(drop_path_p=0.0, return_second_last=True, training_iterations=60, training_error_threshold=-1.0,
                   minimum_step=2e-3)
    gen = g._generic(x0.to(dev), fn, -1.0, 60).cpu()
    rec = solver.SolveRecord(torch.empty(0), torch.empty(0))
    ref = solver.bfgs_solve(x0, objective.ReprojectionClosure(obs, vis, 2, 64), training=True, return_second_last=True,
                            drop_path_p=0.0, record=rec, **kw)
    print("oracle (steps, reason):", list(zip(rec.iterations.tolist(), rec.reason.tolist())))
    plain_ref = solver.bfgs_solve(x0, objective.ReprojectionClosure(obs, vis, 2, 64), **kw)
    print("generic vs oracle      :", ["%.1e" % v for v in rel(gen, ref)])
    print("fused   vs oracle      :", ["%.1e" % v for v in rel(fused.cpu(), ref)])
    print("oracle sl vs oracle eval:", ["%.1e" % v for v in rel(ref, plain_ref)])


if __name__ == "__main__":
    main()
