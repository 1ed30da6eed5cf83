"""Diagnostic (GPU box): determinism of the recording solve and the adjoint.  Runs the same
differentiable fused solve many times in one process, with unrelated kernels in between, and
reports every run whose tape, x or gradients differ bitwise from the first run's (and where).
usage: python tools/adjoint_repeat.py [--runs 40]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=40)
    ap.add_argument("--batch", type=int, default=4)
    args = ap.parse_args()
    from deep_attention_visual_odometry_amd import make_scenes, native_ops

    dev = torch.device("cuda", 0)
    m, n, k, b = 2, 64, 10, args.batch
    s = make_scenes(b, m, n, distortion=False, seed=900 + n + k, drop=0.1)
    x0 = torch.tensor(s.initial, device=dev)
    obs = torch.tensor(s.observations, device=dev)
    vis = torch.tensor(s.visibility, device=dev).to(torch.uint8)
    w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(k)).to(dev)
    first = None
    bad = 0
    for r in range(args.runs):
        # unrelated work in between: other shapes, other kernels, allocator churn
        junk = torch.randn(int(1e6) + 4096 * r, device=dev)
        s2 = make_scenes(8, 4, 256, distortion=True, seed=r, drop=0.0)
        native_ops.ba_solve(torch.tensor(s2.initial, device=dev), torch.tensor(s2.observations, device=dev),
                            torch.tensor(s2.visibility, device=dev), 4, 256, True, iterations=5, hessian_mode=1)
        del junk
        x, status, tape = torch.ops.dava.ba_solve_record(x0, obs, vis, m, n, False, 1e-4, 0.9, -1.0, k, -1.0, 1000,
                                                         True, 0)
        gx, gobs = torch.ops.dava.ba_solve_backward(w, tape, status, obs, vis, m, n, False, k, 0, True)
        torch.cuda.synchronize(dev)
        cur = (x.cpu(), tape.cpu(), gx.cpu(), gobs.cpu())
        if first is None:
            first = cur
            continue
        diffs = [name for name, a, c in zip(("x", "tape", "gx", "gobs"), first, cur) if not torch.equal(a, c)]
        if diffs:
            bad += 1
            rows = (first[2] != cur[2]).any(-1).nonzero().flatten().tolist()
            tv = first[1].view(torch.float32), cur[1].view(torch.float32)
            where = (tv[0] != tv[1]).nonzero().flatten()[:8].tolist()
            print(f"run {r}: differs in {diffs}; gradient rows {rows}; first tape float offsets {where}", flush=True)
    print(f"{bad} of {args.runs - 1} repeats differ", flush=True)


if __name__ == "__main__":
    main()
