"""Diagnostic (GPU box): the differentiable fused solve through BFGSSolver + autograd, repeated in one
process (with the camera-model kernels in between, as in the test suite); reports runs whose x or
gradients differ bitwise from the first.  usage: python tools/adjoint_repeat_autograd.py [runs]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def main():
    import test_gpu_camera_l1 as L1
    import test_gpu_solve_grad as T
    from deep_attention_visual_odometry_amd import make_scenes

    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ray = len(sys.argv) > 2 and sys.argv[2] == "ray"
    dev = torch.device("cuda", 0)
    m, n, k, b = 2, 64, 10, 4
    s = make_scenes(b, m, n, distortion=False, seed=900 + n + k, drop=0.1, ray_angle=ray)
    x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
    w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(k))
    kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
    l1_tests = [getattr(L1, t) for t in dir(L1) if t.startswith("test_")]
    first, bad = None, 0
    for r in range(runs):
        for t in l1_tests:  # perturb: whatever the preceding tests leave behind
            try:
                t(dev) if t.__code__.co_argcount == 1 else None
            except Exception:
                pass
        out, gx, go, st = T._fused_grads(dev, x0, obs, vis, m, n, False, w, ray, **kw)
        cur = (out, gx, go)
        if first is None:
            first = cur
            continue
        d = [nm for nm, a, c in zip(("x", "gx", "gobs"), first, cur) if not torch.equal(a, c)]
        if d:
            bad += 1
            rows = (first[1] != cur[1]).any(-1).nonzero().flatten().tolist()
            print(f"run {r}: differs in {d}, gradient rows {rows}, "
                  f"max rel {(T._rows_rel(cur[1], first[1])).max().item():.3e}", flush=True)
    print(f"{bad} of {runs - 1} repeats differ", flush=True)


if __name__ == "__main__":
    main()
