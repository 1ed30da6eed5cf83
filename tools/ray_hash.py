"""Diagnostic: bitwise fingerprints of x and the gradients of the ray-angle adjoint case (one process)."""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "deep-attention-visual-odometry_amd")]
import torch  # noqa: E402

import test_gpu_solve_grad as T  # noqa: E402
from deep_attention_visual_odometry_amd import make_scenes  # noqa: E402

dev = torch.device("cuda", 0)
m, n, k, b = 2, 64, 10, 4
s = make_scenes(b, m, n, distortion=False, seed=900 + n + k, drop=0.1, ray_angle=True)
x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(k))
kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
out, gx, go, st = T._fused_grads(dev, x0, obs, vis, m, n, False, w, True, **kw)
h = lambda t: hashlib.md5(t.numpy().tobytes()).hexdigest()[:8]  # noqa: E731
print("x", [h(out[i]) for i in range(b)], "gx", [h(gx[i]) for i in range(b)], "status", st[:, 1:].tolist())
