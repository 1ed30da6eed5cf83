import os, sys, torch
sys.path[:0] = ['/root/repo', '/root/repo/tests', '/root/repo/deep-attention-visual-odometry_amd']
os.chdir('/root/repo')
import test_gpu_solve_grad as T
from deep_attention_visual_odometry_amd import make_scenes
dev = torch.device('cuda', 0)
m, n, k, b = 2, 64, 10, 4
s = make_scenes(b, m, n, distortion=False, seed=900 + n + k, drop=0.1, ray_angle=True)
x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(k))
kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
ref, gx_ref, go_ref = T._oracle_grads(x0, obs, vis, m, n, False, w, True, **kw)
for stag in ("default", "0", "default", "0"):
    if stag == "0": os.environ["DAVA_STAGGER"] = "0"
    else: os.environ.pop("DAVA_STAGGER", None)
    out, gx, go, st = T._fused_grads(dev, x0, obs, vis, m, n, False, w, True, **kw)
    print(stag, "x", T._rows_rel(out, ref).tolist(), "gx", T._rows_rel(gx, gx_ref).tolist(), flush=True)
