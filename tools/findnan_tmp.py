import sys, os
sys.path[:0]=['/root/repo','/root/repo/deep-attention-visual-odometry_amd']
import torch
from deep_attention_visual_odometry_amd import make_scenes, native_ops
dev=torch.device('cuda',0)
s = make_scenes(256, 4, 256, distortion=True, seed=2024)
x0 = torch.tensor(s.initial).to(dev); obs=torch.tensor(s.observations).to(dev); vis=torch.tensor(s.visibility).to(dev)
out, err, st = native_ops.ba_solve(x0, obs, vis, 4, 256, True, iterations=100, error_threshold=-1.0, minimum_step=-1.0, want_error=True, want_status=True)
bad = (~torch.isfinite(err)).nonzero().squeeze(-1).tolist()
print("nan problems", bad)
print("status", st[bad].tolist())
for k in (10,20,40,60,80):
    o, e, st2 = native_ops.ba_solve(x0, obs, vis, 4, 256, True, iterations=k, error_threshold=-1.0, minimum_step=-1.0, want_error=True, want_status=True)
    print(k, "nan count", (~torch.isfinite(e)).sum().item(), e[bad].tolist())
