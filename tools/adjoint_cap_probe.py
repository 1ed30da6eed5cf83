"""Diagnostic (GPU box): the adjoint's gradients for one recorded C3 solve, repeated with and without
LDS-held history entries (DAVA_ADJ_LDS_ENTRIES), reporting which rows differ and by how much."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd")]

import torch  # noqa: E402


def main():
    from deep_attention_visual_odometry_amd import make_scenes

    dev = torch.device("cuda", 0)
    m, n, k = 4, 256, int(sys.argv[1]) if len(sys.argv) > 1 else 24
    s = make_scenes(8, m, n, distortion=True, seed=935, drop=0.1)
    x0, obs, vis = (torch.tensor(t).to(dev) for t in (s.initial, s.observations, s.visibility))
    vis = vis.to(torch.uint8)
    w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(5)).to(dev)
    x, status, tape = torch.ops.dava.ba_solve_record(x0, obs, vis, m, n, True, 1e-4, 0.9, -1.0, k, -1.0, 1000, True, 0)
    print("status", status[:, :2].tolist(), flush=True)
    ref = None
    for cap in ["d", "d", "0", "0", "3", "d", "1", "2"]:
        if cap == "d":
            os.environ.pop("DAVA_ADJ_LDS_ENTRIES", None)
        else:
            os.environ["DAVA_ADJ_LDS_ENTRIES"] = cap
        gx, gobs = torch.ops.dava.ba_solve_backward(w, tape, status, obs, vis, m, n, True, k, 0, True)
        torch.cuda.synchronize()
        if ref is None:
            ref = (gx.clone(), gobs.clone())
            continue
        rows = (gx != ref[0]).any(-1).nonzero().flatten().tolist()
        rel = ((gx - ref[0]).norm(dim=-1) / ref[0].norm(dim=-1)).max().item()
        print(f"cap {cap}: rows differing {rows}, max rel {rel:.3e}, obs equal {torch.equal(gobs, ref[1])}", flush=True)


if __name__ == "__main__":
    main()
