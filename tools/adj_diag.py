"""GPU box diagnostic: which backward a create_graph fused solve takes, and its gradient error vs the
oracle, for the C1/C2/C3-shaped cases of tests/test_gpu_solve_grad.py::test_fused_adjoint_matches_oracle.
usage: python tools/adj_diag.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-attention-visual-odometry_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402


def main():
    from deep_attention_visual_odometry_amd import _native as N, make_scenes, native_ops
    from test_gpu_solve_grad import _fused_grads, _oracle_grads, _rows_rel

    print("library", N.LIB_PATH, flush=True)
    dev = torch.device("cuda", 0)
    for m, n, dist, ray, k, b in ((2, 64, False, False, 10, 4), (2, 128, False, False, 20, 4),
                                  (4, 256, False, False, 8, 2)):
        lib = N.load_library()
        sc = native_ops.scene_struct(None, None, m, n, dist, b, 0)
        cfg = native_ops.solver_config(1e-4, 0.9, 1e-4, k, 1e-8, 1000, True, N.DAVA_HESSIAN_COMPACT)
        print("shape", m, n, "tape", int(lib.dava_ba_solve_tape_bytes(sc, cfg)), "bwd ws",
              int(lib.dava_ba_solve_backward_workspace_bytes(sc, cfg)),
              "supported", native_ops.solve_tape_supported(b, m, n, dist, k), flush=True)
        s = make_scenes(b, m, n, distortion=dist, seed=900 + n + k, drop=0.0 if dist else 0.1, ray_angle=ray)
        x0, obs, vis = torch.tensor(s.initial), torch.tensor(s.observations), torch.tensor(s.visibility)
        w = torch.randn(x0.shape, generator=torch.Generator().manual_seed(k))
        kw = dict(iterations=k, error_threshold=-1.0, minimum_step=-1.0)
        ref, gx_ref, go_ref = _oracle_grads(x0, obs, vis, m, n, dist, w, ray, **kw)
        for tag, knob in (("fused", None), ("generic", "GENERIC_BACKWARD")):
            if knob:
                N.set_debug_override(knob, 1)
            out, gx, go, st = _fused_grads(dev, x0, obs, vis, m, n, dist, w, ray, **kw)
            N.clear_debug_overrides()
            print(" ", tag, "x", _rows_rel(out, ref).max().item(), "gx", _rows_rel(gx, gx_ref).tolist(),
                  "go", _rows_rel(go, go_ref).max().item(), flush=True)


if __name__ == "__main__":
    main()
