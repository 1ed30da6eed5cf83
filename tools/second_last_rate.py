"""GPU box: how often a training-mode return_second_last batch falls back to the generic loop.

The fused kernel runs return_second_last itself unless the reference's scatter (bfgs_solver.py:196-212)
would move rows between problems -- i.e. a problem stops by the minimum-step rule while a later problem of
the batch goes on (native_ops.second_last_moves_rows).  This measures that rate on C2- and C3-shaped
training batches with the reference's training defaults (drop_path_p 0.1, 1000 iterations, error 1e-4,
minimum step 1e-8), per batch size, and prints one JSON line per case.

usage: python tools/second_last_rate.py [--batches 8] > gpurun_out/second_last_rate.jsonl
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deep-attention-visual-odometry_amd"))

import torch  # noqa: E402

from deep_attention_visual_odometry_amd import make_scenes, native_ops  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", type=int, default=8)
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    for name, (m, n, dist) in {"C2": (2, 128, False), "C3": (4, 256, True)}.items():
        for b in (8, 32, 64, 256):
            moved, by_rule = 0, 0.0
            for k in range(args.batches):
                s = make_scenes(b, m, n, distortion=dist, seed=9900 + k, first_index=k * b)
                _, _, st = native_ops.ba_solve(torch.tensor(s.initial, device=dev),
                                               torch.tensor(s.observations, device=dev),
                                               torch.tensor(s.visibility, device=dev), m, n, dist, hessian_mode=1,
                                               want_status=True, return_second_last=True, drop_path_p=0.1,
                                               drop_seed=1234 + k)
                moved += int(native_ops.second_last_moves_rows(st))
                by_rule += float((st[:, 1] == 2).float().mean())
            print(json.dumps({"shape": name, "batch": b, "batches": args.batches,
                              "fallback_rate": moved / args.batches,
                              "mean_frac_stopped_by_minimum_step": by_rule / args.batches}), flush=True)


if __name__ == "__main__":
    main()
