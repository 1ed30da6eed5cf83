#!/bin/bash
# GPU box: the drop-in BFGSSolver called as CalibrationNetwork calls it (bench.py --entry closure: its torch
# ray-angle closure, the generic loop) with the compact-history inverse Hessian (default) and with the reference's
# dense (B, P, P) matrix (DAVA_GENERIC_DENSE=1), at C2 (B = 1024) and C3 (B = 256), K = 100 fixed.
# One JSON line per run on stdout: {"tag", "inverse_hessian", "line"}.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for cfg in "C2:--batch 1024 --views 2 --points 128" "C3:--batch 256 --views 4 --points 256"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for v in compact dense; do
    e=""; [ $v = dense ] && e="DAVA_DEBUG_OVERRIDES=1 DAVA_GENERIC_DENSE=1"
    line=$(env $e timeout -k 10 600 python3 bench.py --entry closure --residual ray_angle --no-distortion $args \
             --steps 2 --warmup 1 --cpu-sample 0 --no-live-counters --sustain-seconds 0 2>>/dev/stderr | tail -1) \
      || { echo "closure $tag $v failed" >&2; exit 1; }
    echo "{\"tag\": \"$tag\", \"inverse_hessian\": \"$v\", \"line\": $line}"
  done
done
