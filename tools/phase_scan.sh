#!/bin/bash
# GPU box: per-phase cycle split of the solve (diagnostic build build/var_phase, DAVA_PHASE_TIMING=1)
# for C2 at B = 64 / 256 / 1024 (and its ray-angle form at 256 / 1024), C3 and C5, with the per-problem
# p50 / p99 / max of every phase; one bench process per case, stderr kept.
# usage: tools/phase_scan.sh > gpurun_out/phase_scan.log
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$R/deep-attention-visual-odometry_amd/build/var_phase/libdava_ba.so
run() {
  echo "== $1"
  shift
  env DAVA_DEBUG_OVERRIDES=1 DAVA_LIB=$LIB timeout -k 10 300 python3 "$R/bench.py" --cpu-sample 0 --no-live-counters --sustain-seconds 0 --steps 1 --warmup 0 "$@" 2>&1 \
    | grep -E "dava (phase|objective) cycles" || return 1
}
run C2_b64 --batch 64 --views 2 --points 128 --no-distortion &&
run C2_b256 --batch 256 --views 2 --points 128 --no-distortion &&
run C2_b512 --batch 512 --views 2 --points 128 --no-distortion &&
run C2 --batch 1024 --views 2 --points 128 --no-distortion &&
run C2_ray_b256 --batch 256 --views 2 --points 128 --no-distortion --residual ray_angle &&
run C2_ray --batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle &&
run C3 &&
run C5 --batch 256 --views 16 --points 4096 --no-distortion
