#!/bin/bash
# r05 session 2: GPU suite at the tightened envelope, the GV group-ring variant (bitwise tests under it,
# interleaved C5 A/B), then one bench line per configuration.
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
tools/gpu_run.sh tests || exit 1
RING=$(pwd)/deep-attention-visual-odometry_amd/build/var_ring/libdava_ba.so
env DAVA_DEBUG_OVERRIDES=1 DAVA_LIB=$RING timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lds_staged_history or c5_reference_golden or global_vector or c5_shape" \
  > gpurun_out/tests_ring.log 2>&1 || { tail -20 gpurun_out/tests_ring.log; exit 1; }
tail -1 gpurun_out/tests_ring.log
P="ring:DAVA_LIB=@BUILD@/var_ring/libdava_ba.so"
BENCH_ARGS="--batch 256 --views 16 --points 4096 --no-distortion --steps 2 --warmup 1" tools/ab_env.sh "base:" "$P" "base:" "$P" "base:" "$P" \
  > gpurun_out/ab_c5_ring.log 2>&1 || { tail -3 gpurun_out/ab_c5_ring.log; exit 1; }
cut -c1-100 gpurun_out/ab_c5_ring.log
tools/gpu_run.sh configs || exit 1
echo session2 done
