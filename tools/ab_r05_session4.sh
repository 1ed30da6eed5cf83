#!/bin/bash
# r05 session 4: C2 batch scan (wall clock, no profiler) and the per-CU packing question
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for b in 256 512 768 1024; do
  BENCH_ARGS="--batch $b --views 2 --points 128 --no-distortion --steps 5 --warmup 2" tools/ab_env.sh "B$b:" "B${b}_wg2:DAVA_WG_PER_CU=2" "B$b:" || exit 1
done 2>&1 | cut -c1-160 | tee gpurun_out/c2_batch_scan_r05.log
