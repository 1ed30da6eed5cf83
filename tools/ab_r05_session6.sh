#!/bin/bash
# r05 session 6: C5 with the problems' start times spread over up to one iteration (~350 us): do the
# per-CU history phases stay in step (all CUs streaming at once at the chip's ~5.4 TB/s for this pattern,
# profiles/r05_micro_wide_pass_stream.log) or spread out?
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
BENCH_ARGS="--batch 256 --views 16 --points 4096 --no-distortion --steps 2 --warmup 1" tools/ab_env.sh \
  "base:" "L2_400k:DAVA_STAGGER=400000 DAVA_STAGGER_LEVELS=2" "L4_200k:DAVA_STAGGER=200000 DAVA_STAGGER_LEVELS=4" \
  "L8_100k:DAVA_STAGGER=100000 DAVA_STAGGER_LEVELS=8" "base:" "L2_400k:DAVA_STAGGER=400000 DAVA_STAGGER_LEVELS=2" \
  2>&1 | cut -c1-110 | tee gpurun_out/ab_c5_spread.log
