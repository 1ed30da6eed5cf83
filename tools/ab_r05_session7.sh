#!/bin/bash
# r05 session 7: the staged GV pass as a row-slot ring (2 slots = the r04 scheme, rows copied whole
# instead of S/W interleaved per group): bitwise against HEAD's build, and C5 / C3 A/B
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
A=$(pwd)/deep-attention-visual-odometry_amd/build/var_prev/libdava_ba.so
B=$(pwd)/deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
timeout -k 10 300 python3 tools/lib_compare.py $A $B --views 16 --points 4096 --no-distortion --batch 256 > gpurun_out/rows_bitwise.log 2>&1 || { tail -5 gpurun_out/rows_bitwise.log; exit 1; }
tail -1 gpurun_out/rows_bitwise.log
P="prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so"
BENCH_ARGS="--batch 256 --views 16 --points 4096 --no-distortion --steps 2 --warmup 1" tools/ab_env.sh "cur:" "$P" "cur:" "$P" "cur:" "$P" \
  2>&1 | cut -c1-110 | tee gpurun_out/ab_c5_rowslots.log
