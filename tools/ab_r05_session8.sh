#!/bin/bash
# r05 session 8: the dense sweep software-pipelined through buffer loads / stores (DAVA_SWEEP_PIPE=1,
# the in-tree build) against the predicated form (build/var_nopipe): bitwise check (C3 dense, C5 dense
# at B = 16, the hybrid at cap 8), then interleaved dense-mode A/B at C3 and C5.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
NEW=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
OLD=deep-attention-visual-odometry_amd/build/var_nopipe/libdava_ba.so
timeout -k 10 300 python3 tools/lib_compare.py $OLD $NEW --mode 0 --batch 2048 || exit 1
timeout -k 10 300 python3 tools/lib_compare.py $OLD $NEW --mode 0 --batch 16 --views 16 --points 4096 --no-distortion --k 20 || exit 1
export BENCH_ARGS="--mode dense --steps 2 --warmup 1 --parity-envelope 0"
tools/ab_env.sh "pipe:" "nopipe:DAVA_LIB=@BUILD@/var_nopipe/libdava_ba.so" "pipe:" "nopipe:DAVA_LIB=@BUILD@/var_nopipe/libdava_ba.so" || exit 1
export BENCH_ARGS="--mode dense --steps 2 --warmup 1 --parity-envelope 0 --batch 256 --views 16 --points 4096 --no-distortion --iterations 20"
tools/ab_env.sh "pipe_c5:" "nopipe_c5:DAVA_LIB=@BUILD@/var_nopipe/libdava_ba.so" "pipe_c5:" "nopipe_c5:DAVA_LIB=@BUILD@/var_nopipe/libdava_ba.so" || exit 1
