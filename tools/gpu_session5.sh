#!/bin/bash
# A/B: observation prefetch on/off, C3 and C5, interleaved
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
tools/ab_env.sh "c3pf:" "c3nopf:DAVA_LIB=$V/var_nopf/libdava_ba.so" "c3pf:" "c3nopf:DAVA_LIB=$V/var_nopf/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" tools/ab_env.sh "c5pf:" "c5nopf:DAVA_LIB=$V/var_nopf/libdava_ba.so" || exit 1
