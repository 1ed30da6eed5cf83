#!/bin/bash
# phi'(0) fused into the direction loop: bitwise check against the previous build + A/B
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 200 python3 tools/dump_solve.py gpurun_out/d_new.npz 2>/dev/null &&
DAVA_LIB=$V/var_prev/libdava_ba.so timeout -k 10 200 python3 tools/dump_solve.py gpurun_out/d_prev.npz 2>/dev/null &&
python3 tools/dump_solve.py --compare gpurun_out/d_new.npz gpurun_out/d_prev.npz || exit 1
tools/ab_env.sh "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" \
  tools/ab_env.sh "c2:" "c2prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
