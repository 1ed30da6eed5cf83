#!/bin/bash
# wave priority (s_setprio): high outside the history stream (e1..e3 = level), interleaved A/B
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
A="c3:"; for v in e1 e2 e3; do A="$A c3$v:DAVA_LIB=$V/var_$v/libdava_ba.so"; done
tools/ab_env.sh $A || exit 1
tools/ab_env.sh $A || exit 1
B="c2:"; for v in e1 e2 e3; do B="$B c2$v:DAVA_LIB=$V/var_$v/libdava_ba.so"; done
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" tools/ab_env.sh $B || exit 1
BENCH_ARGS="--steps 1 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" \
  tools/ab_env.sh "c5:" "c5e2:DAVA_LIB=$V/var_e2/libdava_ba.so" || exit 1
