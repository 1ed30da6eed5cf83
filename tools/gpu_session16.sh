#!/bin/bash
# wave priority (s_setprio) during the history stream vs elsewhere: interleaved A/B
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
A="c3:"; for v in p1 p3 e2; do A="$A c3$v:DAVA_LIB=$V/var_$v/libdava_ba.so"; done
tools/ab_env.sh $A || exit 1
tools/ab_env.sh $A || exit 1
B="c2:"; for v in p1 p3 e2; do B="$B c2$v:DAVA_LIB=$V/var_$v/libdava_ba.so"; done
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" tools/ab_env.sh $B || exit 1
