#!/bin/bash
# Phase attribution of the current default C3 kernel + compute-only (no history) variant
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
tools/ab_env.sh "c3:" "c3nosweep:DAVA_LIB=$V/var_nosweep/libdava_ba.so" "c3lds0:DAVA_LDS_HISTORY=0" || exit 1
DAVA_LIB=$V/var_phase/libdava_ba.so timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 1 --warmup 0 2>&1 | grep -E "phase" | cut -c1-300
