#!/bin/bash
# Solver GPU tests after a solve-kernel change + A/B of the trial-slope variant + C2 + C5 phases.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests3.log
[ $rc -le 1 ] || exit $rc
tools/ab_env.sh "c3:" "c3dot:DAVA_LIB=$V/var_dot/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" tools/ab_env.sh "c2:" || exit 1
echo "== phase C5"
DAVA_LIB=$V/var_phase/libdava_ba.so timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 1 --warmup 0 \
  --batch 256 --views 16 --points 4096 --no-distortion 2>&1 | grep -E "phase|value" | cut -c1-300
