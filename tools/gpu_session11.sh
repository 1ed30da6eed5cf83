#!/bin/bash
# paired-view objective sweep: GPU tests + interleaved A/B against the previous build
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py tests/test_gpu_objective.py tests/test_gpu_solve_grad.py \
  -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests11.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests11.log
[ $rc -le 1 ] || exit $rc
tools/ab_env.sh "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" \
  tools/ab_env.sh "c5:" "c5prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" \
  tools/ab_env.sh "c2:" "c2prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
