#!/bin/bash
# Solver GPU tests + C5 / C3 bench after the GV objective-on-LDS (XL) change
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py tests/test_gpu_objective.py tests/test_gpu_solve_grad.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests4.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests4.log
[ $rc -le 1 ] || exit $rc
BENCH_ARGS="--steps 1 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" tools/ab_env.sh "c5:" || exit 1
tools/ab_env.sh "c3:" || exit 1
