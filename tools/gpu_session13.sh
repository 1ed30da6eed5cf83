#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests13.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/gpu_tests13.log
[ $rc -le 1 ] || exit $rc
tools/ab_env.sh "c3:" "c3noq:DAVA_NO_QUEUE=1" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" tools/ab_env.sh "c2:" "c2noq:DAVA_NO_QUEUE=1" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8" \
  tools/ab_env.sh "c3conv:" "c3convnoq:DAVA_NO_QUEUE=1" || exit 1
