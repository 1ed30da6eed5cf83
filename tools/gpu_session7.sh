#!/bin/bash
# full GPU suite + C3 / C5 bench
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests7.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests7.log
[ $rc -le 1 ] || exit $rc
tools/ab_env.sh "c3:" "c3noppt:DAVA_NO_PPT=1" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" tools/ab_env.sh "c5:" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" tools/ab_env.sh "c2:" || exit 1
