#!/bin/bash
# work-queue launch: GPU tests + interleaved A/B against one workgroup per problem (DAVA_NO_QUEUE)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests12.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/gpu_tests12.log
[ $rc -le 1 ] || exit $rc
tools/ab_env.sh "c3q:" "c3noq:DAVA_NO_QUEUE=1" "c3q:" "c3noq:DAVA_NO_QUEUE=1" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" \
  tools/ab_env.sh "c2q:" "c2noq:DAVA_NO_QUEUE=1" "c2q:" "c2noq:DAVA_NO_QUEUE=1" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" \
  tools/ab_env.sh "c5q:" "c5noq:DAVA_NO_QUEUE=1" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8" \
  tools/ab_env.sh "c3convq:" "c3convnoq:DAVA_NO_QUEUE=1" || exit 1
