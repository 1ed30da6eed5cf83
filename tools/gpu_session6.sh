#!/bin/bash
# Register-resident points in the objective (PPT): tests + interleaved A/B vs DAVA_NO_PPT
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py tests/test_gpu_objective.py tests/test_gpu_solve_grad.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests6.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests6.log
[ $rc -le 1 ] || exit $rc
tools/ab_env.sh "c3ppt:" "c3noppt:DAVA_NO_PPT=1" "c3ppt:" "c3noppt:DAVA_NO_PPT=1" || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --batch 256 --views 16 --points 4096 --no-distortion" \
  tools/ab_env.sh "c5ppt:" "c5noppt:DAVA_NO_PPT=1" || exit 1
