#!/bin/bash
# update dots formed inside the fused history pass: parity suite + interleaved A/B
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s19_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s19_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_env.sh "c3:" "c3nodots:DAVA_LIB=$V/var_nodots/libdava_ba.so" "c3:" "c3nodots:DAVA_LIB=$V/var_nodots/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" \
  tools/ab_env.sh "c2:" "c2nodots:DAVA_LIB=$V/var_nodots/libdava_ba.so" "c2:" "c2nodots:DAVA_LIB=$V/var_nodots/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --no-distortion --residual ray_angle" \
  tools/ab_env.sh "c3ray:" "c3raynodots:DAVA_LIB=$V/var_nodots/libdava_ba.so" || exit 1
