#!/bin/bash
# fused history pass leaves its last cross-wave add to the block-wide dots pass:
# bitwise check against the previous form, parity suite, interleaved A/B
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 200 python3 tools/dump_solve.py gpurun_out/d_new.npz 2>/dev/null &&
DAVA_LIB=$V/var_prev/libdava_ba.so timeout -k 10 200 python3 tools/dump_solve.py gpurun_out/d_prev.npz 2>/dev/null &&
python3 tools/dump_solve.py --compare gpurun_out/d_new.npz gpurun_out/d_prev.npz || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s20_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s20_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_env.sh "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --batch 1024 --views 2 --points 128 --no-distortion" \
  tools/ab_env.sh "c2:" "c2prev:DAVA_LIB=$V/var_prev/libdava_ba.so" "c2:" "c2prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
BENCH_ARGS="--steps 3 --warmup 1 --no-distortion --residual ray_angle" \
  tools/ab_env.sh "c3ray:" "c3rayprev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
