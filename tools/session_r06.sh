#!/bin/bash
# Round-6 GPU session (repo root on the box).
#   lean : interleaved timing of the first lean trial index (in-tree = 1, build/var_lean2, build/var_lean3)
#          and d . grad first-trial slopes in LDS mode (build/var_dot1) at C2, C2 ray-angle and C3
#   gvlean: the same for global-vector mode at C5 (build/var_gvlean1, build/var_gvlean2)
#   diag : tools/eval_bitwise.py (the objective's trial forms, bit for bit), phase cycles (build/var_phase)
#          and the closure entry (compact vs dense generic loop)
#   configs: tools/measure_configs.sh on the in-tree build
#   generic: the generic-loop GPU tests, the closure entry (compact vs dense) and tools/closure_profile.py
#   hybrid : tools/hybrid_fold.sh (K = 1,100 fixed: the fold at iteration 1,025 against DENSE, C3 and C5)
# usage: tools/session_r06.sh lean|gvlean|configs|generic|hybrid|diag ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for s in "$@"; do
  case $s in
    lean)
      tools/ab.sh -r 2 -c "C2:--batch 1024 --views 2 --points 128 --no-distortion" \
        -c "C2_ray:--batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle" -c "C3:" \
        "lean1:" "lean2:DAVA_LIB=@BUILD@/var_lean2/libdava_ba.so" "lean3:DAVA_LIB=@BUILD@/var_lean3/libdava_ba.so" \
        "dot1:DAVA_LIB=@BUILD@/var_dot1/libdava_ba.so" 2>&1 | cut -c1-260 || exit 1 ;;
    gvlean)
      tools/ab.sh -r 2 -c "C5:--batch 256 --views 16 --points 4096 --no-distortion --steps 1" \
        "full:" "gvlean1:DAVA_LIB=@BUILD@/var_gvlean1/libdava_ba.so" "gvlean2:DAVA_LIB=@BUILD@/var_gvlean2/libdava_ba.so" \
        2>&1 | cut -c1-260 || exit 1 ;;
    configs)
      tools/measure_configs.sh || exit 1 ;;
    generic)
      echo "== generic-loop GPU tests"
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_solve_grad.py tests/test_gpu_camera_l1.py \
        -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s6_generic_tests.log 2>&1; rc=$?
      tail -2 gpurun_out/s6_generic_tests.log; [ $rc -eq 0 ] || exit 1
      tools/gpu_run.sh closure || exit 1
      echo "== closure profile"
      timeout -k 10 300 python3 tools/closure_profile.py > gpurun_out/closure_profile.log 2>&1 || { tail -5 gpurun_out/closure_profile.log; exit 1; }
      head -1 gpurun_out/closure_profile.log ;;
    hybrid)
      echo "== hybrid fold"
      tools/hybrid_fold.sh > gpurun_out/hybrid_fold.jsonl || exit 1
      cat gpurun_out/hybrid_fold.jsonl ;;
    diag)
      echo "== eval_bitwise"
      timeout -k 10 300 python3 tools/eval_bitwise.py 2>&1 | grep -v amdgpu.ids || exit 1
      tools/gpu_run.sh phase closure || exit 1 ;;
  esac
done
