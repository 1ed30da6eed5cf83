#!/bin/bash
# Round-6 GPU session (repo root on the box).
#   lean : interleaved timing of the first lean trial index (in-tree = 1, build/var_lean2, build/var_lean3)
#          at C2, C2 ray-angle and C3, after a bitwise check of each against the in-tree build
#   diag : tools/eval_bitwise.py (the objective's trial forms, bit for bit), phase cycles (build/var_phase)
#          and the closure entry (compact vs dense generic loop)
# usage: tools/session_r06.sh lean|diag ...
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
        2>&1 | cut -c1-260 || exit 1 ;;
    diag)
      echo "== eval_bitwise"
      timeout -k 10 300 python3 tools/eval_bitwise.py 2>&1 | grep -v amdgpu.ids || exit 1
      tools/gpu_run.sh phase closure || exit 1 ;;
  esac
done
