#!/bin/bash
# Round-6 GPU session (repo root on the box): the in-tree build against the r05 build and a variant.
#   1. bitwise: r05 vs the in-tree build at C2, C3 (B = 2048), C2 ray-angle and C5 (B = 64), full solves row by row
#   2. interleaved timing: r05 / VARIANT / in-tree at C2, C2 ray-angle, C3 and C5
# usage: tools/session_r06.sh [VARIANT_NAME]   (build/var_VARIANT_NAME; default novl)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
V=${1:-novl}
B=deep-attention-visual-odometry_amd/build
LIB=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
for c in "--batch 1024 --views 2 --points 128 --no-distortion" "--batch 2048" \
         "--batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle" \
         "--batch 64 --views 16 --points 4096 --no-distortion"; do
  echo "== bitwise r05 vs new: $c"
  timeout -k 10 300 python3 tools/lib_compare.py $B/var_r05/libdava_ba.so $LIB --seed 20254015 $c 2>&1 | grep -v amdgpu.ids | head -6 || exit 1
done
tools/ab.sh -r 2 -c "C2:--batch 1024 --views 2 --points 128 --no-distortion" \
  -c "C2_ray:--batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle" -c "C3:" \
  -c "C5:--batch 256 --views 16 --points 4096 --no-distortion --steps 1" \
  "r05:DAVA_LIB=@BUILD@/var_r05/libdava_ba.so" "$V:DAVA_LIB=@BUILD@/var_$V/libdava_ba.so" "new:" 2>&1 | cut -c1-260
