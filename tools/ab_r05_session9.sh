#!/bin/bash
# r05 session 9: GV per-entry scalars (rho_j, c_j) in the workspace slice instead of LDS, so the XL image
# fits at any iteration cap (the in-tree build) against HEAD before the change (build/var_head):
# bitwise at C5 K = 100 (XL in both), then C5 at K = 400 (XL only in the new build), interleaved.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
NEW=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
OLD=deep-attention-visual-odometry_amd/build/var_head/libdava_ba.so
timeout -k 10 300 python3 tools/lib_compare.py $OLD $NEW --batch 64 --views 16 --points 4096 --no-distortion --k 100 || exit 1
export BENCH_ARGS="--batch 256 --views 16 --points 4096 --no-distortion --iterations 400 --steps 1 --warmup 1 --parity-envelope 0"
tools/ab_env.sh "slice_k400:" "lds_k400:DAVA_LIB=@BUILD@/var_head/libdava_ba.so" "slice_k400:" "lds_k400:DAVA_LIB=@BUILD@/var_head/libdava_ba.so" || exit 1
export BENCH_ARGS="--batch 256 --views 16 --points 4096 --no-distortion --iterations 100 --steps 1 --warmup 1 --parity-envelope 0"
tools/ab_env.sh "slice_k100:" "lds_k100:DAVA_LIB=@BUILD@/var_head/libdava_ba.so" "slice_k100:" "lds_k100:DAVA_LIB=@BUILD@/var_head/libdava_ba.so" || exit 1
