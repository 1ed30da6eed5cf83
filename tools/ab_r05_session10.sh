#!/bin/bash
# r05 session 10: LDS product coefficients only for the two-pass products (the in-tree build) against HEAD
# before the change (build/var_head): bitwise at C2 / C3 (K = 100), then interleaved A/B at C2 and C3
# (K = 100, fixed) and under the reference's defaults (cap 1000, stopping rules), where the freed LDS
# holds more on-chip history entries.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
NEW=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
OLD=deep-attention-visual-odometry_amd/build/var_head/libdava_ba.so
timeout -k 10 300 python3 tools/lib_compare.py $OLD $NEW --batch 1024 --views 2 --points 128 --no-distortion --k 100 || exit 1
timeout -k 10 300 python3 tools/lib_compare.py $OLD $NEW --batch 2048 --k 100 || exit 1
H="DAVA_LIB=@BUILD@/var_head/libdava_ba.so"
for cfg in "c2:--batch 1024 --views 2 --points 128 --no-distortion" "c3:" \
           "c2def:--batch 1024 --views 2 --points 128 --no-distortion --iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8" \
           "c3def:--iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  export BENCH_ARGS="$args --steps 3 --warmup 1 --parity-envelope 0"
  tools/ab_env.sh "${tag}_new:" "${tag}_head:$H" "${tag}_new:" "${tag}_head:$H" || exit 1
done
