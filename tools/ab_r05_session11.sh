#!/bin/bash
# r05 session 11: session 10's build with the on-chip entries rounded to a multiple of the waves for rows of
# <= 2 groups (C1 / C2), against HEAD (build/var_head): C2 and the C1 shape at K = 100, C2 under defaults.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
H="DAVA_LIB=@BUILD@/var_head/libdava_ba.so"
for cfg in "c2:--batch 1024 --views 2 --points 128 --no-distortion" "c1:--batch 8192 --views 2 --points 64 --no-distortion" \
           "c2def:--batch 1024 --views 2 --points 128 --no-distortion --iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  export BENCH_ARGS="$args --steps 3 --warmup 1 --parity-envelope 0"
  tools/ab_env.sh "${tag}_new:" "${tag}_head:$H" "${tag}_new:" "${tag}_head:$H" || exit 1
done
