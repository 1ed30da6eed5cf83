#!/bin/bash
# Interleaved A/B of the current library against build/var_prev (tools/build_prev.sh) at C3, C2, C1 and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for cfg in "C3:" "C2:--batch 1024 --views 2 --points 128 --no-distortion" "C1:--batch 8192 --views 2 --points 64 --no-distortion" "C5:--batch 256 --views 16 --points 4096 --no-distortion --steps 1"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  echo "== $tag"
  BENCH_ARGS="$args --warmup 1" tools/ab_env.sh "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" "new:DAVA_LIB=@BUILD@/var_new/libdava_ba.so" "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" "new:DAVA_LIB=@BUILD@/var_new/libdava_ba.so" || exit 1
done
