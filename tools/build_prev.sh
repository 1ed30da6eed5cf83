#!/bin/bash
# Build the library from a git revision's sources (default HEAD) into build/var_prev (A/B baseline).
# usage: tools/build_prev.sh [REV] [NAME]
set -euo pipefail
REV=${1:-HEAD}
NAME=${2:-prev}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/csrc" "$T/include"
for f in $(git -C "$R" ls-tree --name-only "$REV" deep-attention-visual-odometry_amd/csrc/); do
  git -C "$R" show "$REV:$f" > "$T/csrc/$(basename "$f")"
done
if [ -n "${CURRENT_HEADER:-}" ]; then cp "$R/include/dava_ba.h" "$T/include/"; else git -C "$R" show "$REV:include/dava_ba.h" > "$T/include/dava_ba.h"; fi
OUT=$R/deep-attention-visual-odometry_amd/build/var_$NAME
mkdir -p "$OUT"
objs=()
for src in "$T"/csrc/*.hip; do
  o="$OUT/$(basename "${src%.hip}").o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fno-slp-vectorize -Wno-unused-function -I"$T/include" -I"$T/csrc" -c "$src" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$OUT/libdava_ba.so"
rm -rf "$T"
echo "built $OUT/libdava_ba.so from $REV"
