#!/bin/bash
# Interleaved A/B of library variants / knobs on one box (run via gpurun from the repo root):
#   1. bitwise check: tools/dump_solve.py with the default build vs build/var_$BASE (skipped if BASE unset)
#   2. for each configuration in $CONFIGS (tag=bench args, ';'-separated), ROUNDS rounds of every spec
# usage: BASE=prev CONFIGS="c2=--batch 1024 --views 2 --points 128 --no-distortion" ROUNDS=2 \
#          tools/ab_session.sh "def:" "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ -n "${BASE:-}" ]; then
  timeout -k 10 300 python3 tools/dump_solve.py gpurun_out/dump_new.npz 2>/dev/null &&
  DAVA_LIB=$R/deep-attention-visual-odometry_amd/build/var_$BASE/libdava_ba.so \
    timeout -k 10 300 python3 tools/dump_solve.py gpurun_out/dump_$BASE.npz 2>/dev/null || { echo "dump failed"; exit 1; }
  python3 tools/dump_solve.py --compare gpurun_out/dump_new.npz gpurun_out/dump_$BASE.npz
  echo "bitwise vs $BASE: exit $?"
fi
IFS=';' read -ra cfgs <<< "${CONFIGS:-c3=--steps 3 --warmup 1}"
for cfg in "${cfgs[@]}"; do
  tag=${cfg%%=*}
  args=${cfg#*=}
  for ((r = 0; r < ${ROUNDS:-2}; r++)); do
    specs=()
    for s in "$@"; do specs+=("${tag}_${s}"); done
    BENCH_ARGS="$args" tools/ab_env.sh "${specs[@]}" || exit 1
  done
done
