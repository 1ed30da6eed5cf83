#!/bin/bash
# Build A/B library variants in parallel: tools/build_variants.sh NAME=FLAGS ... (run in this container)
# e.g. tools/build_variants.sh "dot=-DDAVA_TRIAL_DOT=1" "noslp=-fno-slp-vectorize"
set -uo pipefail
cd "$(dirname "$0")/../deep-attention-visual-odometry_amd"
pids=()
for spec in "$@"; do
  name=${spec%%=*}
  flags=${spec#*=}
  rm -rf "build/var_$name"
  make variant NAME="$name" FLAGS="$flags" > "/tmp/variant_$name.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
for spec in "$@"; do
  name=${spec%%=*}
  if [ -f "build/var_$name/libdava_ba.so" ]; then echo "built $name"; else echo "FAILED $name"; tail -5 "/tmp/variant_$name.log"; rc=1; fi
done
exit $rc
