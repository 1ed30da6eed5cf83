#!/bin/bash
# rocprofv3 recipe for the bench workload (run on the GPU box from the repo root):
#   1. --kernel-trace --stats           -> per-kernel durations (average must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE  (own pass)     -> HBM read bytes  (x2 on gfx950 for 16-B/lane streams, MI355X_MICROARCH.md HBM)
#   3. --pmc WRITE_SIZE  (own pass)     -> HBM write bytes
# Counters are collected with kernel-trace only (no sys/runtime traces), as the pool requires.
# usage: tools/profile.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
  python3 "$R/bench.py" --cpu-sample 0 --no-live-counters --sustain-seconds 0 "$@" > "$OUT/kt_bench.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
  python3 "$R/bench.py" --cpu-sample 0 --no-live-counters --sustain-seconds 0 --steps 1 --warmup 0 "$@" > "$OUT/fetch_bench.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
  python3 "$R/bench.py" --cpu-sample 0 --no-live-counters --sustain-seconds 0 --steps 1 --warmup 0 "$@" > "$OUT/write_bench.log" 2>&1
echo "profile $TAG done"
