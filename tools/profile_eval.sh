#!/bin/bash
# rocprofv3 recipe for the Jacobian sweep alone (tools/eval_sweep.py, ba_evaluate_kernel) at one config:
#   1. --kernel-trace --stats  -> per-launch duration (must agree with eval_sweep.py's HIP events)
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (own passes)  -> fabric bytes per launch
#   4. SQ counters (tools/pmc_sq.sh with KERNEL/PROG)      -> VALUBusy, VALU FLOPs, waits
# usage: tools/profile_eval.sh TAG C3|C5
set -euo pipefail
TAG=$1; CFG=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_eval_${TAG}_$CFG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
  python3 "$R/tools/eval_sweep.py" --config "$CFG" --reps 20 > "$OUT/kt_sweep.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
  python3 "$R/tools/eval_sweep.py" --config "$CFG" --reps 5 > "$OUT/fetch_sweep.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
  python3 "$R/tools/eval_sweep.py" --config "$CFG" --reps 5 > "$OUT/write_sweep.log" 2>&1
cd "$R"
KERNEL=ba_evaluate_kernel PROG=tools/eval_sweep.py tools/pmc_sq.sh "eval_${TAG}_$CFG" --config "$CFG" --reps 5 \
  > "$OUT/sq.log" 2>&1
echo "profile_eval $TAG $CFG done"
