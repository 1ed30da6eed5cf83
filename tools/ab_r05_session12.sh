#!/bin/bash
# r05 session 12: the LDS-mode adjoint reading the tape's scalar row in place when staging it would cost the
# second workgroup per CU (the in-tree build) against HEAD (build/var_head): solve + gradient at C3
# (B = 4096) under the reference's stopping rules with caps 200 (both stage it) and 1000.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for k in 200 1000; do
  for lib in new head; do
    env_lib=""
    [ $lib = head ] && env_lib="DAVA_DEBUG_OVERRIDES=1 DAVA_LIB=$R/deep-attention-visual-odometry_amd/build/var_head/libdava_ba.so"
    for rep in 1 2; do
      out=$(env $env_lib timeout -k 10 300 python3 bench.py --differentiate --iterations $k --error-threshold 1e-4 \
        --minimum-step 1e-8 --cpu-sample 0 --parity-envelope 0 --no-live-counters --sustain-seconds 0 --steps 2 \
        --warmup 1 --batch 4096 2>&1 | tail -1) || { echo "$k $lib failed: $out"; exit 1; }
      echo "K=$k $lib $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], json.dumps(d.get("phases_ms") or d.get("differentiate") or {})[:200])')"
    done
  done
done
