#!/bin/bash
# A/B one bench configuration under different override settings of the same library
# (e.g. DAVA_LDS_HISTORY, DAVA_LIB), one after another in one process each.  The library reads no
# environment: with DAVA_DEBUG_OVERRIDES=1 (set here) the Python binding passes the DAVA_<NAME>
# variables to dava_debug_set_override once, when it loads the library.
# usage: tools/ab_env.sh "TAG:VAR=VAL [VAR=VAL ...]" ... ; extra bench args via BENCH_ARGS
# "@BUILD@" in a value expands to the library's build/ directory (A/B variants: build/var_NAME/).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for spec in "$@"; do
  tag=${spec%%:*}
  envs=${spec#*:}
  [ "$envs" = "$spec" ] && envs=""
  envs=${envs//@BUILD@/$R/deep-attention-visual-odometry_amd/build}
  out=$(env DAVA_DEBUG_OVERRIDES=1 $envs timeout -k 10 300 python3 "$R/bench.py" --cpu-sample 0 --no-live-counters --sustain-seconds 0 ${BENCH_ARGS:---steps 3 --warmup 1} 2>&1 | tail -1) || {
    echo "$tag FAILED: $out"; exit 1; }
  echo "$tag $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"] or {}; g=d["diagnostics"]; print(d["value"], d["ms_per_step"], r.get("achieved"), r.get("frac"), "evals/it", g["objective_evals_per_iteration"], "trials/it", g["line_search_trials_per_iteration"], g.get("mean_steps_per_problem"), g["plan"])')"
done
