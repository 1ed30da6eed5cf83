#!/bin/bash
# Interleaved A/B of bench.py lines under library builds and / or launch overrides (GPU box, repo root).
# Replaces the one-off round-5 session scripts: every session was "these configurations, these variants,
# interleaved R times", optionally after a bitwise check of the variants' results.
#
# usage: tools/ab.sh [-r REPS] [-d] [-x] -c "TAG:BENCH ARGS" [-c ...] "LABEL:ENV" "LABEL:ENV" ...
#   -r REPS   rounds of the interleave (default 2): cfg1 A B, cfg1 A B, ... per configuration
#   -d        time `bench.py --differentiate` (recording solve + adjoint) instead of the solve
#   -x        first compare every variant's solve with the first one's, row by row (tools/lib_compare.py,
#             needs DAVA_LIB in the variant's ENV), at each configuration's shape
#   -c        a configuration: TAG and the bench flags that make it (e.g. "C2:--batch 1024 --views 2
#             --points 128 --no-distortion"); repeatable
#   LABEL:ENV a variant: environment assignments for its bench process.  DAVA_LIB=@BUILD@/var_NAME/libdava_ba.so
#             picks a build (tools/build_prev.sh REV NAME, or `make variant NAME=.. FLAGS=..`), DAVA_<KNOB>=v a
#             launch override (passed to dava_debug_set_override at load); an empty ENV is the in-tree build.
# example: tools/ab.sh -r 3 -x -c "C2:--batch 1024 --views 2 --points 128 --no-distortion" -c "C3:" \
#            "head:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" "new:"
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
REPS=2; DIFF=""; CHECK=""; CFGS=()
while getopts "r:dxc:" o; do
  case $o in
    r) REPS=$OPTARG ;;
    d) DIFF="--differentiate" ;;
    x) CHECK=1 ;;
    c) CFGS+=("$OPTARG") ;;
    *) echo "bad option"; exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ ${#CFGS[@]} -gt 0 ] && [ $# -ge 1 ] || { sed -n '2,20p' "$0"; exit 2; }
BUILD=$R/deep-attention-visual-odometry_amd/build
libof() {  # the DAVA_LIB of a variant's ENV ('' = in-tree)
  local e=${1#*:}; e=${e//@BUILD@/$BUILD}
  for kv in $e; do [ "${kv%%=*}" = DAVA_LIB ] && { echo "${kv#*=}"; return; }; done
  echo "$R/deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so"
}
if [ -n "$CHECK" ]; then
  base=$(libof "$1")
  for cfg in "${CFGS[@]}"; do
    tag=${cfg%%:*}; args=${cfg#*:}
    # the shape flags lib_compare understands
    cmp=$(python3 - "$args" <<'EOF'
import sys, shlex
a = shlex.split(sys.argv[1]); out = []
m = {"--batch": "--batch", "--views": "--views", "--points": "--points", "--iterations": "--k"}
i = 0
while i < len(a):
    if a[i] in m: out += [m[a[i]], a[i + 1]]; i += 2; continue
    if a[i] == "--no-distortion": out.append(a[i])
    if a[i] == "--residual": out += ["--residual", a[i + 1]]; i += 2; continue
    if a[i] == "--mode": out += ["--mode", "0" if a[i + 1] == "dense" else "1"]; i += 2; continue
    i += 1
if "--batch" not in out: out += ["--batch", "8192"]
print(" ".join(out))
EOF
)
    for spec in "${@:2}"; do
      echo "== bitwise $tag ${1%%:*} vs ${spec%%:*}"
      timeout -k 10 600 python3 tools/lib_compare.py "$base" "$(libof "$spec")" --seed 20254015 $cmp || exit 1
    done
  done
fi
for cfg in "${CFGS[@]}"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  echo "== $tag ($args)"
  for ((rep = 1; rep <= REPS; rep++)); do
    for spec in "$@"; do
      label=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
      envs=${envs//@BUILD@/$BUILD}
      out=$(env DAVA_DEBUG_OVERRIDES=1 $envs timeout -k 10 400 python3 bench.py --cpu-sample 0 --parity-envelope 0 \
            --no-live-counters --sustain-seconds 0 $DIFF $args 2>&1 | tail -1) || { echo "$tag $label FAILED: $out"; exit 1; }
      echo "$tag $label $(echo "$out" | python3 -c '
import sys, json
d = json.loads(sys.stdin.read()); r = d.get("roofline") or {}; g = d.get("diagnostics") or {}
pp = g.get("per_problem") or {}
print(d["value"], d["ms_per_step"], "frac", r.get("frac"), "evals/it", g.get("objective_evals_per_iteration"),
      "evals p50/p99/max", [pp.get("evaluations", {}).get(k) for k in ("p50", "p99", "max")],
      json.dumps(d.get("phases_ms") or {}))')"
    done
  done
done
