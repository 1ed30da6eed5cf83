#!/bin/bash
# usage: adj_ab.sh "BENCH ARGS" tag[:lib] ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
args=$1; shift
for spec in "$@"; do
  t=${spec%%:*}; lib=${spec#*:}; [ "$lib" = "$spec" ] && lib=""
  [ -n "$lib" ] && lib=$R/deep-attention-visual-odometry_amd/build/var_$lib/libdava_ba.so
  out=$(env DAVA_DEBUG_OVERRIDES=1 ${lib:+DAVA_LIB=$lib} timeout -k 10 300 python3 $R/bench.py $args 2>&1 | tail -1)
  echo "$t $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"], d["roofline"]["frac"])' 2>&1 | tail -1)"
done
