#!/bin/bash
# A/B the library variants built by `make variant` (same process config, one after another).
# usage: tools/ab_variants.sh NAME... ; extra bench args via BENCH_ARGS
R=${GRAFT_REPO_ROOT:-$(pwd)}
for n in "$@"; do
  lib=$R/deep-attention-visual-odometry_amd/build/var_$n/libdava_ba.so
  out=$(DAVA_LIB=$lib timeout -k 10 300 python3 $R/bench.py --cpu-sample 0 ${BENCH_ARGS:---steps 3 --warmup 1} 2>/dev/null | tail -1)
  echo "$n $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"] or {}; print(d["value"], d["ms_per_step"], r.get("achieved"), r.get("frac"), d["diagnostics"])')"
done
