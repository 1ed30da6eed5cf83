#!/bin/bash
# The reference's stopping rules (1e-4 / 1e-8) under an iteration cap past 1025: COMPACT (the hybrid
# kernel: history, folded into the dense matrix only for a problem still running at iteration 1025)
# against DENSE (what the drop-in's 'auto' mode took for such caps before r05).  One bench line each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
out=gpurun_out/hybrid_defaults.jsonl
: > "$out"
common="--iterations ${ITERS:-2000} --error-threshold 1e-4 --minimum-step 1e-8 --cpu-sample 0 --parity-envelope 0 --no-live-counters --sustain-seconds 0 --steps 3 --warmup 1"
for cfg in "C2:--views 2 --points 128 --no-distortion" "C3:"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for mode in compact dense; do
    echo "== $tag $mode ($(date +%T))"
    timeout -k 10 300 python3 bench.py $common $args --mode $mode > gpurun_out/hd_${tag}_${mode}.log 2>&1 || { tail -5 gpurun_out/hd_${tag}_${mode}.log; exit 1; }
    tail -1 gpurun_out/hd_${tag}_${mode}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'config': '$tag', 'mode': '$mode', 'iterations_cap': ${ITERS:-2000}, 'value': d['value'], 'unit': d['unit'], 'ms_per_step': d['ms_per_step']}))" | tee -a "$out"
  done
done
