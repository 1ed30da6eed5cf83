#!/bin/bash
# GPU box: the HYBRID form's fold (1,024 history entries folded into the dense matrix at iteration 1,025) where
# every problem reaches it -- K = ITERS (default 1,100) fixed iterations -- against DENSE from the start, at C3
# (B = 8192) and C5 (B = 256, P = 12,381: 157 GB of dense matrices).  One JSON line per run.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
common="--iterations ${ITERS:-1100} --cpu-sample 0 --parity-envelope 0 --no-converged-parity --no-live-counters --sustain-seconds 0 --steps 1 --warmup 0"
for cfg in "C3:" "C5:--batch 256 --views 16 --points 4096 --no-distortion"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for mode in compact dense; do
    echo "== $tag $mode ($(date +%T))" >&2
    timeout -k 10 400 python3 bench.py $common $args --mode $mode > gpurun_out/hf_${tag}_${mode}.log 2>&1 \
      || { tail -5 gpurun_out/hf_${tag}_${mode}.log >&2; exit 1; }
    tail -1 gpurun_out/hf_${tag}_${mode}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'config': '$tag', 'mode': '$mode', 'iterations': ${ITERS:-1100}, 'value': d['value'], 'unit': d['unit'], 'ms_per_step': d['ms_per_step']}))"
  done
done
