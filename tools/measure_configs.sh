#!/bin/bash
# One bench line per BASELINE.json configuration that fits one GPU (plus the ray-angle
# residual at C2/C3), into gpurun_out/configs.jsonl.  Run on the GPU box from the repo root.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/configs.jsonl
: > "$OUT"
run() {
  local tag=$1; shift
  if timeout -k 10 600 python3 "$R/bench.py" --cpu-sample 0 --sustain-seconds 0 "$@" > "$R/gpurun_out/cfg_$tag.log" 2>&1; then
    echo "{\"tag\": \"$tag\", \"line\": $(tail -1 "$R/gpurun_out/cfg_$tag.log")}" >> "$OUT"
  else
    echo "config $tag failed"; tail -5 "$R/gpurun_out/cfg_$tag.log"; return 1
  fi
}
run C2 --batch 1024 --views 2 --points 128 --no-distortion &&
run C2_ray --batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle &&
run C3 --steps 3 &&
run C3_pinhole --no-distortion &&
run C3_ray --no-distortion --residual ray_angle &&
run C3_dense --mode dense --steps 1 &&
run C5 --batch 256 --views 16 --points 4096 --no-distortion --steps 1 || exit 1
# solve + gradient (the recording solve and the fused adjoint), C2 / C3 / C5 (DIFF=0 skips them)
if [ "${DIFF:-1}" = 1 ]; then
  run C2_grad --batch 1024 --views 2 --points 128 --no-distortion --differentiate &&
  run C3_grad --differentiate --steps 2 &&
  run C5_grad --batch 256 --views 16 --points 4096 --no-distortion --differentiate --steps 1
fi
