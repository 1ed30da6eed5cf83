#!/bin/bash
# r05 session 3: C2's contention, measured -- SQ counters at B = 512 (two problems per CU, one wave per SIMD)
# and B = 1024 (four per CU, two waves per SIMD), and the per-phase cycle split including B = 512.
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
tools/gpu_run.sh "sq=r05_c2_b512:--batch 512 --views 2 --points 128 --no-distortion" \
  "sq=r05_c2_b1024:--batch 1024 --views 2 --points 128 --no-distortion" || exit 1
timeout -k 10 600 tools/phase_scan.sh > gpurun_out/phase_scan_r05.log 2>&1 || { tail -5 gpurun_out/phase_scan_r05.log; exit 1; }
cat gpurun_out/phase_scan_r05.log
