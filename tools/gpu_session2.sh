#!/bin/bash
# Phase-cycle attribution of the C3 solve (diagnostic builds) + C2 tail check
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
for v in phase phase_nosweep; do
  echo "== $v"
  DAVA_LIB=$V/var_$v/libdava_ba.so timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 1 --warmup 0 2>&1 | grep -E "phase|value" | cut -c1-400 || exit 1
done
echo "== phase C2"
DAVA_LIB=$V/var_phase/libdava_ba.so timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 1 --warmup 0 --batch 1024 --views 2 --points 128 --no-distortion 2>&1 | grep -E "phase|value" | cut -c1-400 || exit 1
timeout -k 10 300 python3 tools/status_stats.py > gpurun_out/status_stats.log 2>&1; cat gpurun_out/status_stats.log
