#!/bin/bash
# r05 session 5: the history pass consuming its on-chip entries and HBM remainder in batches (variant bs):
# bitwise against the default build, interleaved A/B at C2 (B = 1024 and 256), C3 and the C1 shape
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
A=$(pwd)/deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
B=$(pwd)/deep-attention-visual-odometry_amd/build/var_bs/libdava_ba.so
for shape in "--views 2 --points 128 --no-distortion --batch 1024" "--views 4 --points 256 --batch 2048"; do
  timeout -k 10 300 python3 tools/lib_compare.py $A $B $shape > gpurun_out/bs_bitwise.log 2>&1 || { cat gpurun_out/bs_bitwise.log | tail -5; exit 1; }
  tail -2 gpurun_out/bs_bitwise.log
done
P="bs:DAVA_LIB=@BUILD@/var_bs/libdava_ba.so"
( BENCH_ARGS="--batch 1024 --views 2 --points 128 --no-distortion --steps 5 --warmup 2" tools/ab_env.sh "C2:" "$P" "C2:" "$P" "C2:" "$P" &&
  BENCH_ARGS="--batch 256 --views 2 --points 128 --no-distortion --steps 5 --warmup 2" tools/ab_env.sh "C2b256:" "$P" "C2b256:" "$P" &&
  BENCH_ARGS="--steps 3 --warmup 1" tools/ab_env.sh "C3:" "$P" "C3:" "$P" "C3:" "$P" &&
  BENCH_ARGS="--batch 8192 --views 2 --points 64 --no-distortion --steps 3 --warmup 1" tools/ab_env.sh "C1b8k:" "$P" "C1b8k:" "$P" ) \
  2>&1 | cut -c1-110 | tee gpurun_out/ab_batch_serial.log
