#!/bin/bash
# A/B of the packed two-point pair sweep (GV mode) and of -fno-slp-vectorize, interleaved on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V="c_def: c_noslp:DAVA_LIB=@BUILD@/var_noslp/libdava_ba.so c_pack:DAVA_LIB=@BUILD@/var_pack/libdava_ba.so c_packnoslp:DAVA_LIB=@BUILD@/var_packnoslp/libdava_ba.so"
ab() { local tag=$1; shift; export BENCH_ARGS="$*"; for r in 1 2; do tools/ab_env.sh ${V//c_/${tag}_} || exit 1; done; }
{ ab c3 --steps 5 --warmup 1 && ab c5 --batch 256 --views 16 --points 4096 --no-distortion --steps 2 --warmup 1 &&
  ab c2 --batch 1024 --views 2 --points 128 --no-distortion --steps 20 --warmup 3; } 2>&1 | tee gpurun_out/ab_pack.log
