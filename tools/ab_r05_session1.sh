#!/bin/bash
# r05 A/B session 1: intra-CU start stagger at C2, LDS-entry prefetch at C2/C3, intrinsics trace
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
S1="base:"; S2="s0:DAVA_STAGGER=0"; S3="L4s8a:DAVA_STAGGER=29000 DAVA_STAGGER_LEVELS=4 DAVA_STAGGER_SHIFT=8"
S4="L4s8b:DAVA_STAGGER=15000 DAVA_STAGGER_LEVELS=4 DAVA_STAGGER_SHIFT=8"; S5="L2s8:DAVA_STAGGER=58000 DAVA_STAGGER_LEVELS=2 DAVA_STAGGER_SHIFT=8"
P="pf:DAVA_LIB=@BUILD@/var_pf/libdava_ba.so"
BENCH_ARGS="--batch 1024 --views 2 --points 128 --no-distortion --steps 5 --warmup 2" tools/ab_env.sh "$S1" "$S2" "$S3" "$S4" "$S5" "$P" "$S1" "$S2" "$S3" "$S4" "$S5" "$P" > gpurun_out/ab_c2_stagger_pf.log 2>&1 || exit 1
cat gpurun_out/ab_c2_stagger_pf.log | cut -c1-120
BENCH_ARGS="--steps 3 --warmup 1" tools/ab_env.sh "$S1" "$P" "$S1" "$P" > gpurun_out/ab_c3_pf.log 2>&1 || exit 1
cat gpurun_out/ab_c3_pf.log | cut -c1-120
timeout -k 10 600 python3 tools/trace_intrinsics.py > gpurun_out/trace_intrinsics.jsonl 2> gpurun_out/trace_intrinsics.err || { tail -5 gpurun_out/trace_intrinsics.err; exit 1; }
head -8 gpurun_out/trace_intrinsics.jsonl | cut -c1-300
