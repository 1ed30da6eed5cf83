#!/bin/bash
# A/B of whole-library compiler-flag variants (build/var_NAME) against the default build, interleaved,
# at C3, C5 and C2.  usage: tools/ab_flags.sh NAME...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
specs() { local tag=$1; shift; echo "${tag}_def:"; for n in "$@"; do echo "${tag}_$n:DAVA_LIB=@BUILD@/var_$n/libdava_ba.so"; done; }
ab() { local tag=$1 args=$2; shift 2; export BENCH_ARGS="$args"; mapfile -t S < <(specs "$tag" "$@")
  for r in 1 2; do tools/ab_env.sh "${S[@]}" || return 1; done; }
{ ab c3 "--steps 5 --warmup 1" "$@" && ab c5 "--batch 256 --views 16 --points 4096 --no-distortion --steps 2 --warmup 1" "$@" &&
  ab c2 "--batch 1024 --views 2 --points 128 --no-distortion --steps 20 --warmup 3" "$@"; } 2>&1 | tee gpurun_out/ab_flags.log
