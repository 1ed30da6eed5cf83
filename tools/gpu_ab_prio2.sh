#!/bin/bash
# A/B: wave priorities (base/history) 2/0 (default) vs 3/1 vs 3/0, interleaved at C3 and C2.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
echo "## C3"
tools/ab_variants.sh base b3h1 b3h0 base b3h1 b3h0 || exit 1
echo "## C2"
BENCH_ARGS="--batch 1024 --views 2 --points 128 --no-distortion" tools/ab_variants.sh base b3h1 b3h0 base b3h1 b3h0
