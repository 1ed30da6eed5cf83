#!/bin/bash
# A/B: LLVM AMDGPU machine-scheduler strategy for the solve kernel (default vs max-ilp vs
# max-memory-clause), interleaved on one box at C3 and C2, plus bitwise dumps of each variant.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
B=deep-attention-visual-odometry_amd/build
for v in base ilp memclause; do
  DAVA_LIB=$B/var_$v/libdava_ba.so timeout -k 10 120 python3 tools/dump_solve.py gpurun_out/dump_$v.npz > gpurun_out/dump_$v.log 2>&1 || { tail -5 gpurun_out/dump_$v.log; exit 1; }
done
python3 tools/dump_solve.py --compare gpurun_out/dump_base.npz gpurun_out/dump_ilp.npz
python3 tools/dump_solve.py --compare gpurun_out/dump_base.npz gpurun_out/dump_memclause.npz
echo "## C3"
tools/ab_variants.sh base ilp memclause base ilp memclause || exit 1
echo "## C2"
BENCH_ARGS="--batch 1024 --views 2 --points 128 --no-distortion" tools/ab_variants.sh base ilp memclause base ilp memclause
