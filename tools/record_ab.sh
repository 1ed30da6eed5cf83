#!/bin/bash
# A/B of a change to the recording solve (run via gpurun from the repo root): bitwise checks of
# the eval solve and of the adjoint's gradients against build/var_prev, then interleaved timings of
# the eval solve (C3) and of the differentiate line.
set -uo pipefail
mkdir -p gpurun_out
P=$PWD/deep-attention-visual-odometry_amd/build/var_prev/libdava_ba.so
timeout -k 10 200 python3 tools/adjoint_dump.py gpurun_out/adj_new.npz && \
DAVA_LIB=$P timeout -k 10 200 python3 tools/adjoint_dump.py gpurun_out/adj_prev.npz || exit 1
python3 tools/adjoint_dump.py --compare gpurun_out/adj_new.npz gpurun_out/adj_prev.npz; echo "adjoint bitwise exit $?"
BASE=prev CONFIGS="c3=--steps 3 --warmup 1" ROUNDS=2 tools/ab_session.sh "new:" "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" || exit 1
for r in 1 2; do
  for v in new prev; do
    E=""; [ $v = prev ] && E="DAVA_LIB=$P"
    out=$(env $E timeout -k 10 300 python3 bench.py --cpu-sample 0 --differentiate --steps 2 --warmup 1 2>/dev/null | tail -1) || exit 1
    echo "diff_$v $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("phases_ms"))')"
  done
done
