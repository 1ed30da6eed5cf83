set -uo pipefail
mkdir -p gpurun_out
P=$PWD/deep-attention-visual-odometry_amd/build/var_prev/libdava_ba.so
timeout -k 10 200 python3 tools/adjoint_dump.py gpurun_out/adj_new.npz && \
DAVA_LIB=$P timeout -k 10 200 python3 tools/adjoint_dump.py gpurun_out/adj_prev.npz || exit 1
python3 tools/adjoint_dump.py --compare gpurun_out/adj_new.npz gpurun_out/adj_prev.npz; echo "bitwise exit $?"
for r in 1 2; do
  for v in new prev nolds; do
    case $v in new) E="";; prev) E="DAVA_LIB=$P";; nolds) E="DAVA_ADJ_LDS_ENTRIES=0";; esac
    out=$(env $E timeout -k 10 300 python3 bench.py --cpu-sample 0 --differentiate --steps 2 --warmup 1 2>/dev/null | tail -1) || exit 1
    echo "$v $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("phase_ms"))')"
  done
done
