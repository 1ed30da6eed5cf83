set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_generic.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/s2_tests.log
B=deep-attention-visual-odometry_amd/build
for c in "--batch 1024 --views 2 --points 128 --no-distortion" "--batch 8192 --views 2 --points 64 --no-distortion"; do
  timeout -k 10 300 python3 tools/lib_compare.py $B/var_prev/libdava_ba.so $B/var_nomove/libdava_ba.so --seed 20254015 $c 2>&1 | grep -v amdgpu.ids | head -4
done
for cfg in "--batch 1024 --views 2 --points 128" "--batch 256 --views 4 --points 256"; do
  for v in compact dense; do
    e=""; [ $v = dense ] && e="DAVA_DEBUG_OVERRIDES=1 DAVA_GENERIC_DENSE=1"
    env $e timeout -k 10 600 python3 bench.py --entry closure --residual ray_angle --no-distortion $cfg --steps 1 --warmup 1 --cpu-sample 0 --no-live-counters --sustain-seconds 0 > gpurun_out/s2_closure.log 2>&1 || { echo "closure $v failed"; tail -5 gpurun_out/s2_closure.log; exit 1; }
    echo "closure $cfg $v: $(tail -1 gpurun_out/s2_closure.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_memory_bytes"], d["history_bytes"], d["parity"]["vs_fused_ray_angle_solve_max_rel"])')"
  done
done
tools/ab.sh -r 2 -c "C2:--batch 1024 --views 2 --points 128 --no-distortion" -c "C1:--batch 8192 --views 2 --points 64 --no-distortion" -c "C3:" "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" "lean:DAVA_LIB=@BUILD@/var_lean/libdava_ba.so" "nomove:DAVA_LIB=@BUILD@/var_nomove/libdava_ba.so" "both:" "lean2:DAVA_LIB=@BUILD@/var_lean2/libdava_ba.so" 2>&1 | cut -c1-200
