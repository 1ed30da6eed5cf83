#!/bin/bash
# Round-6 GPU session (repo root on the box).
#   lean : interleaved timing of the first lean trial index (in-tree = 1, build/var_lean2, build/var_lean3)
#          and d . grad first-trial slopes in LDS mode (build/var_dot1) at C2, C2 ray-angle and C3
#   gvlean: the same for global-vector mode at C5 (build/var_gvlean1, build/var_gvlean2)
#   diag : tools/eval_bitwise.py (the objective's trial forms, bit for bit), phase cycles (build/var_phase)
#          and the closure entry (compact vs dense generic loop)
#   configs: tools/measure_configs.sh on the in-tree build
#   generic: the generic-loop GPU tests, the closure entry (compact vs dense) and tools/closure_profile.py
#   hybrid : tools/hybrid_fold.sh (K = 1,100 fixed: the fold at iteration 1,025 against DENSE, C3 and C5)
#   defaults: the reference's defaults (cap 1,000, stopping rules) at C2, C3, C5
#   profiles: tools/profile.sh (kernel trace, FETCH_SIZE, WRITE_SIZE) at C3, C2, C5
# usage: tools/session_r06.sh lean|gvlean|configs|generic|hybrid|defaults|profiles|diag ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for s in "$@"; do
  case $s in
    lean)
      tools/ab.sh -r 2 -c "C2:--batch 1024 --views 2 --points 128 --no-distortion" \
        -c "C2_ray:--batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle" -c "C3:" \
        "lean1:" "lean2:DAVA_LIB=@BUILD@/var_lean2/libdava_ba.so" "lean3:DAVA_LIB=@BUILD@/var_lean3/libdava_ba.so" \
        "dot1:DAVA_LIB=@BUILD@/var_dot1/libdava_ba.so" 2>&1 | cut -c1-260 || exit 1 ;;
    gvlean)
      tools/ab.sh -r 2 -c "C5:--batch 256 --views 16 --points 4096 --no-distortion --steps 1" \
        "full:" "gvlean1:DAVA_LIB=@BUILD@/var_gvlean1/libdava_ba.so" "gvlean2:DAVA_LIB=@BUILD@/var_gvlean2/libdava_ba.so" \
        2>&1 | cut -c1-260 || exit 1 ;;
    configs)
      tools/measure_configs.sh || exit 1 ;;
    generic)
      echo "== generic-loop GPU tests"
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_solve_grad.py tests/test_gpu_camera_l1.py \
        -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s6_generic_tests.log 2>&1; rc=$?
      tail -2 gpurun_out/s6_generic_tests.log; [ $rc -eq 0 ] || exit 1
      tools/gpu_run.sh closure || exit 1
      echo "== closure profile"
      timeout -k 10 300 python3 tools/closure_profile.py > gpurun_out/closure_profile.log 2>&1 || { tail -5 gpurun_out/closure_profile.log; exit 1; }
      head -1 gpurun_out/closure_profile.log ;;
    l1)
      echo "== legacy L1 model GPU tests"
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_camera_l1.py -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/s6_l1_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s6_l1_tests.log; [ $rc -eq 0 ] || exit 1 ;;
    fold)
      echo "== fold: bitwise r05 vs new at K = 1,100 (every problem folds at iteration 1,025)"
      B=deep-attention-visual-odometry_amd/build
      LIB=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
      for c in "--batch 64 --views 2 --points 128 --no-distortion" "--batch 64" "--batch 16 --views 16 --points 4096 --no-distortion"; do
        timeout -k 10 300 python3 tools/lib_compare.py $B/var_r05/libdava_ba.so $LIB --seed 20254015 --k 1100 $c 2>&1 \
          | grep -v amdgpu.ids | head -4 || exit 1
      done
      echo "== fold timing"
      tools/hybrid_fold.sh > gpurun_out/hybrid_fold_new.jsonl || exit 1
      cat gpurun_out/hybrid_fold_new.jsonl
      echo "== hybrid GPU tests"
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_hybrid.py -m gpu -x -q --timeout 200 --timeout-method thread \
        > gpurun_out/s6_hybrid_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s6_hybrid_tests.log; [ $rc -eq 0 ] || exit 1 ;;
    foldab)
      B=deep-attention-visual-odometry_amd/build
      LIB=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
      echo "== fold rows: bitwise 8 vs 16 / 32 at K = 1,100"
      for v in fold16 fold32 rl16 rl32; do
        timeout -k 10 300 python3 tools/lib_compare.py $LIB $B/var_$v/libdava_ba.so --seed 20254015 --k 1100 --batch 64 2>&1 \
          | grep -v amdgpu.ids | head -2 || exit 1
      done
      echo "== fold rows: timing (K = 1,100 fixed, compact = hybrid)"
      for cfg in "C3:" "C5:--batch 256 --views 16 --points 4096 --no-distortion"; do
        tag=${cfg%%:*}; args=${cfg#*:}
        for v in rows8 fold16 fold32 rl16 rl32; do
          e=""; [ $v != rows8 ] && e="DAVA_DEBUG_OVERRIDES=1 DAVA_LIB=$B/var_$v/libdava_ba.so"
          out=$(env $e timeout -k 10 400 python3 bench.py --iterations 1100 --cpu-sample 0 --parity-envelope 0 \
                --no-converged-parity --no-live-counters --sustain-seconds 0 --steps 1 --warmup 0 $args 2>&1 | tail -1) \
            || { echo "$tag $v failed"; exit 1; }
          echo "$tag $v $(echo "$out" | python3 -c 'import sys, json; d = json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
        done
      done ;;
    defab)
      tools/ab.sh -r 2 -c "C2def:--batch 1024 --views 2 --points 128 --no-distortion --iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8 --no-converged-parity" \
        -c "C3def:--iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8 --no-converged-parity" \
        "r05:DAVA_LIB=@BUILD@/var_r05/libdava_ba.so" "new:" 2>&1 | cut -c1-200 || exit 1 ;;
    bitwise)
      B=deep-attention-visual-odometry_amd/build
      LIB=deep-attention-visual-odometry_amd/deep_attention_visual_odometry_amd/_lib/libdava_ba.so
      for c in "--batch 1024 --views 2 --points 128 --no-distortion" "--batch 2048" \
               "--batch 1024 --views 2 --points 128 --no-distortion --residual ray_angle" \
               "--batch 64 --views 16 --points 4096 --no-distortion"; do
        echo "== bitwise r05 vs new: $c"
        timeout -k 10 300 python3 tools/lib_compare.py $B/var_r05/libdava_ba.so $LIB --seed 20254015 $c 2>&1 \
          | grep -v amdgpu.ids | head -3 || exit 1
      done ;;
    final)
      tools/gpu_run.sh tests smoke bench || exit 1 ;;
    foldvar)
      B=deep-attention-visual-odometry_amd/build
      for v in intree rl16 shfl32 rows8; do
        e=""; [ $v != intree ] && e="DAVA_DEBUG_OVERRIDES=1 DAVA_LIB=$B/var_$v/libdava_ba.so"
        echo "== $v"
        env $e timeout -k 10 300 python3 -u -m pytest tests/test_gpu_hybrid.py -m gpu -q --timeout 200 --timeout-method thread \
          -k "ray_angle" 2>&1 | grep -E "passed|failed|Error" | tail -3
      done ;;
    c2scan)
      echo "== C2 / C2 ray-angle batch scan"
      for bsz in 256 1024 4096 8192; do
        for res in reprojection ray_angle; do
          out=$(timeout -k 10 300 python3 bench.py --batch $bsz --views 2 --points 128 --no-distortion --residual $res \
                --cpu-sample 0 --parity-envelope 0 --no-live-counters --sustain-seconds 0 --steps 3 --warmup 1 2>&1 | tail -1) \
            || { echo "c2scan $bsz $res failed"; exit 1; }
          echo "B=$bsz $res $(echo "$out" | python3 -c 'import sys, json; d = json.loads(sys.stdin.read()); r = d["roofline"]; g = d["diagnostics"]["per_problem"]; print(d["value"], d["ms_per_step"], "frac", r["frac"], "evals p50/p99/max", [g["evaluations"][k] for k in ("p50", "p99", "max")])')"
        done
      done ;;
    c2waves)
      tools/ab.sh -r 2 -c "C2:--batch 1024 --views 2 --points 128 --no-distortion" \
        -c "C2b256:--batch 256 --views 2 --points 128 --no-distortion" \
        "w2:" "w4:DAVA_SOLVE_WAVES=4" 2>&1 | cut -c1-200 || exit 1 ;;
    extra)
      echo "== C3 at B = 65,536 on one GPU (the 8-GPU global batch)"
      timeout -k 10 400 python3 bench.py --batch 65536 --cpu-sample 0 --parity-envelope 0 --no-converged-parity \
        --no-live-counters --sustain-seconds 0 --steps 2 --warmup 1 > gpurun_out/extra_b65536.log 2>&1 || exit 1
      tail -1 gpurun_out/extra_b65536.log | cut -c1-200
      echo "== C3 solve + gradient at the reference's default cap (B = 4096, stopping rules)"
      timeout -k 10 400 python3 bench.py --batch 4096 --differentiate --iterations 1000 --error-threshold 1e-4 \
        --minimum-step 1e-8 --cpu-sample 0 --no-live-counters --sustain-seconds 0 --steps 2 --warmup 1 \
        > gpurun_out/extra_grad_defaults.log 2>&1 || exit 1
      tail -1 gpurun_out/extra_grad_defaults.log | cut -c1-200 ;;
    hybrid)
      echo "== hybrid fold"
      tools/hybrid_fold.sh > gpurun_out/hybrid_fold.jsonl || exit 1
      cat gpurun_out/hybrid_fold.jsonl ;;
    defaults)
      echo "== reference defaults (cap 1,000, stopping rules 1e-4 / 1e-8)"
      for cfg in "C2:--batch 1024 --views 2 --points 128 --no-distortion" "C3:" "C5:--batch 256 --views 16 --points 4096 --no-distortion"; do
        tag=${cfg%%:*}; args=${cfg#*:}
        timeout -k 10 300 python3 bench.py --iterations 1000 --error-threshold 1e-4 --minimum-step 1e-8 --cpu-sample 0 \
          --no-converged-parity --no-live-counters --sustain-seconds 0 --steps 2 --warmup 1 $args > gpurun_out/def_$tag.log 2>&1 \
          || { tail -5 gpurun_out/def_$tag.log; exit 1; }
        echo "{\"tag\": \"${tag}_defaults\", \"line\": $(tail -1 gpurun_out/def_$tag.log)}" >> gpurun_out/defaults.jsonl
        tail -1 gpurun_out/def_$tag.log | cut -c1-160
      done ;;
    profiles)
      tools/gpu_run.sh profile=r06_c3 "profile_cfg=r06_c2:--batch 1024 --views 2 --points 128 --no-distortion" \
        profile_c5=r06_c5 || exit 1 ;;
    diag)
      echo "== eval_bitwise"
      timeout -k 10 300 python3 tools/eval_bitwise.py 2>&1 | grep -v amdgpu.ids || exit 1
      tools/gpu_run.sh phase closure || exit 1 ;;
  esac
done
