#!/bin/bash
# One parameterised GPU-box session (run via gpurun from the repo root).  Each argument is a step,
# run in order; the first failing step ends the session (no GPU step runs after a failure).
#   tests[=PYTEST_ARGS]   pytest -m gpu (default: the whole suite); e.g. 'tests=-k "golden or headline"' 
#   smoke                 __graft_entry__.smoke()
#   bench[=BENCH_ARGS]    python bench.py (default flags) -> gpurun_out/bench.log
#   configs               tools/measure_configs.sh (one bench line per configuration)
#   profile=TAG           tools/profile.sh TAG (kernel trace + FETCH_SIZE + WRITE_SIZE passes, C3)
#   profile_c5=TAG        tools/profile.sh TAG on the C5 configuration
#   profile_cfg=TAG:ARGS  tools/profile.sh TAG with bench ARGS (e.g. the C2 configuration)
#   sq=TAG[:BENCH_ARGS]   tools/pmc_sq.sh (SQ busy/VALU/MFMA counters) for a configuration
#   micro=P               tools/micro/solve_pass_stream P (the history pass alone; P > 512: the headline's rows)
#   eval=TAG              tools/eval_sweep.py (C3, C5) + tools/profile_eval.sh TAG for both
#   ab=SPEC;SPEC...       tools/ab_env.sh with the given specs (BENCH_ARGS from the environment)
#   phase                 tools/phase_scan.sh (needs build/var_phase: make variant NAME=phase FLAGS=-DDAVA_PHASE_TIMING=1)
#   closure               tools/closure_scan.sh (bench --entry closure: compact vs dense generic loop, C2 and C3)
# usage: tools/gpu_run.sh tests smoke bench profile=r02a
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() { echo "== $* ($(date +%T))"; }
for s in "$@"; do
  name=${s%%=*}
  val=${s#*=}
  [ "$val" = "$s" ] && val=""
  case $name in
    tests)
      step tests "$val"
      # PYTEST_ARGS may quote a -k expression: tests='-k "a or b"'
      eval "timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${val}" \
        > gpurun_out/tests.log 2>&1
      rc=$?; grep -E "passed|failed|error" gpurun_out/tests.log | tail -3
      [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/tests.log | head -20; exit $rc; } ;;
    smoke)
      step smoke
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail -5 gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      step bench "$val"
      timeout -k 10 500 python3 bench.py ${val} > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
      tail -1 gpurun_out/bench.log | cut -c1-600 ;;
    configs)
      step configs
      tools/measure_configs.sh || exit 1 ;;
    profile)
      step profile "$val"
      tools/profile.sh "$val" > gpurun_out/prof_$val.log 2>&1 || { tail -5 gpurun_out/prof_$val.log; exit 1; }
      tail -1 gpurun_out/prof_$val.log ;;
    profile_c5)
      step profile_c5 "$val"
      tools/profile.sh "$val" --batch 256 --views 16 --points 4096 --no-distortion --steps 2 --warmup 1 \
        > gpurun_out/prof_$val.log 2>&1 || { tail -5 gpurun_out/prof_$val.log; exit 1; }
      tail -1 gpurun_out/prof_$val.log ;;
    profile_cfg)
      step profile_cfg "$val"
      tag=${val%%:*}; args=${val#*:}
      tools/profile.sh "$tag" $args > gpurun_out/prof_$tag.log 2>&1 || { tail -5 gpurun_out/prof_$tag.log; exit 1; }
      tail -1 gpurun_out/prof_$tag.log ;;
    micro)
      step micro "$val"
      timeout -k 10 300 tools/micro/solve_pass_stream "$val" > gpurun_out/micro_$val.log 2>&1 \
        || { tail -5 gpurun_out/micro_$val.log; exit 1; }
      cat gpurun_out/micro_$val.log ;;
    eval)
      step eval "$val"
      timeout -k 10 300 python3 tools/eval_sweep.py > gpurun_out/eval_sweep_$val.jsonl 2>gpurun_out/eval_sweep_$val.err \
        || { tail -5 gpurun_out/eval_sweep_$val.err; exit 1; }
      cut -c1-400 gpurun_out/eval_sweep_$val.jsonl
      for c in C3 C5; do
        tools/profile_eval.sh "$val" $c > gpurun_out/prof_eval_${val}_$c.log 2>&1 || { tail -5 gpurun_out/prof_eval_${val}_$c.log; exit 1; }
      done ;;
    sq)
      step sq "$val"
      tag=${val%%:*}; args=${val#*:}; [ "$args" = "$val" ] && args=""
      tools/pmc_sq.sh "$tag" $args > gpurun_out/sq_$tag.log 2>&1 || { tail -5 gpurun_out/sq_$tag.log; exit 1; }
      tail -3 gpurun_out/sq_$tag.log ;;
    phase)
      step phase
      tools/phase_scan.sh > gpurun_out/phase_scan.log 2>&1 || { tail -5 gpurun_out/phase_scan.log; exit 1; }
      cut -c1-300 gpurun_out/phase_scan.log ;;
    closure)
      step closure "$val"
      tools/closure_scan.sh > gpurun_out/closure.jsonl 2> gpurun_out/closure.err || { tail -5 gpurun_out/closure.err; exit 1; }
      cut -c1-400 gpurun_out/closure.jsonl ;;
    ab)
      step ab "$val"
      IFS=';' read -ra specs <<< "$val"
      tools/ab_env.sh "${specs[@]}" || exit 1 ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
