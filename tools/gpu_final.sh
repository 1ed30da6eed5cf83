#!/bin/bash
# End-of-round evidence: full GPU suite, smoke, default bench (with CPU baseline), every
# configuration, rocprofv3 kernel trace + PMC traffic of the default C3 launch.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/final_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-300
tools/measure_configs.sh || exit 1
TAG=${1:-r01d}
tools/profile.sh ${TAG}_c3 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log
