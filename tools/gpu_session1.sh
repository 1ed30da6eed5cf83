#!/bin/bash
# GPU suite + LDS-history A/B (run on the GPU box from the repo root)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc   # fault / abort / timeout: start nothing more on the GPU
tools/ab_env.sh "lds_default:" "lds0:DAVA_LDS_HISTORY=0" "lds18:DAVA_LDS_HISTORY=18" "lds12:DAVA_LDS_HISTORY=12" \
  "nosweep:DAVA_LIB=$PWD/deep-attention-visual-odometry_amd/build/var_nosweep/libdava_ba.so DAVA_LDS_HISTORY=0" \
  > gpurun_out/ab1.log 2>&1
rc2=$?
cat gpurun_out/ab1.log
exit $(( rc > rc2 ? rc : rc2 ))
