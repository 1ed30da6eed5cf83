#!/bin/bash
# wave priority default: bitwise check against the build without it, full GPU suite, A/B
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
timeout -k 10 200 python3 tools/dump_solve.py gpurun_out/d_new.npz 2>/dev/null &&
DAVA_LIB=$V/var_prev/libdava_ba.so timeout -k 10 200 python3 tools/dump_solve.py gpurun_out/d_prev.npz 2>/dev/null &&
python3 tools/dump_solve.py --compare gpurun_out/d_new.npz gpurun_out/d_prev.npz || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s18_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s18_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_env.sh "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" "c3:" "c3prev:DAVA_LIB=$V/var_prev/libdava_ba.so" || exit 1
