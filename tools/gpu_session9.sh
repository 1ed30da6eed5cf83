#!/bin/bash
# rocprofv3 profile of the default C3 kernel, then an interleaved A/B of build variants
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/deep-attention-visual-odometry_amd/build
tools/profile.sh r01b_c3 > gpurun_out/prof_r01b.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/prof_r01b.log; exit 1; }
tail -1 gpurun_out/prof_r01b.log
tools/ab_env.sh "c3:" "w3fp0:DAVA_LIB=$V/var_w3fp0/libdava_ba.so" "noslp:DAVA_LIB=$V/var_noslp/libdava_ba.so" \
  "dot:DAVA_LIB=$V/var_dot/libdava_ba.so" "fp0:DAVA_LIB=$V/var_fp0/libdava_ba.so" \
  "c3:" "w3fp0:DAVA_LIB=$V/var_w3fp0/libdava_ba.so" "noslp:DAVA_LIB=$V/var_noslp/libdava_ba.so" \
  "dot:DAVA_LIB=$V/var_dot/libdava_ba.so" "fp0:DAVA_LIB=$V/var_fp0/libdava_ba.so"
