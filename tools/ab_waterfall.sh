set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "C2:--batch 1024 --views 2 --points 128 --no-distortion" "C3:" "C1:--batch 8192 --views 2 --points 64 --no-distortion"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  echo "== $tag"
  BENCH_ARGS="$args --steps 3 --warmup 1" tools/ab_env.sh "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" "wf:" "prev:DAVA_LIB=@BUILD@/var_prev/libdava_ba.so" "wf:" || exit 1
done
