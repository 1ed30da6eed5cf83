set -uo pipefail
mkdir -p gpurun_out
: > gpurun_out/c2_scan.jsonl
for b in 64 256 512 1024 2048; do
  timeout -k 10 200 python3 bench.py --cpu-sample 0 --batch $b --views 2 --points 128 --no-distortion --steps 5 --warmup 2 > gpurun_out/c2_$b.log 2>&1 || { tail -5 gpurun_out/c2_$b.log; exit 1; }
  echo "{\"b\": $b, \"line\": $(tail -1 gpurun_out/c2_$b.log)}" >> gpurun_out/c2_scan.jsonl
done
