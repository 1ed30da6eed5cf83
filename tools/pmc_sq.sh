#!/bin/bash
# SQ instruction-mix / stall counters of the solve kernel (one rocprofv3 pass per counter set).
# usage: tools/pmc_sq.sh TAG [bench args...]    -> gpurun_out/sq_TAG/{a,b}/...
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES"
i=0
for set in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/bench.py" --cpu-sample 0 --steps 1 --warmup 0 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bfgs_ba_solve_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k:24s} {v:.4g}")
PY
