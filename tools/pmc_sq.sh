#!/bin/bash
# SQ instruction-mix / stall / VALU / MFMA counters of the solve kernel (one rocprofv3 pass per set,
# kernel trace only -- no sys/runtime traces with --pmc, as the pool requires).
# usage: tools/pmc_sq.sh TAG [bench args...]    -> gpurun_out/sq_TAG/p{1,2,3}/..., summary on stdout
#        KERNEL=ba_evaluate_kernel PROG=tools/eval_sweep.py tools/pmc_sq.sh TAG [prog args...]
#        (another program and kernel: PROG runs with the given args instead of bench.py's)
set -uo pipefail
KERNEL=${KERNEL:-bfgs_ba_solve_kernel}
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES"
C="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for set in "$A" "$B" "$C"; do
  i=$((i+1))
  if [ -n "${PROG:-}" ]; then
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o p$i --output-format csv -- \
      python3 "$R/$PROG" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  else
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o p$i --output-format csv -- \
      python3 "$R/bench.py" --cpu-sample 0 --no-live-counters --sustain-seconds 0 --steps 1 --warmup 0 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  fi
done
python3 - "$OUT" "$KERNEL" <<'PY'
import csv, glob, sys, collections
out, kernel = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float)
launches = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            launches[f].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
n = max((len(v) for v in launches.values()), default=1)
print(f"kernel {kernel}: counters summed over {n} launch(es) per pass (divide by it for per-launch figures)")
for k, v in sorted(tot.items()):
    print(f"{k:28s} {v:.4g}")
CUS, SIMDS, XCDS = 256, 1024, 8
gui = tot.get("GRBM_GUI_ACTIVE", 0.0) / XCDS  # rocprofv3 sums GRBM over the 8 XCDs; the formulas want the max
if gui > 0:
    print("derived (rocprofv3's gfx94x formulas, GRBM_GUI_ACTIVE / 8 XCDs as the per-XCD max):")
    print(f"  VALUBusy %          {100 * tot.get('SQ_ACTIVE_INST_VALU', 0) / CUS / gui:.1f}")
    print(f"  MfmaUtil %          {100 * tot.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gui * SIMDS):.3f}")
    print(f"  kernel clock cycles {gui:.4g}")
if tot.get("SQ_ACTIVE_INST_VALU"):
    print(f"  VALUUtilization %   {100 * tot.get('SQ_THREAD_CYCLES_VALU', 0) / (tot['SQ_ACTIVE_INST_VALU'] * 64):.1f}  (active lanes per VALU instruction)")
if tot.get("SQ_WAVE_CYCLES"):
    w = tot["SQ_WAVE_CYCLES"]
    print(f"  wave cycles: waiting {100 * tot.get('SQ_WAIT_ANY', 0) / w:.1f}%  issue-stalled "
          f"{100 * tot.get('SQ_WAIT_INST_ANY', 0) / w:.1f}%  issuing {100 * tot.get('SQ_ACTIVE_INST_ANY', 0) / w:.1f}%")
PY
