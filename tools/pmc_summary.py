"""Summarise a tools/profile.sh run into profiles/ (tracked).

usage: python tools/pmc_summary.py gpurun_out/prof_TAG TAG KEY
  KEY = the bench configuration key (e.g. dense_B8192_M4_N256_D1_K100) that
        bench.py looks up in profiles/pmc_traffic.json.

HBM bytes per launch of the solve kernel = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a
wide coalesced (16 B/lane) streaming read (MI355X_MICROARCH.md, HBM section), which
is exactly the access pattern of the inverse-Hessian sweep; WRITE_SIZE is exact for
16 B/lane streaming stores.
"""
import csv
import json
import os
import shutil
import sys

KERNEL = "bfgs_ba_solve_kernel"


def rows(path):
    with open(path) as fh:
        return list(csv.DictReader(fh))


def main():
    src, tag, key = sys.argv[1:4]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(repo, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    trace = [r for r in rows(os.path.join(src, "kt", "kt_kernel_trace.csv")) if KERNEL in r["Kernel_Name"]]
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
    fetch = [float(r["Counter_Value"]) for r in rows(os.path.join(src, "fetch", "fetch_counter_collection.csv"))
             if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    write = [float(r["Counter_Value"]) for r in rows(os.path.join(src, "write", "write_counter_collection.csv"))
             if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE"]
    fetch_b = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    meta = trace[0]
    summary = {
        "tag": tag,
        "kernel": meta["Kernel_Name"],
        "launches_traced": len(dur),
        "avg_duration_ms": sum(dur) / len(dur) / 1e6,
        "vgpr": meta.get("VGPR_Count"), "sgpr": meta.get("SGPR_Count"), "lds_bytes": meta.get("LDS_Block_Size"),
        "grid": meta.get("Grid_Size"), "workgroup": meta.get("Workgroup_Size"),
        "fetch_size_kib_raw": sum(fetch) / len(fetch),
        "write_size_kib_raw": sum(write) / len(write),
        "hbm_read_bytes_per_launch": fetch_b,
        "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "correction": "read = 2 x FETCH_SIZE (gfx950 16 B/lane stream), write = WRITE_SIZE; KiB -> bytes",
    }
    with open(os.path.join(dst, f"{tag}_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=2)
    tj_path = os.path.join(dst, "pmc_traffic.json")
    tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
    import datetime

    tj[key] = {"tag": tag, "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
               "avg_duration_ms": summary["avg_duration_ms"],
               "date": datetime.date.today().isoformat()}
    with open(tj_path, "w") as fh:
        json.dump(tj, fh, indent=2, sort_keys=True)
    print(json.dumps(summary, indent=2))


if __name__ == "__main__":
    main()
