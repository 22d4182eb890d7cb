#!/usr/bin/env python3
"""Summarise rocprofv3 passes of bench.py into profiles/ (committed evidence).

    python tools/pmc_traffic.py TAG [--round r01]

Reads gpurun_out/prof_TAG_{kt,fetch,write}/ and writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<round>_pmc.json           per-launch HBM bytes of the reduce kernel
  profiles/pmc_traffic.json           the figure bench.py reports as roofline.traffic

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a
16-B-per-lane coalesced streaming read (MI355X_MICROARCH.md §HBM), WRITE_SIZE
is exact for 16-B-per-lane streaming stores.
"""
import argparse
import csv
import json
import pathlib
import shutil
import statistics

ROOT = pathlib.Path(__file__).resolve().parents[1]
KERNEL = "k_reduce_vec<double, 0"
N_ELEMS = 1 << 25


def counter(path, name):
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
    return [float(r["Counter_Value"]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--round", default="r01")
    a = ap.parse_args()
    out = ROOT / "gpurun_out"
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    kt = out / f"prof_{a.tag}_kt" / "run_kernel_stats.csv"
    shutil.copy(kt, prof / f"{a.round}_kernel_stats.csv")
    stats = [r for r in csv.DictReader(open(kt)) if KERNEL in r["Name"]][0]
    fetch = counter(out / f"prof_{a.tag}_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    write = counter(out / f"prof_{a.tag}_write" / "run_counter_collection.csv", "WRITE_SIZE")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    hbm = (2 * f_kib + w_kib) * 1024
    alg = 3 * N_ELEMS * 8
    avg_ns = float(stats["AverageNs"])
    summary = {
        "kernel": stats["Name"], "dispatches": int(stats["Calls"]), "avg_ns": avg_ns,
        "min_ns": float(stats["MinNs"]), "max_ns": float(stats["MaxNs"]),
        "achieved_GBps_from_rocprof_avg": round(alg / avg_ns, 1),
        "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib,
        "pmc_dispatches": [len(fetch), len(write)],
        "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes_per_launch": alg,
        "hbm_over_algorithmic": round(hbm / alg, 4),
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950 FETCH_SIZE halving)",
        "command": "rocprofv3 ... -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10",
    }
    (prof / f"{a.round}_pmc.json").write_text(json.dumps(summary, indent=1) + "\n")
    (prof / "pmc_traffic.json").write_text(json.dumps({"reduce_f64_sum_256MiB": {
        "hbm_bytes_per_launch": round(hbm), "source": f"profiles/{a.round}_pmc.json"}}, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
