#!/usr/bin/env python3
"""Print the figures of one round's committed evidence (profiles/<tag>_*.json)
in the wording of DESIGN.md's results table, so that the table is copied from
the files and not retyped.

    python tools/results_table.py r03
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
PROF = ROOT / "profiles"
tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
b = json.loads((PROF / f"{tag}_bench.json").read_text())
pmc = json.loads((PROF / f"{tag}_pmc.json").read_text())
r = b["roofline"]
pct = lambda x: f"{100 * x:.1f}%"          # noqa: E731
print(f"kernel: {r['kernel_mean_ms'] * 1e3:.2f} us mean launch -> {r['achieved']:.0f} GB/s = {pct(r['frac'])}")
print(f"stamped: {r['kernel_stamped_mean_ms'] * 1e3:.2f} us mean, {r['kernel_stamped_min_ms'] * 1e3:.2f} us min")
print(f"rocprof: {pmc['avg_ns'] / 1e3:.2f} us avg = {pmc['achieved_GBps_from_rocprof_avg']:.0f} GB/s, "
      f"{abs(pmc['avg_ns'] / 1e6 - r['kernel_mean_ms']) / r['kernel_mean_ms']:.1%} from the bench's events; "
      f"min {pmc['min_ns'] / 1e3:.2f}, max {pmc['max_ns'] / 1e3:.2f} us; {pmc['dispatches']} dispatches")
print(f"PMC: {pmc['hbm_bytes_per_launch']:,} B = {pmc['hbm_over_algorithmic']:.4f}x")
print(f"value: {b['value']:.0f} GiB/s traffic = {b['payload_gibs']:.0f} GiB/s payload")
s = b.get("kernel_sustained")
if s:
    print(f"sustained: {s['launches']} launches in {s['seconds']} s: median {pct(s['frac_median'])}, slowest window "
          f"{pct(s['frac_min'])}, first {pct(s['frac_first_window'])}, last {pct(s['frac_last_window'])}")
ks = b["kernel_sizes"]
for dt, op in (("f64", "sum"), ("i32", "sum"), ("f64", "prod"), ("i32", "prod")):
    rows = [x for x in ks["rows"] if x[0] == dt and x[1] == op]
    print(f"{dt} {op}: " + ", ".join(f"{x[2] >> 20} MiB {pct(x[5])} / {pct(x[7])}" for x in rows))
print("edge_fit:", ks["edge_fit"])
for key in ("ring_batches", "direct_batches"):
    for x in ks[key]["rows"]:
        print(f"{key}: {x[0]}: {pct(x[4])} / {pct(x[6])} ({x[3]} / {x[5]} us)")
c = b["cpu_baseline"]
print(f"cpu: {c['value']} GiB/s traffic ({c['payload_gibs']} payload), GPU/CPU {b['value'] / c['value']:.0f}x; "
      f"concurrent {c['concurrent']['aggregate_gibs']} ({c['concurrent']['per_proc_min_gibs']}-"
      f"{c['concurrent']['per_proc_max_gibs']}) on cores {c['concurrent']['cores']}")
print("config1:", b["config1"])
h = b["host_staged"]
print(f"host: pinned {h['pinned']['ms']} ms = {h['pinned']['pcie_gbs']} GB/s; pageable {h['pageable']['ms']} ms = "
      f"{h['pageable']['pcie_gbs']} GB/s")
print("elapsed:", b["elapsed_s"])
for w in (2, 4, 8):
    p = PROF / f"{tag}_bench_n{w}_onegpu_rehearsal.json"
    if not p.exists():
        continue
    l = json.loads(p.read_text())
    ring = l["ring"]
    print(f"N={w}: total {l['elapsed_s']['total']} s; " + "; ".join(
        f"{k} ok={v.get('ok')} {v.get('ms_per_reduce_scatter')} ms" for k, v in ring.items() if isinstance(v, dict)))
    rc = ring.get("rccl", {})
    for key in ("chunk_sweep", "inflight_sweep"):
        if key in rc:
            print(f"   {key}: {len(rc[key]['rows'])} rows, by_algo {rc[key]['by_algo']}, "
                  f"elapsed {l['elapsed_s'].get('ring.rccl.' + key)} + ring_algo {l['elapsed_s'].get('ring.rccl.ring_algo')} s")
    for key in ("ring_algo", "one_ring", "four_rings"):
        if key in rc and "ms_per_reduce_scatter" in rc[key]:
            print(f"   {key}: {rc[key]['ms_per_reduce_scatter']} ms")
    if "rccl_native" in rc and isinstance(rc["rccl_native"], dict):
        n = rc["rccl_native"]
        print(f"   rccl_native: rccl's own {n.get('rccl_reduce_scatter_ms')} ms; f64 prod max diff/tol "
              f"{n.get('f64_prod_max_diff_over_tol')}, bit-identical {n.get('f64_prod_bit_identical_frac')}")
    x = ring.get("xgmi", {})
    if "last_call_phases" in x:
        print("   xgmi path:", x["last_call_phases"]["path"])
