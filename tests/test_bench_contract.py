"""The committed bench line (profiles/r02_bench.json, printed by bench.py on
MI355X) keeps the driver's contract: BASELINE.json's metric, the required keys,
a roofline object whose fraction is its own achieved/peak, and a CPU baseline
naming its sample and core count.  The PMC traffic it carries must come from
profiles/pmc_traffic.json, and the N>1 rehearsal lines must carry a ring leg
whose device-side checks all passed."""
import json

import pytest

from conftest import ROOT

PROF = ROOT / "profiles"
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _line(name):
    return json.loads((PROF / name).read_text().splitlines()[0])


def test_bench_line_keys_and_metric():
    line = _line("r02_bench.json")
    base = json.loads((ROOT / "BASELINE.json").read_text())
    for k in REQUIRED:
        assert k in line, k
    assert line["metric"] == base["metric"]
    assert line["n_gpus"] == 1 and line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["vs_baseline"] is None and not base["published"]
    assert "workload" in line["config"] and line["value"] > 0


def test_roofline_is_self_consistent():
    line = _line("r02_bench.json")
    r = line["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-4)
    # achieved = algorithmic bytes per launch / mean launch time
    assert r["achieved"] == pytest.approx(r["bytes_per_launch"] / (r["kernel_mean_ms"] * 1e-3) / 1e9, rel=1e-3)
    assert r["bytes_per_launch"] == 3 * (256 << 20)
    traffic = json.loads((PROF / "pmc_traffic.json").read_text())
    assert r["traffic"] is not None and 0.99 < r["traffic"] / r["bytes_per_launch"] < 1.05
    # the line carries the PMC figure of the preceding counter pass (bench.py reads pmc_traffic.json)
    pmc = traffic["reduce_f64_sum_256MiB"]["hbm_bytes_per_launch"]
    assert r["traffic"] == pytest.approx(pmc, rel=1e-4)


def test_cpu_baseline_names_its_sample():
    cpu = _line("r02_bench.json")["cpu_baseline"]
    assert cpu["kind"] in ("reference", "port") and cpu["cores"] >= 1 and cpu["value"] > 0
    assert cpu["sample"] and cpu["unit"]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rehearsal_lines_checked_out(world):
    line = _line(f"r02_bench_n{world}_onegpu_rehearsal.json")
    assert line["n_gpus"] == world and line["metric"] == _line("r02_bench.json")["metric"]
    ring = line["ring"]
    legs = [v for v in ring.values() if isinstance(v, dict)]
    assert legs and all(v.get("ok") is True for v in legs)
    assert all(v.get("host_buffers_ok", True) is True for v in legs)
    # every transport ran, the RCCL ring included, and nothing was redone
    assert {"xgmi", "rccl"} <= set(ring)
    for v in legs:
        for row in v.get("config5_prod_mixed", []):
            assert row["ok"] is True
        phases = v.get("last_call_phases", {})
        assert phases.get("redone") is False and phases.get("calls_redone_total") == 0
        small = v.get("eager_4KiB")
        if small:
            assert small["reduce_scatter"]["ok"] and small["all_reduce"]["ok"]
        nat = v.get("rccl_native")
        if isinstance(nat, dict):
            assert nat["i32_sum_bit_exact"] and nat["f64_sum_within_tol"]
            # product rows were added after the round-2 rehearsals; checked when present
            assert nat.get("i32_prod_bit_exact", True) and nat.get("f64_prod_within_tol", True)
            assert nat.get("i32_all_reduce_bit_exact", True) and nat.get("i32_all_gather_bit_exact", True)


def test_batch_launch_at_defaults_above_70_percent():
    """The executor's reduce launch at the library defaults (4 MiB x 4
    inflight x 2 rings, one pgk_reduce_ranges launch) keeps >= 70% of the HBM
    peak, and the size table starts at the in-ring sizes."""
    ks = _line("r02_bench.json")["kernel_sizes"]
    assert {r[2] for r in ks["rows"]} >= {4 << 20, 16 << 20, 32 << 20, 64 << 20}
    first = ks["ring_batches"]["rows"][0]
    assert first[:3] == [4 << 20, 4, 2]
    assert first[5] >= 0.70 and first[7] >= 0.70


# ---- the r03_* lines: the same contract, plus the sweeps on both schedules, the clocks and the data path ----

def test_r03_bench_line_contract():
    line = _line("r03_bench.json")
    base = json.loads((ROOT / "BASELINE.json").read_text())
    for k in REQUIRED + ("elapsed_s", "time_budget_s"):
        assert k in line, k
    assert line["metric"] == base["metric"] and line["n_gpus"] == 1 and line["vs_baseline"] is None
    r = line["roofline"]
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-4) and r["peak"] == 8000.0
    assert r["achieved"] == pytest.approx(r["bytes_per_launch"] / (r["kernel_mean_ms"] * 1e-3) / 1e9, rel=1e-3)
    pmc = json.loads((PROF / "pmc_traffic.json").read_text())["reduce_f64_sum_256MiB"]["hbm_bytes_per_launch"]
    assert r["traffic"] == pytest.approx(pmc, rel=1e-4) and 0.99 < r["traffic"] / r["bytes_per_launch"] < 1.05
    cpu = line["cpu_baseline"]
    assert cpu["kind"] in ("reference", "port") and cpu["cores"] >= 1 and cpu["value"] > 0 and cpu["sample"]
    # every leg is clocked and the whole run fits the budget it was given
    el = line["elapsed_s"]
    assert {"kernel_sizes", "kernel_leg", "cpu_baseline", "total"} <= set(el)
    assert el["total"] <= line["time_budget_s"]


def test_r03_executor_launch_at_defaults():
    """The reduce launch the ring executor makes at the library defaults
    (PG_REDUCE_BYTES = 128 MiB pending over two rings, one pgk_reduce_ranges
    launch) reaches 78% of the HBM peak kernel-stamped; the single transport
    group it replaced (4 MiB x 4 x 2 rings) is kept beside it."""
    ks = _line("r03_bench.json")["kernel_sizes"]
    cols = ks["ring_batches"]["columns"]
    first, group = ks["ring_batches"]["rows"][0], ks["ring_batches"]["rows"][1]
    assert first[cols.index("bytes_per_operand")] == 128 << 20 and first[cols.index("rings")] == 2
    assert first[cols.index("stamped_frac")] >= 0.78 and first[cols.index("frac")] >= 0.78
    assert group[cols.index("bytes_per_operand")] == 32 << 20
    assert first[cols.index("frac")] > group[cols.index("frac")]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_r03_rehearsal_lines_checked_out(world):
    line = _line(f"r03_bench_n{world}_onegpu_rehearsal.json")
    assert line["n_gpus"] == world and line["metric"] == _line("r03_bench.json")["metric"]
    assert line["elapsed_s"]["total"] <= line["time_budget_s"]
    ring = line["ring"]
    assert {"xgmi", "rccl"} <= set(ring)
    legs = [v for v in ring.values() if isinstance(v, dict) and "skipped" not in v]
    assert legs and all(v.get("ok") is True for v in legs)
    for name, v in ring.items():
        if not isinstance(v, dict) or "skipped" in v:
            continue
        assert f"ring.{name}" in line["elapsed_s"]
        phases = v["last_call_phases"]
        assert phases["redone"] is False and phases["calls_redone_total"] == 0
        # the library itself names the data path that ran
        assert phases["path"]["transport"] == ("xgmi" if name.startswith("xgmi") else "rccl")
        assert v["in_ring_reduce"]["launches_per_rank"] >= 1
        for key in ("config5_prod_mixed", "eager_4KiB", "rccl_native", "host_buffers"):
            part = v.get(key)
            if part is None or (isinstance(part, dict) and "skipped" in part):
                continue
            if key == "config5_prod_mixed":
                assert all(row["ok"] is True for row in part)
            elif key == "eager_4KiB":
                assert part["reduce_scatter"]["ok"] and part["all_reduce"]["ok"]
            elif key == "host_buffers":
                assert part["ok"] is True
            else:
                assert part["i32_sum_bit_exact"] and part["f64_sum_within_tol"]
                assert part["i32_prod_bit_exact"] and part["f64_prod_within_tol"]
                assert part["i32_all_reduce_bit_exact"] and part["i32_all_gather_bit_exact"]


@pytest.mark.parametrize("world,key,knob", [(4, "chunk_sweep", "chunk_bytes"), (8, "inflight_sweep", "inflight")])
def test_r03_sweeps_cover_both_schedules(world, key, knob):
    """BASELINE configs 3 and 4 name a ring with a PG_CHUNK_BYTES / PG_INFLIGHT
    sweep: every committed sweep row names its schedule (`algo`), both the W-1
    round ring and the direct exchange are swept over every value, and each row
    carries the roofline fraction of the reduce launches inside it.  A row
    without `algo` fails here."""
    sw = _line(f"r03_bench_n{world}_onegpu_rehearsal.json")["ring"]["rccl"][key]
    cols = sw["columns"]
    assert cols[:5] == ["size", "rounds", "inflight", "time_us", "GB/s"]     # reference README.md:85
    for need in ("chunk_bytes", "is_default", "algo", "in_ring_reduce_frac"):
        assert need in cols, need
    a, k, f = cols.index("algo"), cols.index(knob), cols.index("in_ring_reduce_frac")
    for row in sw["rows"]:
        assert len(row) == len(cols) and row[a] in ("ring", "direct"), row
        assert 0.0 < row[f] <= 1.0, row
    values = {1 << e for e in range(16, 29)} if knob == "chunk_bytes" else {1, 2, 4, 8, 16}
    for algo in ("ring", "direct"):
        assert {row[k] for row in sw["rows"] if row[a] == algo} == values, algo
        assert sum(row[cols.index("is_default")] for row in sw["rows"] if row[a] == algo) == 1
    assert set(sw["by_algo"]) == {"ring", "direct"} and sw["truncated_by_time_budget"] is False


@pytest.mark.parametrize("world", [2, 4, 8])
def test_r03_rehearsals_ran_their_preflight(world):
    """At N > 1 each rank's first exchange on every transport happens in a child
    process before the measuring process touches the GPU; the line records what
    the children found and how long they took."""
    line = _line(f"r03_bench_n{world}_onegpu_rehearsal.json")
    assert line["ring_preflight"] == {t: "ok" for t in ("xgmi", "xgmi_push", "xgmi_read", "rccl")}
    assert 0 < line["elapsed_s"]["ring.preflight"] < 60


def test_r03_refused_preflight_costs_only_that_transport():
    """The same run with the xgmi reach check forced to fail (PG_XGMI_FAIL_REACH
    = -1, no fault involved): the xgmi legs are recorded as not run, with the
    child's reason, the rccl leg and the primary line are there as ever."""
    line = _line("r03_bench_n2_preflight_refused.json")
    pf = line["ring_preflight"]
    assert pf["rccl"] == "ok" and "cannot map a peer's device memory" in pf["xgmi"]
    assert line["ring"]["xgmi"]["error"].startswith("no leg: preflight failed")
    assert line["ring"]["xgmi_push"]["error"].startswith("no leg: preflight failed")
    assert line["ring"]["rccl"]["ok"] is True and line["value"] > 0
