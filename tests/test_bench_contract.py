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
    # round 2: every transport ran, the RCCL ring included, and nothing was redone
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
