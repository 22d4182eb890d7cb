#!/usr/bin/env python3
"""Copy one tools/round_evidence.sh run from gpurun_out/ into profiles/ (the
committed evidence), so every figure in profiles/ comes from the same box and
the same call.

    python tools/collect_evidence.py r02
"""
import json
import pathlib
import shutil
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
OUT, PROF = ROOT / "gpurun_out", ROOT / "profiles"


def first_json(path):
    for line in path.read_text().splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), tag, "--round", tag], check=True,
                   stdout=subprocess.DEVNULL)
    bench = first_json(OUT / "bench.log")
    (PROF / f"{tag}_bench.json").write_text(json.dumps(bench) + "\n")
    shutil.copy(OUT / f"prof_{tag}_kt.log", PROF / f"{tag}_bench_under_rocprof.log")
    for src, dst in (("sweep_kernel.csv", f"{tag}_sweep_quick.csv"), ("latency.csv", f"{tag}_latency_xgmi_w2_onegpu.csv"),
                     ("latency_rccl.csv", f"{tag}_latency_rccl_w2_onegpu.csv"), ("pytest_gpu.log", f"{tag}_pytest_gpu.log")):
        if (OUT / src).exists():
            shutil.copy(OUT / src, PROF / dst)
    for w in (2, 4, 8):
        if (OUT / f"bench_n{w}.log").exists():
            (PROF / f"{tag}_bench_n{w}_onegpu_rehearsal.json").write_text(
                json.dumps(first_json(OUT / f"bench_n{w}.log")) + "\n")
    for src, dst in (("host_direct.log", f"{tag}_host_direct_probe.txt"), ("gather.log", f"{tag}_gather_probe.txt"),
                     ("edge_lab.log", f"{tag}_edge_lab.txt")):
        if (OUT / src).exists():
            (PROF / dst).write_text("".join(l + "\n" for l in (OUT / src).read_text().splitlines()
                                            if "amdgpu.ids" not in l))
    if (OUT / "host_pipe.log").exists():
        (PROF / f"{tag}_host_pipe_probe.txt").write_text(
            "".join(l + "\n" for l in (OUT / "host_pipe.log").read_text().splitlines() if "amdgpu.ids" not in l))
    pmc = json.loads((PROF / f"{tag}_pmc.json").read_text())
    r = bench["roofline"]
    print(f"bench: value {bench['value']} GiB/s, kernel {r['kernel_mean_ms'] * 1e3:.2f} us = {r['achieved']} GB/s "
          f"({r['frac']:.1%}); stamped {r['kernel_stamped_mean_ms'] * 1e3:.2f} us; rocprof avg {pmc['avg_ns'] / 1e3:.2f} us "
          f"= {pmc['achieved_GBps_from_rocprof_avg']} GB/s; HBM/alg {pmc['hbm_over_algorithmic']}")


if __name__ == "__main__":
    main()
