#!/usr/bin/env python3
"""EXPERIMENTS ONLY: a few launches of the shipped 8-source fold
(pgk_reduce_multi, double sum) for a rocprofv3 counter pass:

    rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python3 tools/lab/fold_pmc.py [MiB ...]
    rocprofv3 --pmc WRITE_SIZE ...                                    (each counter in its own pass)
    python tools/lab/fold_pmc.py --summary FETCH_DIR WRITE_DIR        (per-launch HBM bytes vs 9 x size)

Sources rotate over a 4 GiB pool.  HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB:
on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads.
"""
import csv
import ctypes
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
import re

# the fold's two forms: one tile (one 16-B vector per work-item per source) per
# wave, or the burst form with U vectors per work-item (from 32 MiB per source)
FORMS = re.compile(r"k_reduce_multi_(vec<double, 0, 8>|burst<double, 0, 8, (\d+)>)")


def summary(fetch_dir, write_dir):
    def rows(d, name):
        out = {}
        for r in csv.DictReader(open(pathlib.Path(d) / "run_counter_collection.csv")):
            m = FORMS.search(r["Kernel_Name"])
            if m and r["Counter_Name"] == name:
                per_item = int(m.group(2)) if m.group(2) else 1
                out.setdefault((m.group(0), int(r["Grid_Size"]) * 16 * per_item), []).append(float(r["Counter_Value"]))
        return out
    f, w = rows(fetch_dir, "FETCH_SIZE"), rows(write_dir, "WRITE_SIZE")
    res = []
    for kernel, size in sorted(f, key=lambda t: t[1]):
        key = (kernel, size)
        hbm = (2 * statistics.median(f[key]) + statistics.median(w[key])) * 1024
        res.append({"kernel": kernel, "MiB_per_source": size >> 20, "launches": [len(f[key]), len(w[key])],
                    "FETCH_SIZE_KiB_median": statistics.median(f[key]),
                    "WRITE_SIZE_KiB_median": statistics.median(w[key]),
                    "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes_per_launch": 9 * size,
                    "hbm_over_algorithmic": round(hbm / (9 * size), 4)})
    print(json.dumps(res, indent=1))


if len(sys.argv) > 1 and sys.argv[1] == "--summary":
    summary(sys.argv[2], sys.argv[3])
    sys.exit(0)

sys.path[:0] = [str(ROOT), str(ROOT / "rdma-ring-collectives_amd")]
import torch  # noqa: E402

import pgamd  # noqa: E402

lib = pgamd.load()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
POOL = 4 << 30
pool = torch.empty(POOL // 8, dtype=torch.float64, device="cuda").uniform_(-1, 1)
VP = ctypes.c_void_p
for mib in [int(a) for a in sys.argv[1:]] or [16, 32, 64]:
    size = mib << 20
    sets = POOL // (9 * size)
    for k in range(12):
        b0 = pool.data_ptr() + 9 * size * (k % sets)
        srcs = (VP * 8)(*[b0 + size * j for j in range(8)])
        pgamd.check(lib.pgk_reduce_multi(b0 + 8 * size, srcs, 8, size // 8, 1, 0, sh), "fold")
    torch.cuda.synchronize()
    print(f"{mib} MiB x 8: 12 launches", flush=True)
