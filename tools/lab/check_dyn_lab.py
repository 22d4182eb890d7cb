#!/usr/bin/env python3
"""EXPERIMENTS ONLY: results of tools/lab/dyn_lab.hip's (or, with --lab wgt,
wgt_lab.hip's) variants against torch (dst + src), at ragged and full sizes,
and the ticket counters back at zero after every launch.  Prints one line per
variant and size; exits 1 on a mismatch.

    python tools/lab/check_dyn_lab.py [--lab dyn|wgt] [name filter]"""
import ctypes
import pathlib
import sys

import torch

HERE = pathlib.Path(__file__).resolve().parent
LAB = "dyn"
if "--lab" in sys.argv:
    i = sys.argv.index("--lab")
    LAB = sys.argv[i + 1]
    del sys.argv[i:i + 2]
lab = ctypes.CDLL(str(HERE / f"lib{LAB}lab.so"))
lab.edge_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_void_p]
lab.edge_name.restype = ctypes.c_char_p
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
bad = 0
only = sys.argv[1] if len(sys.argv) > 1 else ""
for v in range(64):
    name = lab.edge_name(v)
    if not name:
        break
    name = name.decode()
    if only not in name:
        continue
    for n in (2, 2048, 4094, 4096 + 2 * 17, 1 << 20, (1 << 20) + 2 * 777, 3 * (1 << 22) + 2 * 5, 1 << 25):
        x = torch.rand(n, dtype=torch.float64, device="cuda")
        y = torch.rand(n, dtype=torch.float64, device="cuda")
        ref = x + y
        for rep in range(3):                    # the counters must reset between launches
            d = x.clone()
            rc = lab.edge_launch(v, d.data_ptr(), y.data_ptr(), n, sh, None, None)
            torch.cuda.synchronize()
            ok = rc == 0 and torch.equal(d, ref) and lab.dyn_counters_clear() == 1
            if not ok:
                bad += 1
                print(f"FAIL {name} n={n} rep={rep} rc={rc} clear={lab.dyn_counters_clear()}", flush=True)
                break
        else:
            print(f"ok   {name} n={n}", flush=True)
sys.exit(1 if bad else 0)
