import os, sys, time, pathlib, ctypes, subprocess
R = pathlib.Path.cwd()
sys.path[:0] = [str(R), str(R / "rdma-ring-collectives_amd")]
import torch, pgamd
lib = pgamd.load()
n = 1 << 25
for th in ("1", "2", "4", "8"):
    out = subprocess.run([sys.executable, "-c", f"""
import os,sys,time,torch
os.environ['PG_COPY_THREADS']='{th}'
sys.path[:0]=['{R}','{R}/rdma-ring-collectives_amd']
import pgamd
lib=pgamd.load()
n={n}
d=torch.rand(n,dtype=torch.float64); s=torch.rand(n,dtype=torch.float64)
lib.pgx_reduce_host(d.data_ptr(), s.data_ptr(), n, 1, 0, 0)
t=time.perf_counter()
for _ in range(3): lib.pgx_reduce_host(d.data_ptr(), s.data_ptr(), n, 1, 0, 0)
dt=(time.perf_counter()-t)/3
print('threads {th}: %.2f ms  pcie %.1f GB/s' % (dt*1e3, 3*n*8/dt/1e9))
"""], capture_output=True, text=True)
    print(out.stdout.strip(), out.stderr.strip()[-200:] if out.returncode else "")
