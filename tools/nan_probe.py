import sys, numpy as np, torch
import pathlib; R=pathlib.Path(__file__).resolve().parents[1]; sys.path[:0]=[str(R), str(R/'rdma-ring-collectives_amd')]
import pgamd
lib=pgamd.load()
a=np.array([np.inf, 0.0, np.nan, -np.nan, np.inf, 1e308], np.float64)
b=np.array([-np.inf, 0.0, 1.0, 1.0, 0.0, 1e308], np.float64)
for op in (0,1):
    A=torch.from_numpy(a.copy()).cuda(); B=torch.from_numpy(b).cuda()
    lib.pgk_reduce(A.data_ptr(), B.data_ptr(), a.size, 1, op, torch.cuda.current_stream().cuda_stream)
    g=A.cpu().numpy()
    c=(a+b) if op==0 else (a*b)
    print("op",op,"gpu",[hex(x) for x in g.view(np.uint64)],"cpu",[hex(x) for x in c.view(np.uint64)])
