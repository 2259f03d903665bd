"""Launch one octsam_gemm shape repeatedly (rocprofv3 kernel traces / PMC passes).
usage: gemm_prof.py M N K [iters] [act]; env FAST selects octsam_gemm_set_fast_path (A/B)"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K

M, N, Kd = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
act = int(sys.argv[5]) if len(sys.argv) > 5 else 0
A = torch.randn(M, Kd, device="cuda", dtype=torch.bfloat16)
W = torch.randn(N, Kd, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(N, device="cuda")
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
_lib.load().octsam_gemm_set_fast_path(int(os.environ.get("FAST", "1")))
for _ in range(iters):
    K.gemm(A, W, M=M, N=N, K=Kd, out=out, bias=bias, act=act)
torch.cuda.synchronize()
print("done")
