"""The decoder's largest image-side weight gradient (final-attention K|V dW: dY [P*4096, 384]^T X [P*4096, 256],
split-K 64 ways, k-major operands -> gemm_glds_kernel) launched N times, for rocprofv3 passes. Diagnostic only.
usage: dw_prof.py [launches]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rows, O, I, split = 688128, 384, 256, 64
ks = rows // split
g = torch.Generator().manual_seed(0)
dy = torch.randn(rows, O, generator=g).to("cuda", torch.bfloat16)
x = torch.randn(rows, I, generator=g).to("cuda", torch.bfloat16)
part = torch.empty(split, O, I, device="cuda")
for _ in range(n):
    K.gemm(dy, x, M=O, N=I, K=ks, out=part, a_mode=1, b_mode=1, lda=O, ldb=I, batch=split, stride_a=ks * O,
           stride_b=ks * I, stride_c=O * I)
torch.cuda.synchronize()
print("ok")
