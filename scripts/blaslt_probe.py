"""torch.matmul (hipBLASLt) on the encoder's GEMM shapes, for reading its kernel choice from a rocprofv3 kernel
trace (the Tensile kernel names encode macro tile, wave tiling and MFMA shape). Diagnostic only."""
import torch

for M, N, K in ((32768, 2304, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 768, 768), (8192, 8192, 8192)):
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        torch.matmul(A, W.t(), out=out)
torch.cuda.synchronize()
print("ok")
