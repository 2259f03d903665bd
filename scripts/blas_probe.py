"""torch.matmul (hipBLASLt) vs octsam_gemm on the encoder's GEMM shapes (bf16 in, bf16 out): what a vendor
library reaches on MI355X, as a yardstick for gemm8."""
import sys, os, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for M, N, Kd in [(39200, 2304, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 768, 768), (688128, 256, 256)]:
    A = torch.randn(M, Kd, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(N, Kd, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ms_t = t(lambda: torch.matmul(A, W.t(), out=out))
    ms_o = t(lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out))
    f = 2 * M * N * Kd
    print(json.dumps({"M": M, "N": N, "K": Kd, "hipblaslt_us": round(ms_t * 1e3, 1), "hipblaslt_tf": round(f / ms_t / 1e9),
                      "octsam_us": round(ms_o * 1e3, 1), "octsam_tf": round(f / ms_o / 1e9)}), flush=True)
