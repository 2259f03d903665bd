"""Patch-embedding GEMM timing (M = 8*4096, N = K = 768, fp32 out + periodic fp32 positional addend): the
two-workgroup kernel (lean kind 12) vs the 8-phase kernel's general register epilogue (fast path bit 1024). Diagnostic only."""
import sys, os, torch, json
sys.path.insert(0, os.getcwd())
from dilabhelmholtzoct_amd import _lib, kernels
lib=_lib.load()
L,B,N,K=4096,8,768,768; M=L*B
A=torch.randn(M,K,device='cuda').to(torch.bfloat16); W=(torch.randn(N,K,device='cuda')/K**0.5).to(torch.bfloat16)
bias=torch.randn(N,device='cuda'); pos=torch.randn(L,N,device='cuda'); out=torch.empty(M,N,device='cuda')
res={}
for _ in range(3):
  for fast in (1, 1|1024):
    lib.octsam_gemm_set_fast_path(fast)
    f=lambda: kernels.gemm(A,W,M=M,N=N,K=K,out=out,bias=bias,residual=pos,r_remap=(L,B))
    for _ in range(3): f()
    torch.cuda.synchronize(); s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20): f()
    e.record(); torch.cuda.synchronize()
    res[fast]=min(res.get(fast,1e9), s.elapsed_time(e)*1e3/20)
print(json.dumps({"patch_embed_gemm4w_us": round(res[1],1), "patch_embed_gemm8_general_us": round(res[1|1024],1)}))

# the neck's conv3x3 (M = 8*4096, N = C = 256, K = 9C, fp32 out): two-workgroup kernel vs generic register-staged
C = 256
x = torch.randn(8 * 4096, C, device='cuda').to(torch.bfloat16)
Wc = (torch.randn(C, 9 * C, device='cuda') / 48).to(torch.bfloat16)
oc = torch.empty(8 * 4096, C, device='cuda')
res = {}
for _ in range(3):
    for fast in (1, 1 | 1024):
        lib.octsam_gemm_set_fast_path(fast)
        f = lambda: kernels.gemm(x, Wc, M=8 * 4096, N=C, K=9 * C, out=oc, a_mode=3, conv_c=C)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            f()
        e.record()
        torch.cuda.synchronize()
        res[fast] = min(res.get(fast, 1e9), s.elapsed_time(e) * 1e3 / 20)
lib.octsam_gemm_set_fast_path(1)
print(json.dumps({"neck_conv3x3_gemm4w_us": round(res[1], 1), "neck_conv3x3_generic_us": round(res[1 | 1024], 1)}))
