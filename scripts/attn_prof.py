"""Launch one ViT attention shape repeatedly (for rocprofv3 kernel traces / PMC passes).
usage: attn_prof.py side nseq heads head_dim [iters]"""
import sys
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dilabhelmholtzoct_amd import kernels as K

side, nseq, heads, hd = (int(v) for v in sys.argv[1:5])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
T = side * side
g = torch.Generator().manual_seed(0)
qkv = torch.randn(nseq, T, 3 * heads * hd, generator=g).to("cuda", torch.bfloat16)
o = torch.empty(nseq, T, heads * hd, device="cuda", dtype=torch.bfloat16)
R = torch.randn(2 * side - 1, hd, device="cuda") * 0.02
for _ in range(iters):
    K.vit_attention(qkv, o, R, R, nseq=nseq, side=side, heads=heads)
torch.cuda.synchronize()
print("done")
