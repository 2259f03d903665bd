"""Determinism probe (diagnostic): repeated ViT attention launches (windowed + global) and encoder forwards
must give identical bits; prints the number of differing elements per repeat."""
import sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '.')
from dilabhelmholtzoct_amd import kernels
from dilabhelmholtzoct_amd.model import SamModel
dev = torch.device('cuda', 0)
torch.manual_seed(0)
for side, nseq in ((64, 8), (14, 200)):
    T = side * side
    qkv = (torch.randn(nseq * T, 3 * 768, device=dev) * 0.5).to(torch.bfloat16)
    rh = torch.randn(2 * side - 1, 64, device=dev) * 0.1
    rw = torch.randn(2 * side - 1, 64, device=dev) * 0.1
    outs = []
    for _ in range(4):
        o = torch.empty(nseq * T, 768, device=dev, dtype=torch.bfloat16)
        kernels.vit_attention(qkv, o, rh, rw, nseq=nseq, side=side, heads=12)
        outs.append(o)
    torch.cuda.synchronize()
    print('attn side', side, [int((outs[0] != x).sum()) for x in outs[1:]])
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
px = torch.randn(2, 3, 1024, 1024, device=dev)
e = [model.vision_encoder.forward_nhwc(px) for _ in range(3)]
torch.cuda.synchronize()
print('encoder', [int((e[0] != x).sum()) for x in e[1:]])
