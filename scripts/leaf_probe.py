"""Decoder forward/backward with the weight-gradient leaf stream, twice, synchronising after each phase
(diagnostic for the leaf-stream schedule)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd.model import SamModel  # noqa: E402

dev = torch.device("cuda", 0)
extra = [torch.cuda.Stream(device=dev) for _ in range(int(os.environ.get("EXTRA_STREAMS", "0")))]
model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
dec = model.mask_decoder
B, N = 2, 3
emb = torch.randn(B, 256, 64, 64, device=dev)
for leaf in (True, False):
    dec.leaf_overlap = leaf
    for it in range(3):
        t0 = time.time()
        out = model(image_embeddings=emb, input_boxes=torch.rand(B, N, 4, device=dev) * 1024, multimask_output=False)
        torch.cuda.synchronize()
        print("leaf", leaf, "it", it, "fwd ok", round(time.time() - t0, 3), flush=True)
        out.pred_masks.float().sum().backward()
        torch.cuda.synchronize()
        print("leaf", leaf, "it", it, "bwd ok", round(time.time() - t0, 3), flush=True)
