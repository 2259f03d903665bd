"""DiceCE backward timing at the workload shape (B = 8 images, N = 21 prompts, 496 x 512 maps): the kernel the
process selects (OCTSAM_DICECE_SCALAR=1: scalar form, else the 4-pixel form) over several grid sizes; prints the
dmask checksum so two processes can be compared bitwise. Diagnostic only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import losses  # noqa: E402

g = torch.Generator().manual_seed(0)
B, N, H, W = 8, 21, 496, 512
masks = (torch.randn(B, N, H, W, generator=g) * 3).cuda()
gt = (torch.rand(B, N, H, W, generator=g) > 0.7).to(torch.uint8).cuda()
part = losses._dice_partials(masks, gt)
out = {"scalar": os.environ.get("OCTSAM_DICECE_SCALAR") == "1"}
for nblk in (512, 1024, 2048, 4096):
    for _ in range(3):
        loss, dm = losses.dicece_forward_backward(masks, gt, part, nblk=nblk)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        loss, dm = losses.dicece_forward_backward(masks, gt, part, nblk=nblk)
    e.record()
    torch.cuda.synchronize()
    out[f"nblk{nblk}_us"] = round(s.elapsed_time(e) * 1e3 / 20, 1)
out["dmask_sum"] = float(dm.double().sum())
out["dmask_abs"] = float(dm.double().abs().sum())
out["loss"] = [float(v) for v in loss.cpu()]
print(json.dumps(out), flush=True)
