"""Time the HIP data path (components + prompts + gt + processor) per batch of 8 OCT images, and its kernels."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import data
from dilabhelmholtzoct_amd.components import collate_device
from dilabhelmholtzoct_amd.preprocess import DeviceProcessor

dev = torch.device("cuda")
ds = data.synthetic_oct(seed=77, n=8)
imgs = np.stack([d["image"] for d in ds])
labs = np.stack([d["label"] for d in ds])
proc = DeviceProcessor(dev)
for _ in range(3):
    collate_device(imgs, labs, "bboxes", dev, processor=proc)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    collate_device(imgs, labs, "bboxes", dev, processor=proc)
torch.cuda.synchronize()
print(f"HIP data path: {(time.perf_counter() - t0) * 100:.2f} ms per 8 images")
