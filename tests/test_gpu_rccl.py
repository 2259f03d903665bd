"""The RCCL path on a one-GPU box: an ``nccl`` (= RCCL on ROCm) process group of world size 1.

* FusedTrainStep(process_group=pg, graphs=True, pipeline=True) runs the side-stream RCCL all-reduce of the flat
  decoder gradient and the deferred (overlapped) Adam update; over 4 steps with alternating batches its losses
  and decoder parameters must equal the single-process step's bit for bit (an all-reduce over one rank and the
  division by 1 are exact).
* bench.py under a launcher's environment (WORLD_SIZE=1) takes its nccl init / global-N MAX / timing
  all-reduce path and prints its JSON line.
The multi-rank semantics are covered by the gloo tests (tests/test_gpu_dp.py, tests/test_dist_cpu.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    from dilabhelmholtzoct_amd import data
    proc = data.make_processor()
    out = []
    for seed in (21, 22):
        sd = data.SAMDataset(data.synthetic_oct(seed=seed, n=2), {"prompt_type": "bboxes"}, epoch_seed=0)
        out.append(data.process_batch(proc, data.custom_collate([sd[0], sd[1]]), "bboxes"))
    return out


def _run(pg, batches, dev):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, topological=True, process_group=pg, graphs=True, pipeline=True)
    bs = [data.to_device_batch(b, dev) for b in batches]
    losses = []
    for i in range(4):
        nxt = bs[(i + 1) % 2] if i + 1 < 4 else None
        losses.append(step.step(bs[i % 2], next_batch=nxt).clone())
    step.flush()
    torch.cuda.synchronize()
    return torch.stack(losses).cpu(), model.mask_decoder.flat.detach().cpu().clone(), step


def _worker(rank, port, path):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    batches = _batches()
    l_pg, p_pg, step = _run(dist.group.WORLD, batches, dev)
    assert step.overlap  # the side-stream all-reduce + deferred Adam path
    l_one, p_one, _ = _run(None, batches, dev)
    torch.save({"l_pg": l_pg, "p_pg": p_pg, "l_one": l_one, "p_one": p_one}, path)
    dist.destroy_process_group()


def test_fused_step_rccl_world1_matches_single_process(cuda, tmp_path):
    path = str(tmp_path / "rccl.pt")
    mp.spawn(_worker, args=(_port(), path), nprocs=1, join=True)
    r = torch.load(path, weights_only=True)
    assert torch.isfinite(r["l_pg"]).all()
    assert torch.equal(r["l_pg"], r["l_one"]), (r["l_pg"], r["l_one"])
    assert torch.equal(r["p_pg"], r["p_one"])


def test_bench_rccl_world1(cuda):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "2",
           "--cpu-baseline", "0", "--val", "0", "--data-path", "0", "--e2e-steps", "0", "--topo-all", "0",
           "--loop-images", "0", "--roof-steps", "0", "--val-protocol", "0", "--top-off", "0"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["config"]["process_group"] == "nccl"
