"""Data-parallel training step on the GPU: two ranks (one process each, both on cuda:0, gloo over device
tensors standing in for RCCL on this one-GPU box) run FusedTrainStep with the side-stream gradient
all-reduce, the deferred (overlapped) Adam update and hipGraph replay. After two steps their decoder
parameters must equal each other bitwise and match the single-process eager step on the combined 2-image
batch (the reference's single-process semantics, training_utils.py:41-69) up to summation order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch():
    from dilabhelmholtzoct_amd import data
    sd = data.SAMDataset(data.synthetic_oct(seed=5, n=2), {"prompt_type": "bboxes"}, epoch_seed=0)
    items = [sd[0], sd[1]]
    full = data.process_batch(data.make_processor(), data.custom_collate(items), "bboxes")
    n = int(full["gt_u8"].shape[1])
    shards = []
    for it in items:
        b = data.process_batch(data.make_processor(), data.custom_collate([it]), "bboxes")
        shards.append(data.pad_prompts(b, n))  # global-N padding, as the single-process collate pads
    return full, shards


def _worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    _, shards = _global_batch()
    batch = data.to_device_batch(shards[rank], dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, topological=True, process_group=dist.group.WORLD, graphs=True)
    assert step.overlap
    step.step(batch, n_global=2)
    step.flush()  # the all-reduced (global-batch) gradient of step 1 is in flat_grad
    torch.cuda.synchronize()
    torch.save(model.mask_decoder.flat_grad.detach().cpu(), f"{path}.g{rank}")
    step.step(batch, n_global=2)
    step.flush()
    torch.cuda.synchronize()
    torch.save(model.mask_decoder.flat.detach().cpu(), f"{path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_step_matches_single_process(cuda, tmp_path):
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    path = str(tmp_path / "flat")
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0, p.exitcode
    f0 = torch.load(f"{path}.0", weights_only=True)
    f1 = torch.load(f"{path}.1", weights_only=True)
    g0 = torch.load(f"{path}.g0", weights_only=True)
    g1 = torch.load(f"{path}.g1", weights_only=True)
    assert torch.equal(f0, f1) and torch.equal(g0, g1)
    full, _ = _global_batch()
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
    step = FusedTrainStep(model, topological=True)
    batch = data.to_device_batch(full, cuda)
    init = model.mask_decoder.flat.detach().clone()
    step.step(batch)
    gref = model.mask_decoder.flat_grad.detach().cpu().double()
    step.step(batch)
    ref = model.mask_decoder.flat.detach().cpu()
    # gradient of the global batch: same up to summation order (bf16 GEMM operands, fixed-order reductions)
    g = g0.double()
    cos = float(g @ gref / (g.norm() * gref.norm()))
    assert cos > 0.9999, cos
    assert float((g - gref).norm() / gref.norm()) < 1e-2
    # parameters after two Adam steps: Adam normalises each element's step to ~lr = 1e-3, so elements
    # with near-zero gradients may move differently; the bulk must agree
    err = (f0 - ref).abs()
    assert err.max().item() < 2.5e-3, err.max().item()
    assert (err > 1e-4).float().mean().item() < 0.05
    assert (ref - init.cpu()).abs().max().item() > 1e-4


def _worker_pipe(rank, world, port, path, pipeline):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    _, shards = _global_batch()
    batch = data.to_device_batch(shards[rank], dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    step = FusedTrainStep(model, topological=True, process_group=dist.group.WORLD, graphs=True, pipeline=pipeline)
    losses = [step.step(batch, n_global=2, next_batch=batch if k < 3 else None).clone() for k in range(4)]
    step.flush()
    torch.cuda.synchronize()
    torch.save({"flat": model.mask_decoder.flat.detach().cpu(), "losses": torch.stack(losses).cpu()},
               f"{path}.{int(pipeline)}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_with_encoder_lookahead(cuda, tmp_path):
    """The encoder lookahead under data parallelism (deferred Adam, side-stream all-reduce, the next encoder
    queued before the deferred update): losses and parameters bit-identical to the DP step without it."""
    path = str(tmp_path / "pipe")
    ctx = mp.get_context("spawn")
    for pipeline in (False, True):
        port = _port()
        procs = [ctx.Process(target=_worker_pipe, args=(r, 2, port, path, pipeline)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0, p.exitcode
    for rank in range(2):
        a = torch.load(f"{path}.0.{rank}", weights_only=True)
        b = torch.load(f"{path}.1.{rank}", weights_only=True)
        assert torch.equal(a["losses"], b["losses"])
        assert torch.equal(a["flat"], b["flat"])
