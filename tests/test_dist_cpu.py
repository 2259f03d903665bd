"""Data-parallel host logic on CPU with torch.distributed gloo, world size 2 (the GPU path uses the same
code over RCCL): loader sharding (global order, first-batch skip on the global batch), global-N prompt
padding, the weighted gradient all-reduce equal to the single-process mean, and the topological-loss
batch nesting following the global batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dilabhelmholtzoct_amd import data, train
from dilabhelmholtzoct_amd.losses import topo_entries


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.group.WORLD
    out = {}
    # weighted gradient average: rank r holds n_r images with mean gradient g_r
    n_local = [3, 1][rank]
    g = torch.full((5,), float(rank + 1)) * torch.arange(5.0)
    train.allreduce_weighted(g, pg, n_local, 4)
    out["g"] = g.tolist()
    # equal shards: plain mean
    h = torch.full((3,), float(rank))
    train.allreduce_weighted(h, pg, 2, 4)
    out["h"] = h.tolist()
    out["max"] = train._collective_max([7, 19][rank], pg)
    out["sum"] = train._collective_sum(torch.tensor([rank + 1, 10], dtype=torch.int64), pg).tolist()
    # global-N padding: each rank pads its own collate to the global max
    labs = np.load(os.path.join(os.path.dirname(__file__), "golden", "data_golden.npz"))["labels"]
    items = [{"image": np.repeat((lab * 18)[:, :, None], 3, 2).astype(np.uint8), "label": lab} for lab in labs[:2]]
    ds = data.SAMDataset(items, {"prompt_type": "bboxes"}, epoch_seed=5)
    mine = [ds[rank]]
    N = train._collective_max(train._n_prompts(mine), pg)
    b = data.pad_prompts(data.process_batch(data.make_processor(), data.custom_collate(mine)), N)
    out["gt"] = b["gt_u8"][0].double().numpy().copy()
    out["boxes"] = b["input_boxes"][0].numpy().copy()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want_g = ((3 * 1 + 1 * 2) / 4 * torch.arange(5.0)).tolist()
    for r in (0, 1):
        assert np.allclose(res[r]["g"], want_g)
        assert np.allclose(res[r]["h"], [0.5, 0.5, 0.5])
        assert res[r]["max"] == 19
        assert res[r]["sum"] == [3, 20]
    # single-process collate of both images == per-rank padded batches
    labs = np.load(os.path.join(os.path.dirname(__file__), "golden", "data_golden.npz"))["labels"]
    items = [{"image": np.repeat((lab * 18)[:, :, None], 3, 2).astype(np.uint8), "label": lab} for lab in labs[:2]]
    ds = data.SAMDataset(items, {"prompt_type": "bboxes"}, epoch_seed=5)
    both = data.process_batch(data.make_processor(), data.custom_collate([ds[0], ds[1]]))
    for r in (0, 1):
        assert np.array_equal(res[r]["gt"], both["gt_u8"][r].double().numpy())
        assert np.allclose(res[r]["boxes"], both["input_boxes"][r].numpy())


@pytest.mark.parametrize("n,bs,world", [(10, 2, 2), (9, 2, 2), (7, 3, 1), (5, 2, 4), (16, 8, 2)])
def test_global_batches_partition(n, bs, world):
    ref = [list(range(s, min(n, s + bs * world))) for s in range(0, n, bs * world)]
    per_rank = [train.global_batches(n, bs, world, r) for r in range(world)]
    assert all(len(p) == len(ref) for p in per_rank)
    for k, gb in enumerate(ref):
        got = [i for r in range(world) for i in per_rank[r][k]]
        assert got == gb
        sizes = [len(per_rank[r][k]) for r in range(world)]
        assert max(sizes) - min(sizes) <= 1
    sh = [train.global_batches(n, bs, world, r, shuffle=True, seed=1, epoch=2) for r in range(world)]
    flat = sorted(i for r in range(world) for b in sh[r] for i in b)
    assert flat == list(range(n))


def test_topo_nesting_follows_global_batch():
    # one image per rank but a global batch of 2: per-image rule, not per-prompt
    assert topo_entries(1, 5, "first", global_batch=2) == [[0]]
    assert topo_entries(1, 5, "all", global_batch=2) == [[0, 1, 2, 3, 4]]
    assert topo_entries(1, 5, "first") == [[n] for n in range(5)]


def test_bench_spawns_one_process_per_rank(capfd):
    """`python bench.py --gpus N` without a launcher starts N rank processes with the torchrun environment
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1) and relays rank 0's line (verdict r1 #7)."""
    import argparse
    import sys
    import bench
    code = ("import os; r = os.environ; print(r['RANK'], r['LOCAL_RANK'], r['WORLD_SIZE'], r['MASTER_ADDR'], "
            "bool(r['MASTER_PORT'])); raise SystemExit(0)")
    rc = bench.spawn_ranks(argparse.Namespace(gpus=3), cmd=[sys.executable, "-c", code])
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert out == ["0 0 3 127.0.0.1 True"]
