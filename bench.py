#!/usr/bin/env python3
"""Benchmark: train images/sec of the OCT-SAM training step (BASELINE.json metric) on MI355X.

Workload (BASELINE.json configs[2], the configuration the metric is quoted on: "top-loss on"):
sam-vit-base, --prompt=bboxes, --top=True, bf16 compute, batch 8 per GPU, 1024x1024 processed OCT
images (synthetic OCT-like label maps, N = max components in the batch prompts per image), one step =
encoder fwd + prompt encoder + mask decoder fwd/bwd + post-processing + DiceCE + topological loss +
Adam (ref:octsam/models/training_utils.py:46-69). Inputs are resident in HBM before timing starts.

Multi-GPU: one process per GPU (torchrun), weak scaling (8 images per rank), RCCL all-reduce of the
flat mask-decoder gradient before Adam; max over ranks of the timed region.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "train imgs/sec (1024² OCT, vit-base, top-loss on) + val Dice; 1→8 GPUs"
MI355X_BF16_DENSE_TFLOPS = 2500.0  # /opt/skills/guides/MI355X_MICROARCH.md (dense, no sparsity)
# HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes (FETCH_SIZE x2 for
# gfx950's half-counted wide reads + WRITE_SIZE; scripts/gpu_round.sh -> scripts/pmc_traffic.py), same bench
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "traffic_gemm8.json")


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=8, help="images per GPU")
    p.add_argument("--model", default="facebook/sam-vit-base")
    p.add_argument("--prompt", default="bboxes", choices=["bboxes", "points", "both"])
    p.add_argument("--top", type=int, default=1)
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle step (rank 0, N=1)")
    p.add_argument("--cpu-steps", type=int, default=2)
    p.add_argument("--val", type=int, default=8, help="val images for the Dice readout (0 = skip)")
    p.add_argument("--data-path", type=int, default=1,
                   help="time building one batch on the host (reference data path) vs the HIP data path")
    p.add_argument("--no-events", action="store_true", help="do not record per-kernel HIP events")
    p.add_argument("--eager", action="store_true", help="launch every kernel from Python (no hipGraph replay)")
    p.add_argument("--roof-steps", type=int, default=2, help="eager steps timed per GEMM launch for the roofline")
    return p.parse_args()


DOMINANT = "gemm8_kernel<0, EPI> (8-phase 256x256 bf16 NT GEMM: encoder QKV/proj/MLP, neck, decoder projections)"


class GemmEventTimer:
    """Wraps kernels.gemm: HIP events on the launch stream (torch's current stream, which every wrapper
    passes to the library) around every GEMM launch in the timed region; octsam_gemm_last_path() tells
    which kernel ran, and only the dominant one (path 2 = gemm8_kernel) is kept. Accumulates algorithmic
    FLOPs 2*M*N*K*batch of those launches."""

    def __init__(self):
        from dilabhelmholtzoct_amd import kernels
        self.k = kernels
        self.orig = kernels.gemm
        self.active = False
        self.events = []
        self.flops = 0.0
        self.bytes = 0.0

    def __enter__(self):
        orig = self.orig

        from dilabhelmholtzoct_amd import _lib
        lib = _lib.load()

        def wrapped(A, B, **kw):
            if self.active:
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                out = orig(A, B, **kw)
                e.record()
                if lib.octsam_gemm_last_path() == 2:
                    self.events.append((s, e))
                    self.flops += 2.0 * kw["M"] * kw["N"] * kw["K"] * kw.get("batch", 1)
                    # compulsory bytes: A, B read once, C written once (+ residual read), per launch
                    bt = kw.get("batch", 1)
                    osz = kw["out"].element_size()
                    r = kw.get("residual")
                    self.bytes += bt * (2.0 * (kw["M"] + kw["N"]) * kw["K"] + kw["M"] * kw["N"] * osz +
                                        (kw["M"] * kw["N"] * r.element_size() if r is not None else 0))
                return out
            return orig(A, B, **kw)

        self.k.gemm = wrapped
        # modules imported the function object by name; patch their references too
        import dilabhelmholtzoct_amd.model as m
        import dilabhelmholtzoct_amd.decoder as d
        m.K.gemm = wrapped
        d.K.gemm = wrapped
        return self

    def __exit__(self, *a):
        self.k.gemm = self.orig

    def result(self):
        torch.cuda.synchronize()
        ms = sum(s.elapsed_time(e) for s, e in self.events)
        n = len(self.events)
        return ms, n, self.flops


def make_batch(args, rank, device, processor):
    from dilabhelmholtzoct_amd import data
    ds = data.synthetic_oct(seed=1000 + rank, n=args.batch)
    sd = data.SAMDataset(ds, {"prompt_type": args.prompt}, epoch_seed=rank)
    batch = data.custom_collate([sd[i] for i in range(len(sd))])
    return data.process_batch(processor, batch, args.prompt)


def workload_name(args) -> str:
    short = args.model.rsplit("/", 1)[-1]
    desc = f"{short}, --prompt={args.prompt}, --top={bool(args.top)}, bf16, batch {args.batch}/GPU"
    if short == "sam-vit-base" and args.prompt == "bboxes":
        return f"BASELINE configs[{2 if args.top else 1}]: {desc}"
    if args.prompt == "both":
        return f"BASELINE configs[4] prompt mode (box + point per component) on {desc}"
    if short == "sam-vit-large" and args.prompt == "points" and args.top:
        return f"BASELINE configs[3] (per-GPU slice of batch 32 over 8 GPUs): {desc}"
    return desc


def time_data_path(args, device, processor, reps=3):
    """Outside the timed step: one batch (B images, prompts, gt, pixel_values) built by the reference's host
    data path (SAMDataset with scipy components + custom_collate + SamProcessor, then the H2D copy) vs the
    HIP data path (uint8 images / label maps uploaded, components + prompts + gt + processor on the GPU)."""
    import random
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.components import collate_device
    from dilabhelmholtzoct_amd.preprocess import DeviceProcessor
    ds = data.synthetic_oct(seed=77, n=args.batch)
    imgs = np.stack([np.array(ds[i]["image"]) for i in range(args.batch)])
    labs = np.stack([np.array(ds[i]["label"]) for i in range(args.batch)])
    dproc = DeviceProcessor(device)

    def host():
        sd = data.SAMDataset(ds, {"prompt_type": args.prompt}, epoch_seed=0)
        b = data.process_batch(processor, data.custom_collate([sd[i] for i in range(args.batch)]), args.prompt)
        return data.to_device_batch(b, device)

    def dev():
        hooks = [(lambda i=i: data.seed_sample(0, i, 0)) for i in range(args.batch)]
        return collate_device(imgs, labs, args.prompt, device, seed_hooks=hooks, processor=dproc)

    out = {}
    for name, fn in (("host_ms", host), ("hip_ms", dev)):
        np.random.seed(0)
        random.seed(0)
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            b = fn()
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t0) * 1e3 / reps, 2)
        out["gt_" + name[:-3]] = b["gt_u8"]
    same = bool(torch.equal(out.pop("gt_host").cpu(), out.pop("gt_hip").cpu()))
    out.update({"images": args.batch, "gt_identical": same,
                "note": "per batch, outside the timed step; host = SAMDataset+collate+SamProcessor+H2D"})
    log(f"data path: host {out['host_ms']} ms, HIP {out['hip_ms']} ms per {args.batch} images")
    return out


def cpu_baseline(args, batch_cpu):
    """CPU oracle step (oracle/step_ref.py: transformers SamModel fp32 + restated DiceCE/topo + Adam) on a
    bounded sample (1 image, all its prompts), timed on this host's cores."""
    from oracle.step_ref import CpuReferenceStep
    # the GPU box shows the whole machine's CPUs; this job's share is OMP_NUM_THREADS (16 there)
    ncores = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    ncores = min(ncores, share) if share > 0 else min(ncores, 16)
    torch.set_num_threads(ncores)
    step = CpuReferenceStep(args.model, topological=bool(args.top), seed=0)
    one = {k: (v[:1] if isinstance(v, torch.Tensor) and v.dim() > 0 else v) for k, v in batch_cpu.items()}
    step.step(one)  # warm-up
    log(f"cpu baseline: warm-up done on {ncores} threads")
    t0 = time.time()
    for _ in range(args.cpu_steps):
        step.step(one)
        log(f"cpu baseline: step {time.time() - t0:.1f} s")
    dt = time.time() - t0
    n_prompts = int(one["gt_u8"].shape[1])
    return {"value": round(args.cpu_steps / dt, 5), "unit": "imgs/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{args.cpu_steps} timed steps (+1 warm-up) of batch 1 ({n_prompts} {args.prompt}), fp32, "
                      f"oracle/step_ref.py on {ncores} host threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)
        pg = dist.group.WORLD
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep, class_confusion, mean_dice, predict_masks

    processor = data.make_processor()
    batch_cpu = make_batch(args, rank, device, processor)
    if world > 1:  # global-N padding: every rank pads prompts to the global max (single-process collate)
        import torch.distributed as dist
        n = torch.tensor([batch_cpu["gt_u8"].shape[1]], device=device)
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        batch_cpu = data.pad_prompts(batch_cpu, int(n.item()))
    batch = data.to_device_batch(batch_cpu, device)
    N = int(batch["gt_u8"].shape[1])

    model = SamModel.from_pretrained(args.model, seed=0).to(device)
    step = FusedTrainStep(model, lr=1e-3, topological=bool(args.top), process_group=pg, graphs=not args.eager)

    def barrier():
        if pg is not None:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    log(f"rank {rank}: N={N} prompts/image, warm-up")
    for _ in range(args.warmup):
        step.step(batch)
    step.flush()
    barrier()
    log(f"rank {rank}: timing {args.steps} steps")
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = step.step(batch)
    step.flush()  # a deferred (overlapped) update belongs to the timed work
    barrier()
    dt = time.perf_counter() - t0
    # Roofline of the dominant kernel: HIP events around each of its launches. Graph replays run no
    # Python, so the launches are timed in `roof_steps` eager steps of the same batch right after the
    # timed region (same kernels, shapes and stream); rocprofv3 over the graph run must agree.
    timer = GemmEventTimer() if not args.no_events and args.roof_steps > 0 else None
    if timer:
        graphs = step.graphs
        step.graphs = False
        timer.__enter__()
        timer.active = True
        for _ in range(args.roof_steps):
            step.step(batch)
        step.flush()
        timer.active = False
        timer.__exit__()
        step.graphs = graphs
    if pg is not None:
        import torch.distributed as dist
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    imgs = args.batch * world * args.steps
    value = imgs / dt
    loss_h = loss.cpu().tolist()

    roof = None
    if timer:
        ms, n, flops = timer.result()
        if n:
            achieved = flops / (ms * 1e-3) / 1e12
            traffic = None
            if os.path.exists(TRAFFIC_JSON):
                traffic = round(json.load(open(TRAFFIC_JSON))["hbm_bytes_per_launch"])
            roof = {"bound": "mfma", "kernel": DOMINANT,
                    "achieved": round(achieved, 2), "peak": MI355X_BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / MI355X_BF16_DENSE_TFLOPS, 4), "traffic": traffic,
                    "traffic_source": os.path.relpath(TRAFFIC_JSON, ROOT) if traffic is not None else None,
                    "compulsory_bytes_per_launch": round(timer.bytes / n),
                    "launches": n, "avg_launch_us": round(ms * 1e3 / n, 2),
                    "share_of_step": round(ms / args.roof_steps / (dt * 1e3 / args.steps), 4)}

    log(f"rank {rank}: {dt * 1e3 / args.steps:.2f} ms/step")
    val_dice = None
    if args.val and rank == 0:
        vb = data.to_device_batch(make_batch(argparse.Namespace(batch=args.val, prompt=args.prompt), 999, device,
                                             processor), device)
        masks = predict_masks(model, vb)
        val_dice = round(mean_dice(class_confusion(masks, vb["gt_u8"], vb["mask_values"])), 5)

    data_path = None
    if args.data_path and rank == 0:
        data_path = time_data_path(args, device, processor)

    cpu = None
    if args.cpu_baseline and rank == 0 and world == 1:
        try:
            cpu = cpu_baseline(args, batch_cpu)
        except Exception as e:  # the baseline must never hide the GPU result
            cpu = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 4), "unit": "imgs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic OCT-like 496x512 label maps -> 1024x1024 processed images, {N} "
                    f"{'point' if args.prompt == 'points' else 'box'} prompts/image (batch max), random-init "
                    f"weights (seed 0)",
            "config": {"workload": workload_name(args), "model": args.model, "global_batch": args.batch * world,
                       "prompts_per_image": N, "prompt": args.prompt, "top": bool(args.top),
                       "parallelism": f"dp{world}", "exec": "eager" if args.eager else "hipgraph"},
            "loss_last_step": {"dice": loss_h[0], "ce": loss_h[1], "topo": loss_h[2], "total": loss_h[3]},
            "val_dice": val_dice,
            "data_path": data_path,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
