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
MI355X_HBM_GBS = 8000.0  # HBM3E peak, same guide
# SURVEY.md §8(d) algorithmic decoder traffic per prompt: every inter-kernel image-side tensor written and
# read once, E = 4096 tokens x 256 ch x 2 B: 12 E forward, 24 E backward
_E = 4096 * 256 * 2
DEC_FWD_BYTES_PER_PROMPT = 12 * _E
DEC_BWD_BYTES_PER_PROMPT = 24 * _E
# HBM bytes per launch of the dominant kernel family from the committed rocprofv3 PMC passes (FETCH_SIZE x2 for
# gfx950's half-counted wide reads + WRITE_SIZE; scripts/gpu_traffic.sh -> scripts/pmc_traffic.py), same bench.
# The family files (round 4) average the same launch set as roofline.compulsory_bytes_per_launch (octsam_gemm path 2:
# gemm8_kernel, gemm8p_kernel, gemm4w_kernel); the older gemm8-only files are used only where no family file exists.
FAMILY_KERNELS = "gemm8_kernel,gemm8p_kernel,gemm4w_kernel"


def traffic_json(args) -> str:
    """PMC traffic file of the dominant GEMM family for this workload: vit-base bf16 -> traffic_gemm_family.json,
    otherwise traffic_gemm_family_<model>_<dtype>.json; falls back to the gemm8-only traffic_gemm8*.json."""
    short = args.model.rsplit("/", 1)[-1]
    tag = "" if (short == "sam-vit-base" and args.dtype == "bf16") else f"_{short}_{args.dtype}"
    fam = os.path.join(ROOT, "profiles", f"traffic_gemm_family{tag}.json")
    return fam if os.path.exists(fam) else os.path.join(ROOT, "profiles", f"traffic_gemm8{tag}.json")


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
    p.add_argument("--gemm-fast-path", type=int, default=1,
                   help="octsam_gemm_set_fast_path value for the run (1: default; A/B only)")
    p.add_argument("--fork-topo", type=int, default=1,
                   help="persistence + transport beside the DiceCE backward (FusedTrainStep.fork_topo; 0: A/B)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"],
                   help="16-bit operand type of the frozen encoder (fp16: BASELINE configs[4]); the decoder is bf16")
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle step (rank 0, N=1)")
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--cpu-batch8", type=int, default=1, help="also time one CPU oracle step of the full batch")
    p.add_argument("--val", type=int, default=8, help="val images for the Dice readout (0 = skip)")
    p.add_argument("--data-path", type=int, default=1,
                   help="time building one batch on the host (reference data path) vs the HIP data path")
    p.add_argument("--no-events", action="store_true", help="do not record per-kernel HIP events")
    p.add_argument("--eager", action="store_true", help="launch every kernel from Python (no hipGraph replay)")
    p.add_argument("--pipeline", type=int, default=1,
                   help="encoder lookahead (graph mode): the next step's frozen-encoder phase replays on a side "
                        "stream during this step's decoder; every timed step still runs its own encoder")
    p.add_argument("--roof-steps", type=int, default=2, help="eager steps timed per GEMM launch for the roofline")
    p.add_argument("--e2e-steps", type=int, default=10,
                   help="steps of the end-to-end loop (a new batch per step through the HIP data path)")
    p.add_argument("--topo-all", type=int, default=1, help="time the topo_mode='all' reading of batch_iter too")
    p.add_argument("--val-protocol", type=int, default=1,
                   help="the val-Dice protocol of tests/test_gpu_val_dice.py beside the committed oracle values")
    p.add_argument("--top-off", type=int, default=1,
                   help="with --top 1: also time the --top=False step on the same batch (BASELINE configs[1])")
    p.add_argument("--loop-images", type=int, default=128,
                   help="time train.training() over an epoch of this many synthetic images (0 = skip)")
    return p.parse_args()


def dominant_name(args) -> str:
    e = "bf16" if args.dtype == "bf16" else "fp16 (encoder) / bf16 (decoder)"
    return (f"gemm8w_kernel / gemm8_kernel family (256x256 {e} NT GEMMs: the ping-pong 8-wave kernel, the 8-phase "
            "kernel and its persistent form, and the two-workgroup 256x128 gemm4w_kernel: the encoder's QKV, "
            "attention projection, MLP1 and MLP2, the neck, the decoder's image-side projections)")


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
                path = lib.octsam_gemm_last_path()
                if path == 2:
                    fl = 2.0 * kw["M"] * kw["N"] * kw["K"] * kw.get("batch", 1)
                    # compulsory bytes: A, B read once, C written once (+ residual read), per launch
                    bt = kw.get("batch", 1)
                    osz = kw["out"].element_size()
                    r = kw.get("residual")
                    by = bt * (2.0 * (kw["M"] + kw["N"]) * kw["K"] + kw["M"] * kw["N"] * osz +
                               (kw["M"] * kw["N"] * r.element_size() if r is not None else 0))
                    self.events.append((s, e, fl, by))
                    self.flops += fl
                    self.bytes += by
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
        ms = sum(s.elapsed_time(e) for s, e, _, _ in self.events)
        n = len(self.events)
        return ms, n, self.flops

    def by_bound(self):
        """The family's launches split by their compulsory arithmetic intensity against the MI355X ridge
        (dense bf16 peak / HBM peak): compute-bound launches (encoder, neck) in TFLOP/s, memory-bound ones
        (the decoder's K = 128-384 image-side projections) in GB/s of compulsory bytes."""
        ridge = MI355X_BF16_DENSE_TFLOPS * 1e12 / (MI355X_HBM_GBS * 1e9)
        out = {}
        for name, sel in (("mfma_bound", lambda f, b: f / b >= ridge), ("hbm_bound", lambda f, b: f / b < ridge)):
            ev = [(s.elapsed_time(e), f, b) for s, e, f, b in self.events if sel(f, b)]
            if not ev:
                continue
            ms = sum(x[0] for x in ev)
            fl = sum(x[1] for x in ev)
            by = sum(x[2] for x in ev)
            if name == "mfma_bound":
                a = fl / (ms * 1e-3) / 1e12
                out[name] = {"bound": "mfma", "achieved": round(a, 2), "peak": MI355X_BF16_DENSE_TFLOPS,
                             "unit": "TFLOP/s", "frac": round(a / MI355X_BF16_DENSE_TFLOPS, 4), "launches": len(ev),
                             "avg_launch_us": round(ms * 1e3 / len(ev), 2)}
            else:
                a = by / (ms * 1e-3) / 1e9
                out[name] = {"bound": "hbm", "achieved": round(a, 1), "peak": MI355X_HBM_GBS, "unit": "GB/s",
                             "frac": round(a / MI355X_HBM_GBS, 4), "launches": len(ev),
                             "avg_launch_us": round(ms * 1e3 / len(ev), 2),
                             "work": "compulsory bytes: A, B, C once (+ residual)"}
        return out


class CallTimer:
    """HIP events (torch's current stream = the launch stream of every wrapper) around each call of
    ``owner.name`` while active; ``work(*a, **kw)`` gives the call's algorithmic FLOPs or bytes."""

    def __init__(self, owner, name, work):
        self.owner, self.name, self.work = owner, name, work
        self.orig = getattr(owner, name)
        self.events, self.total = [], 0.0
        self.active = False

    def __enter__(self):
        orig = self.orig

        def wrapped(*a, **kw):
            if not self.active:
                return orig(*a, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = orig(*a, **kw)
            e.record()
            self.events.append((s, e))
            self.total += self.work(*a, **kw)
            return out

        setattr(self.owner, self.name, wrapped)
        return self

    def __exit__(self, *a):
        setattr(self.owner, self.name, self.orig)

    def result(self):
        torch.cuda.synchronize()
        return sum(s.elapsed_time(e) for s, e in self.events), len(self.events), self.total


def attn_flops(qkv, out, rh, rw, *, nseq, side, heads, grid=0, pad_row=None):
    """QK^T and PV of one octsam_vit_attention launch: 4 * T^2 * head_dim * heads * nseq, T = side^2 (the
    windowed layers' padded 14x14 windows included, as the reference computes them); head_dim from the
    rel-pos tables (64 vit-b/l, 80 vit-h)."""
    T = side * side
    return 4.0 * T * T * rh.shape[-1] * heads * nseq


def make_batch(args, rank, device, processor):
    from dilabhelmholtzoct_amd import data
    ds = data.synthetic_oct(seed=1000 + rank, n=args.batch)
    sd = data.SAMDataset(ds, {"prompt_type": args.prompt}, epoch_seed=rank)
    batch = data.custom_collate([sd[i] for i in range(len(sd))])
    return data.process_batch(processor, batch, args.prompt)


def workload_name(args) -> str:
    short = args.model.rsplit("/", 1)[-1]
    desc = f"{short}, --prompt={args.prompt}, --top={bool(args.top)}, {args.dtype}, batch {args.batch}/GPU"
    if short == "sam-vit-base" and args.prompt == "bboxes":
        return f"BASELINE configs[{2 if args.top else 1}]: {desc}"
    if short == "sam-vit-huge" and args.prompt == "both" and args.top and args.dtype == "fp16":
        return f"BASELINE configs[4] (per-GPU slice of batch 64 over 8 GPUs): {desc}"
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


def end_to_end(args, step, device, rank, world, pg, n_raw=4):
    """value_end_to_end: the step fed a NEW batch every iteration, as the reference's loop is
    (training_utils.py:41-55): uint8 images + label maps (n_raw distinct synthetic sets, re-drawn prompts
    every epoch) -> HIP data path (components, prompts, gt, processor; components.collate_device) on a side
    stream, overlapped with the previous step (built while the GPU runs that step's forward), then copied into
    the captured graphs' inputs. Disk decoding of the dataset is not included (no dataset on disk)."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.components import collate_device
    from dilabhelmholtzoct_amd.preprocess import DeviceProcessor
    raw = []
    for k in range(n_raw):
        ds = data.synthetic_oct(seed=5000 + 100 * rank + k, n=args.batch)
        raw.append((np.stack([d["image"] for d in ds]), np.stack([d["label"] for d in ds])))
    dproc = DeviceProcessor(device)
    side = torch.cuda.Stream(device=device)
    main_stream = torch.cuda.current_stream(device)

    def prep(i):
        imgs, labs = raw[i % n_raw]
        hooks = [(lambda j=j, e=i: data.seed_sample(e, j, rank)) for j in range(args.batch)]
        with torch.cuda.stream(side):
            b = collate_device(imgs, labs, args.prompt, device, seed_hooks=hooks, processor=dproc)
            b.pop("prompt_raw")
            if pg is not None:  # global-N padding (a tiny MAX all-reduce on the main process group)
                b = _pad_global(b, pg, device)
            ev = torch.cuda.Event()
            ev.record(side)
        for v in b.values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(main_stream)
        return b, ev

    def run(n):
        # batches are built two ahead (during step i: batch i + 2) so that step i can name batch i + 1 for the
        # encoder lookahead; the last step names none (exactly n encoder passes)
        ready = [prep(0), prep(1)]
        for i in range(n):
            cur, ev = ready[0]
            main_stream.wait_event(ev)
            nb = None
            if i + 1 < n:
                main_stream.wait_event(ready[1][1])
                nb = ready[1][0]
            holder = []
            step.step(cur, between=lambda i=i: holder.append(prep(i + 2)), next_batch=nb)
            ready = [ready[1], holder[0]]
        step.flush()

    log(f"rank {rank}: end-to-end warm-up (one capture per batch shape)")
    run(2 * n_raw)
    if pg is not None:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.e2e_steps)
    torch.cuda.synchronize()
    if pg is not None:
        import torch.distributed as dist
        dist.barrier()
    dt = time.perf_counter() - t0
    if pg is not None:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    value = args.batch * world * args.e2e_steps / dt
    log(f"rank {rank}: end-to-end {dt * 1e3 / args.e2e_steps:.2f} ms/step ({value:.1f} imgs/s)")
    return {"value": round(value, 4), "unit": "imgs/s", "ms_per_step": round(dt * 1e3 / args.e2e_steps, 3),
            "steps": args.e2e_steps, "distinct_raw_batches": n_raw,
            "note": "new batch per step: uint8 images + label maps -> HIP components/prompts/gt/processor on a "
                    "side stream overlapped with the previous step; no disk decode"}


def _pad_global(b, pg, device):
    import torch.distributed as dist
    from dilabhelmholtzoct_amd import data
    n = torch.tensor([b["gt_u8"].shape[1]], device=device)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=pg)
    return data.pad_prompts(b, int(n.item())) if int(n.item()) > b["gt_u8"].shape[1] else b


def topo_all_sensitivity(args, model, batch, steps=5):
    """ms/step with the topo_mode='all' reading of torch_topological's batch_iter (every prompt's diagrams,
    2*B*N persistence maps per step instead of 2*B; SURVEY.md §8(a) A17 — the reading is unpinned), with the
    transport on the device (the step's default, octsam_topo_w2) and on the host between the graphs (w2_host:
    octsam_topo_host after a device sync, the round-2 path) for comparison."""
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    pipe = bool(args.pipeline) and not args.eager
    B, N = batch["gt_u8"].shape[:2]
    out = {"persistence_maps_per_step": 2 * B * N, "entries": B, "steps": steps}
    for w2 in ("device", "host"):
        st = FusedTrainStep(model, lr=1e-3, topological=True, topo_mode="all", graphs=not args.eager, pipeline=pipe,
                            w2=w2)
        for i in range(2):
            st.step(batch, next_batch=batch if i == 0 else None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            st.step(batch, next_batch=batch if i + 1 < steps else None)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        key = "" if w2 == "device" else "w2_host_"
        out[key + "ms_per_step"] = round(dt * 1e3 / steps, 3)
        out[key + "imgs_per_s"] = round(B * steps / dt, 2)
        del st
    log(f"topo_mode=all: {out}")
    return out


def top_off_leg(args, model, batch, steps=10):
    """BASELINE configs[1] beside the headline configs[2]: the same model, batch and execution (hipGraphs + encoder
    lookahead) with --top=False (the DiceCE-only step, ref:octsam/models/training_utils.py:62-68), timed like the
    headline (inputs resident, `steps` back-to-back steps, the last one naming no next batch)."""
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    pipe = bool(args.pipeline) and not args.eager
    B = batch["gt_u8"].shape[0]
    st = FusedTrainStep(model, lr=1e-3, topological=False, graphs=not args.eager, pipeline=pipe)
    for i in range(3):
        st.step(batch, next_batch=batch if i < 2 else None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        st.step(batch, next_batch=batch if i + 1 < steps else None)
    st.flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del st
    out = {"workload": "configs[1]: sam-vit-base, --prompt=bboxes, --top=False, bf16, B=8 per GPU",
           "value": round(B * steps / dt, 4), "unit": "imgs/s", "ms_per_step": round(dt * 1e3 / steps, 3),
           "steps": steps}
    log(f"top off (configs[1]): {out}")
    return out


def val_protocol(args, device):
    """The val-Dice half of the metric on the multi-seed protocol of tests/valdice_protocol.py (SURVEY.md §8(d);
    ref:octsam/models/training_utils.py:113-156, 246), HIP side of tests/test_gpu_val_dice.py: the synthetic vit-b
    weights (seed 0) with the ORACLE-made warm start (tests/golden/valdice_warm_oracle.safetensors: decoder + Adam
    state), then per (training, held-out) seed pair 4 epochs (64 steps) on 128 scans, the 32 held-out scans scored
    after every epoch, beside the fp32 oracle's values from the same start (tests/golden/valdice_oracle.json, made by
    tests/golden/make_valdice_golden.py on MI355X with the oracle alone, so they hold for any HIP build). Batches come
    from the HIP data path as in the test (valdice_protocol.device_batches: bit-identical to the host SAMDataset +
    collate + SamProcessor path, test_gpu_training_loop.py); the step is the benchmarked one (hipGraphs + encoder
    lookahead)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import valdice_protocol as P
    gold = json.load(open(P.ORACLE_JSON))
    gold_pairs = {(g["train_seed"], g["val_seed"]): g for g in gold["pairs"]}
    t0 = time.perf_counter()
    epoch_batches = P.device_batches(device)
    state, adam = P.load_warm()
    runner = P.HipRunner(device, state, epoch_batches)
    pairs = []
    for idx, (tr, va) in enumerate(P.SEEDS):
        if idx + 1 < len(P.SEEDS):  # the next pair's scans, synthesised on a host thread meanwhile
            epoch_batches.prefetch(P.SEEDS[idx + 1][0], P.N_TRAIN)
            epoch_batches.prefetch(P.SEEDS[idx + 1][1], P.N_VAL)
        hip = [round(P.dice_of(c), 5) for _, c in runner.run(state, adam, tr, va,
                                                              val_batches=epoch_batches(va, P.N_VAL, 0))]
        epoch_batches.forget(tr, P.N_TRAIN)
        epoch_batches.forget(va, P.N_VAL)
        if (idx + 1) % 16 == 0:
            log(f"val protocol: {idx + 1}/{len(P.SEEDS)} pairs ({time.perf_counter() - t0:.0f} s)")
        g = gold_pairs[(tr, va)]
        pairs.append({"train_seed": tr, "val_seed": va, "hip": hip, "oracle": g["oracle_dice"],
                      "diff": [round(h - o, 5) for h, o in zip(hip, g["oracle_dice"])],
                      "oracle_perturbed": P.perturbed_of(g), "oracle_spread": g.get("spread")})
    del runner
    n = len(pairs)
    mean_diff = [round(sum(p["diff"][i] for p in pairs) / n, 5) for i in range(len(P.CHECKPOINTS))]
    verdict = P.mean_diff_verdict([p["hip"] for p in pairs], [p["oracle"] for p in pairs],
                                  [p["oracle_perturbed"] for p in pairs])
    out = {"steps": P.CHECKPOINTS, "n_pairs": n, "mean_diff": mean_diff,
           "se": [v["se"] for v in verdict], "noise_floor_mean": [v.get("noise_floor_mean") for v in verdict],
           "max_abs_mean_diff": round(max(abs(d) for d in mean_diff), 5), "tolerance": P.TOL,
           "within": bool(max(abs(d) for d in mean_diff) <= P.TOL),
           "within_ci95": bool(all(v["ci_ok"] for v in verdict)), "checkpoints": verdict,
           "seconds": round(time.perf_counter() - t0, 1),
           "protocol": "tests/valdice_protocol.py (oracle-made warm start; per seed pair 4 epochs x 16 steps; 32 "
                       "held-out scans; strict |mean over pairs of Dice_HIP - Dice_oracle| <= tolerance; within_ci95: "
                       "|mean| + 2 SE <= tolerance)",
           "oracle_source": "tests/golden/valdice_oracle.json", "pairs": pairs}
    log(f"val protocol: mean diff {mean_diff} ({out['seconds']} s)")
    torch.cuda.empty_cache()
    return out


def time_training_loop(args, device, n_images=128):
    """The drop-in loop itself (train.training, ref:octsam/models/training.py:184 -> training_utils.py:27-80) over a
    synthetic n_images-image epoch: its defaults (hipGraphs + encoder lookahead, HIP data path on a side stream),
    the first-batch skip included; timed over the second epoch's training pass (the first captures the graphs),
    validation and evaluation excluded. value = images trained / epoch time."""
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.train import training
    cfg = {"batch_size": args.batch, "epochs": 2, "learning_rate": 1e-3, "topological": bool(args.top),
           "prompt_type": args.prompt, "evaluate": False, "checkpoint": None, "data_seed": 0, "seed": 0,
           "encoder_dtype": args.dtype}
    hist = training(args.model, cfg, data.synthetic_oct(seed=4000, n=n_images),
                    data.synthetic_oct(seed=4001, n=args.batch), device=device, log=lambda *a: None)
    t = hist["train_time_s"][-1]
    trained = n_images - args.batch  # training_utils.py:40-44 skips each epoch's first batch
    out = {"value": round(trained / t, 2), "unit": "imgs/s", "epoch_s": round(t, 4), "images_trained": trained,
           "loader_images": n_images, "train_loss": hist["train_loss"],
           "note": "train.training() defaults (graphs + lookahead, HIP data path); 2nd epoch's training pass"}
    log(f"training loop: {out['value']} imgs/s ({t * 1e3:.1f} ms per {n_images}-image epoch)")
    return out


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args, batch_cpu):
    """CPU oracle step (oracle/step_ref.py: transformers SamModel fp32 + restated DiceCE/topo + Adam) timed on
    this host's cores: the headline sample is batch 1 (one image, all its prompts) with the
    bench's --top, 1 warm-up + cpu_steps timed steps; beside it batch 1 with the other --top setting
    (configs[0] is top off) and one batch-8 step (configs[1]/[2]'s batch) — bounded, so the default bench
    finishes in minutes."""
    from oracle.step_ref import CpuReferenceStep
    # the GPU box shows the whole machine's CPUs; this job's share is OMP_NUM_THREADS (16 there)
    ncores = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    ncores = min(ncores, share) if share > 0 else min(ncores, 16)
    torch.set_num_threads(ncores)

    def timed(top, b, steps, warm):
        step = CpuReferenceStep(args.model, topological=top, seed=0)
        for _ in range(warm):
            step.step(b)
        t0 = time.time()
        for _ in range(steps):
            step.step(b)
        dt = time.time() - t0
        log(f"cpu baseline: batch {int(b['gt_u8'].shape[0])} top={top}: {dt / steps:.2f} s/step")
        return int(b["gt_u8"].shape[0]) * steps / dt

    one = {k: (v[:1] if isinstance(v, torch.Tensor) and v.dim() > 0 else v) for k, v in batch_cpu.items()}
    value = timed(bool(args.top), one, args.cpu_steps, 1)
    points = [{"batch": 1, "top": not bool(args.top), "steps": args.cpu_steps,
               "imgs_per_s": round(timed(not bool(args.top), one, args.cpu_steps, 1), 5)}]
    if args.cpu_batch8:
        points.append({"batch": int(batch_cpu["gt_u8"].shape[0]), "top": bool(args.top), "steps": 1,
                       "imgs_per_s": round(timed(bool(args.top), batch_cpu, 1, 0), 5)})
    n_prompts = int(one["gt_u8"].shape[1])
    return {"value": round(value, 5), "unit": "imgs/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"{args.cpu_steps} timed steps (+1 warm-up) of batch 1 ({n_prompts} {args.prompt}), "
                      f"--top={bool(args.top)}, fp32, oracle/step_ref.py on {ncores} host threads",
            "points": points}


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(args, cmd=None) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes (one per GPU, RCCL rendezvous on
    127.0.0.1) as children — before this process touches the GPU — relay rank 0's JSON line, return the
    worst exit code. torchrun's own environment (WORLD_SIZE set) skips this."""
    import subprocess
    port = str(_free_port())
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, WORLD_SIZE=str(args.gpus), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(cmd, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    out = procs[0].communicate()[0]
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    sys.stdout.write(out)
    sys.stdout.flush()
    return max(rcs, key=abs)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    pg = None
    if world > 1 or "WORLD_SIZE" in os.environ:  # a launcher's ranks (torchrun; world 1 included): RCCL
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)
        pg = dist.group.WORLD
    from dilabhelmholtzoct_amd import data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep, class_confusion, mean_dice, predict_masks

    processor = data.make_processor()
    batch_cpu = make_batch(args, rank, device, processor)
    if pg is not None:  # global-N padding: every rank pads prompts to the global max (single-process collate)
        import torch.distributed as dist
        n = torch.tensor([batch_cpu["gt_u8"].shape[1]], device=device)
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        batch_cpu = data.pad_prompts(batch_cpu, int(n.item()))
    batch = data.to_device_batch(batch_cpu, device)
    N = int(batch["gt_u8"].shape[1])

    model = SamModel.from_pretrained(args.model, seed=0).to(device)
    if args.dtype == "fp16":
        model.set_encoder_dtype(torch.float16)
    pipe = bool(args.pipeline) and not args.eager
    step = FusedTrainStep(model, lr=1e-3, topological=bool(args.top), process_group=pg, graphs=not args.eager,
                          pipeline=pipe)
    step.fork_topo = bool(args.fork_topo)
    if args.gemm_fast_path != 1:  # (A/B of octsam_gemm's paths, e.g. 8193: the 8-phase kernel instead of the ping-pong one)
        from dilabhelmholtzoct_amd import _lib
        _lib.load().octsam_gemm_set_fast_path(args.gemm_fast_path)

    def barrier():
        if pg is not None:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    log(f"rank {rank}: N={N} prompts/image, warm-up")
    # with the encoder lookahead, the last step of each loop names no next batch: nothing of a timed step runs
    # before the timer starts, and the timed region holds exactly `steps` encoder passes
    for i in range(args.warmup):
        step.step(batch, next_batch=batch if i + 1 < args.warmup else None)
    step.flush()
    barrier()
    log(f"rank {rank}: timing {args.steps} steps")
    t0 = time.perf_counter()
    loss = None
    for i in range(args.steps):
        loss = step.step(batch, next_batch=batch if i + 1 < args.steps else None)
    step.flush()  # a deferred (overlapped) update belongs to the timed work
    barrier()
    dt = time.perf_counter() - t0
    # the same graphs without the lookahead hint (each step runs its own encoder in line): the sequential rate
    seq_ms = None
    if pipe:
        nseq = max(3, args.steps // 2)
        barrier()
        t1 = time.perf_counter()
        for _ in range(nseq):
            step.step(batch)
        step.flush()
        barrier()
        seq_ms = (time.perf_counter() - t1) * 1e3 / nseq
        log(f"rank {rank}: sequential (no lookahead) {seq_ms:.2f} ms/step")
    # Roofline of the dominant kernel: HIP events around each of its launches. Graph replays run no
    # Python, so the launches are timed in `roof_steps` eager steps of the same batch right after the
    # timed region (same kernels, shapes and stream); rocprofv3 over the graph run must agree. The same
    # eager steps time the encoder attention kernels, the patch embedding and the decoder fwd / bwd (the
    # north_star's roofline split: MFMA share of encoder attention, HBM GB/s of the patch-embed/decoder path).
    timer = GemmEventTimer() if not args.no_events and args.roof_steps > 0 else None
    split = {}
    if timer:
        from dilabhelmholtzoct_amd import kernels as Kmod
        from dilabhelmholtzoct_amd.decoder import MaskDecoder
        P = args.batch * N
        hidden = model.config.vision.hidden_size
        timers = {
            "attn": CallTimer(Kmod, "vit_attention", attn_flops),
            "patch": CallTimer(Kmod, "patchify_bf16", lambda px, out: px.numel() * 4.0 + out.numel() * 2.0),
            "dec_fwd": CallTimer(MaskDecoder, "forward_impl", lambda *a, **k: P * DEC_FWD_BYTES_PER_PROMPT),
            "dec_bwd": CallTimer(MaskDecoder, "backward_impl", lambda *a, **k: P * DEC_BWD_BYTES_PER_PROMPT),
        }
        graphs = step.graphs
        step.graphs = False
        timer.__enter__()
        for t in timers.values():
            t.__enter__()
            t.active = True
        timer.active = True
        for _ in range(args.roof_steps):
            step.step(batch)
        step.flush()
        timer.active = False
        for t in timers.values():
            t.active = False
            t.__exit__()
        timer.__exit__()
        step.graphs = graphs
        ams, an, aflops = timers["attn"].result()
        pms, pn, pbytes = timers["patch"].result()
        fms, fn_, fbytes = timers["dec_fwd"].result()
        bms, bn, bbytes = timers["dec_bwd"].result()
        if an:
            a_tf = aflops / (ams * 1e-3) / 1e12
            split["encoder_attention"] = {
                "bound": "mfma", "achieved": round(a_tf, 2), "peak": MI355X_BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                "frac": round(a_tf / MI355X_BF16_DENSE_TFLOPS, 4), "launches": an,
                "avg_launch_us": round(ams * 1e3 / an, 2),
                "work": "4*T^2*head_dim*heads*sequences per launch (global T=4096, windowed T=196 padded)"}
        if fn_ and bn:
            dbytes = pbytes + fbytes + bbytes
            dms = pms + fms + bms
            gbs = dbytes / (dms * 1e-3) / 1e9
            split["decoder_hbm"] = {
                "bound": "hbm", "achieved": round(gbs, 1), "peak": MI355X_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / MI355X_HBM_GBS, 4),
                "ms_per_step": {"patch_embed": round(pms / args.roof_steps, 3),
                                "decoder_fwd": round(fms / args.roof_steps, 3),
                                "decoder_bwd": round(bms / args.roof_steps, 3)},
                "work": f"patch-embed 18 B/pixel-triple (fp32 in, bf16 out); decoder {DEC_FWD_BYTES_PER_PROMPT / 1e6:.1f} "
                        f"MB fwd + {DEC_BWD_BYTES_PER_PROMPT / 1e6:.1f} MB bwd per prompt (SURVEY.md §8(d): 12 E + "
                        f"24 E, E = 4096*256*2 B), {P} prompts"}
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
            tj = traffic_json(args)
            traffic_set = None
            if os.path.exists(tj):
                tjd = json.load(open(tj))
                traffic = round(tjd["hbm_bytes_per_launch"])
                traffic_set = ("the same launch set as compulsory_bytes_per_launch (" + tjd["kernel"] + ")"
                               if "," in tjd["kernel"] else
                               f"{tjd['kernel']} launches only (compulsory_bytes_per_launch averages the whole family)")
            roof = {"bound": "mfma", "kernel": dominant_name(args),
                    "achieved": round(achieved, 2), "peak": MI355X_BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / MI355X_BF16_DENSE_TFLOPS, 4), "traffic": traffic,
                    "traffic_source": os.path.relpath(tj, ROOT) if traffic is not None else None,
                    "traffic_launch_set": traffic_set,
                    "compulsory_bytes_per_launch": round(timer.bytes / n),
                    "launches": n, "avg_launch_us": round(ms * 1e3 / n, 2),
                    "share_of_step": round(ms / args.roof_steps / (dt * 1e3 / args.steps), 4)}
            roof["family_by_intensity"] = timer.by_bound()
            roof.update(split)

    e2e = None
    if args.e2e_steps > 0 and not args.eager:
        e2e = end_to_end(args, step, device, rank, world, pg)
    topo_all = None
    if args.topo_all and args.top and rank == 0 and world == 1:
        topo_all = topo_all_sensitivity(args, model, batch)
    top_off = None
    if args.top_off and args.top and rank == 0 and world == 1:
        top_off = top_off_leg(args, model, batch, steps=args.steps)
    loop = None
    if args.loop_images and rank == 0 and world == 1 and not args.eager:
        loop = time_training_loop(args, device, args.loop_images)

    log(f"rank {rank}: {dt * 1e3 / args.steps:.2f} ms/step")
    val_dice = val_metrics = val_proto = None
    if args.val and rank == 0:
        vb = data.to_device_batch(make_batch(argparse.Namespace(batch=args.val, prompt=args.prompt), 999, device,
                                             processor), device)
        masks = predict_masks(model, vb)
        val_dice = round(mean_dice(class_confusion(masks, vb["gt_u8"], vb["mask_values"])), 5)
        from dilabhelmholtzoct_amd.metrics import EvalAccumulator
        acc = EvalAccumulator()
        acc.add(masks, vb["gt_u8"], vb["mask_values"])
        val_metrics = {k: round(v, 5) for k, v in acc.compute()["mean"].items()}
    if args.val_protocol and rank == 0 and world == 1 and args.model == "facebook/sam-vit-base":
        val_proto = val_protocol(args, device)

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
            "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "bf16" else "fp16 encoder, bf16 decoder (fp32 master weights)",
            "data": f"synthetic OCT-like 496x512 label maps -> 1024x1024 processed images, {N} "
                    f"{'point' if args.prompt == 'points' else 'box'} prompts/image (batch max), random-init "
                    f"weights (seed 0)",
            "config": {"workload": workload_name(args), "model": args.model, "global_batch": args.batch * world,
                       "prompts_per_image": N, "prompt": args.prompt, "top": bool(args.top),
                       "parallelism": f"dp{world}",
                       "process_group": None if pg is None else "nccl",
                       "exec": "eager" if args.eager else
                       ("hipgraph + encoder lookahead (next step's frozen encoder on a side stream during this "
                        "step's decoder; each timed step runs its own encoder)" if pipe else "hipgraph")},
            "sequential_ms_per_step": None if seq_ms is None else round(seq_ms, 3),
            "loss_last_step": {"dice": loss_h[0], "ce": loss_h[1], "topo": loss_h[2], "total": loss_h[3]},
            "val_dice_protocol": val_proto,
            "val_dice_after_timed_steps": val_dice,
            "val_metrics_mean": val_metrics,
            "data_path": data_path,
            "value_end_to_end": e2e["value"] if e2e else None,
            "end_to_end": e2e,
            "training_loop": loop,
            "topo_mode_all": topo_all,
            "top_off": top_off,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
