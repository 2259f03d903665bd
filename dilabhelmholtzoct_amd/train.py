"""The OCT-SAM training step and loop on liboctsam_hip.so.

``FusedTrainStep`` is one iteration of ref:octsam/models/training_utils.py:46-69 on HBM-resident
inputs: frozen ViT encoder forward -> prompt encoder -> mask decoder forward -> fused post-processing
+ DiceCE (+ topological loss) -> decoder backward -> Adam, all as HIP kernels with no torch autograd in
between. In data-parallel runs the flat decoder gradient is all-reduced (RCCL) before Adam.

``training(base_model, config)`` mirrors training_utils.training (:27-80): first-batch skip per
epoch (:40-44), epoch loss / len(dataloader) (:70), validate_model with the reference's double
accumulation (:351-379), state_dict save (:77) and the per-class Dice evaluation (:82-270, the
metric the reference reports as "Mean dice").
"""
from __future__ import annotations

import math
import os
import time

import torch

from . import kernels as K
from .losses import dicece_forward_backward, postproc_backward, postproc_forward, topo_forward_backward
from .model import SamModel


class FusedTrainStep:
    def __init__(self, model: SamModel, lr: float = 1e-3, weight_decay: float = 0.0, topological: bool = False,
                 lamda: float = 0.1, interp: int = 50, betas=(0.9, 0.999), eps: float = 1e-8,
                 topo_mode: str = "first", process_group=None):
        self.model = model
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.topological, self.lamda, self.interp, self.topo_mode = topological, lamda, interp, topo_mode
        dec = model.mask_decoder
        self.exp_avg = torch.zeros_like(dec.flat, requires_grad=False)
        self.exp_avg_sq = torch.zeros_like(dec.flat, requires_grad=False)
        self.t = 0
        self.pg = process_group
        self._pe = None

    def image_pe(self):
        G = self.model.shared_image_embedding.positional_embedding
        tag = (G._version, G.data_ptr())
        if self._pe is None or self._pe[0] != tag:
            self._pe = (tag, self.model.image_pe())
        return self._pe[1]

    @torch.no_grad()
    def forward_backward(self, pixel_values, gt_u8, input_boxes=None, input_points=None, input_labels=None,
                         crop=(992, 1024), orig=(496, 512), global_batch=None, backward=True):
        """Returns a device float64 tensor [4] = (dice, ce, topo, total). With backward=True leaves the
        decoder gradient in mask_decoder.flat_grad. global_batch: images in the global (all-rank) batch,
        which fixes the topological loss's batch nesting."""
        model = self.model
        dec = model.mask_decoder
        emb = model.vision_encoder.forward_nhwc(pixel_values)
        tokens = model.prompt_tokens(input_points, input_labels, input_boxes)
        B, N = tokens.shape[:2]
        H, W = orig
        low, _, saved = dec.forward_impl(emb, self.image_pe(), tokens,
                                         model.prompt_encoder.no_mask_embed.weight.detach(), False)
        gt = gt_u8.reshape(B * N, H, W)
        masks, dpart = postproc_forward(low.view(B * N, 256, 256), crop, orig, gt)
        masks = masks.view(B, N, H, W)
        loss3, dmask = dicece_forward_backward(masks, gt_u8.view(B, N, H, W), dpart)
        topo = 0.0
        if self.topological:
            topo = topo_forward_backward(masks, gt_u8.view(B, N, H, W), dmask if backward else None,
                                         lamda=self.lamda, interp=self.interp, feat_d=1, loss_q=2,
                                         mode=self.topo_mode, global_batch=global_batch)
        if backward:
            dlow = postproc_backward(dmask.view(B * N, H, W), 256, crop, orig)
            dec.backward_impl(saved, dlow.view(B, N, 1, 256, 256))
        loss = torch.empty(4, device=loss3.device, dtype=torch.float64)
        loss[0:2] = loss3[0:2]
        loss[2] = topo
        loss[3] = loss3[2] + topo
        return loss

    @torch.no_grad()
    def allreduce_grads(self, n_local=None, n_global=None):
        """Data-parallel gradient of the global-batch loss: every loss term is a per-image mean, so the
        global gradient is sum_r n_r g_r / sum_r n_r (n = images on the rank; equal shards -> plain mean).
        One RCCL all-reduce of the flat fp32 decoder gradient (16 MB for vit-b)."""
        if self.pg is None:
            return
        allreduce_weighted(self.model.mask_decoder.flat_grad, self.pg, n_local, n_global)

    @torch.no_grad()
    def optimizer_step(self):
        dec = self.model.mask_decoder
        self.t += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.t
        bc2 = 1.0 - b2 ** self.t
        K.adam(dec.flat, dec.flat_grad, self.exp_avg, self.exp_avg_sq, beta1=b1, beta2=b2, eps=self.eps,
               weight_decay=self.wd, step_size=self.lr / bc1, bc2_sqrt=math.sqrt(bc2), params_bf16=dec.flat_b16)

    def step(self, batch: dict, n_global=None):
        """batch: device tensors from data.process_batch/to_device_batch. n_global: images in the global
        batch (data parallel; None = this rank's batch is the whole batch)."""
        crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
        orig = tuple(int(v) for v in batch["original_sizes"][0])
        n_local = int(batch["pixel_values"].shape[0])
        loss = self.forward_backward(batch["pixel_values"], batch["gt_u8"], input_boxes=batch.get("input_boxes"),
                                     input_points=batch.get("input_points"), input_labels=batch.get("input_labels"),
                                     crop=crop, orig=orig, global_batch=n_global)
        self.allreduce_grads(n_local, n_global)
        self.optimizer_step()
        return loss


def allreduce_weighted(t: torch.Tensor, pg, n_local=None, n_global=None):
    """t <- sum_r n_r t_r / sum_r n_r over the process group (n = None: plain mean over ranks)."""
    import torch.distributed as dist
    world = dist.get_world_size(pg)
    if n_local is None or n_global is None or n_local * world == n_global:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
        t.div_(world)
        return t
    t.mul_(float(n_local))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
    t.div_(float(n_global))
    return t


# --------------------------------------------------------------------------------- evaluation
@torch.no_grad()
def predict_masks(model: SamModel, batch: dict) -> torch.Tensor:
    """Post-processed logits [B, N, H, W] (training_utils.py:121-125)."""
    crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
    orig = tuple(int(v) for v in batch["original_sizes"][0])
    out = model(pixel_values=batch["pixel_values"], input_boxes=batch.get("input_boxes"),
                input_points=batch.get("input_points"), multimask_output=False)
    B, N = out.pred_masks.shape[:2]
    masks, _ = postproc_forward(out.pred_masks.reshape(B * N, 256, 256).float().contiguous(), crop, orig)
    return masks.view(B, N, orig[0], orig[1])


@torch.no_grad()
def class_confusion(masks: torch.Tensor, gt_u8: torch.Tensor, mask_values: torch.Tensor, num_classes: int = 14):
    """Per-class pooled (tp, fp, fn) of sigmoid(mask) > 0.5 vs gt, with the reference's early break when a
    background-valued prompt follows the first one (training_utils.py:126-134). int64 [C, 3]."""
    conf = torch.zeros(num_classes, 3, dtype=torch.int64)
    pred = masks > 0.0  # sigmoid(x) > 0.5  <=>  x > 0
    gt = gt_u8.bool()
    tp = (pred & gt).sum((2, 3)).cpu()
    fp = (pred & ~gt).sum((2, 3)).cpu()
    fn = (~pred & gt).sum((2, 3)).cpu()
    mv = mask_values.cpu()
    B, N = mv.shape
    for b in range(B):
        for c in range(N):
            v = int(mv[b, c])
            if v == 0 and c > 0:
                break
            conf[v, 0] += tp[b, c]
            conf[v, 1] += fp[b, c]
            conf[v, 2] += fn[b, c]
    return conf


def mean_dice(conf: torch.Tensor) -> float:
    """'Mean dice' of training_utils.py:156,246: mean over classes of 2tp/(2tp+fp+fn) (0 if empty)."""
    d = []
    for tp, fp, fn in conf.tolist():
        den = 2 * tp + fp + fn
        d.append(2 * tp / den if den else 0.0)
    return sum(d) / len(d)


# --------------------------------------------------------------------------------- training loop (A1)
def global_batches(n_items: int, batch_size: int, world: int = 1, rank: int = 0, shuffle: bool = False,
                   seed: int = 0, epoch: int = 0):
    """Per-rank index lists of every global batch, in loader order. The global loader is the reference's
    DataLoader(batch_size=batch_size * world, shuffle) (training_utils.py:286); rank r takes a contiguous
    slice of each global batch, so the first-batch skip (:40-44) and len(dataloader) (:70) refer to the
    global order. A ragged last batch is split as evenly as possible (a rank may get none)."""
    order = list(range(n_items))
    if shuffle:
        g = torch.Generator().manual_seed(seed * 1000003 + epoch)
        order = torch.randperm(n_items, generator=g).tolist()
    G = batch_size * world
    out = []
    for s in range(0, n_items, G):
        gb = order[s:s + G]
        q, r = divmod(len(gb), world)
        lo = rank * q + min(rank, r)
        out.append(gb[lo:lo + q + (1 if rank < r else 0)])
    return out


def _collective_max(v: int, pg) -> int:
    if pg is None:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.int64, device=_pg_device(pg))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
    return int(t.item())


def _collective_sum(t: torch.Tensor, pg) -> torch.Tensor:
    if pg is None:
        return t
    import torch.distributed as dist
    dev = _pg_device(pg)
    u = t.to(dev)
    dist.all_reduce(u, op=dist.ReduceOp.SUM, group=pg)
    return u.to(t.device)


def _pg_device(pg):
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(pg) == "nccl" else torch.device("cpu")


def _load_split(config: dict, split: str):
    import datasets
    return datasets.load_from_disk(config["dataset"])[split]


def _batch_for(items, processor, prompt, n_target, device):
    from . import data
    b = data.process_batch(processor, data.custom_collate(items), prompt)
    b = data.pad_prompts(b, n_target)
    return data.to_device_batch(b, device)


def _n_prompts(items):
    return max((len(it[3]) for it in items), default=0)


def training(base_model: str, config: dict, train_data=None, valid_data=None, device=None, process_group=None,
             log=print):
    """ref:octsam/models/training_utils.py:27-80 on liboctsam_hip.so. config keys as the reference CLI builds
    them (training.py): learning_rate, weight_decay, epochs, batch_size, shuffle, topological, prompt_type,
    checkpoint, display_name, time, evaluate, dataset (HF save_to_disk path, used when train_data /
    valid_data are not given). Returns {"train_loss": [...], "valid_loss": [...], "dice": per-class list,
    "mean_dice": float, "checkpoint": path or None}.

    Data parallel (process_group given): every rank processes its slice of each global batch; prompts are
    padded to the global batch N; gradients are combined as the single-process loss would be."""
    from . import data
    from .model import SamModel
    import torch.distributed as dist
    pg = process_group
    world = dist.get_world_size(pg) if pg is not None else 1
    rank = dist.get_rank(pg) if pg is not None else 0
    device = device or torch.device("cuda", torch.cuda.current_device())
    model = SamModel.from_pretrained(base_model, seed=config.get("seed", 0)).to(device)
    processor = data.make_processor()
    train_data = train_data if train_data is not None else _load_split(config, "train")
    valid_data = valid_data if valid_data is not None else _load_split(config, "test")
    prompt = config.get("prompt_type", "bboxes")
    tds = data.SAMDataset(train_data, config, epoch_seed=config.get("data_seed"))
    vds = data.SAMDataset(valid_data, config, epoch_seed=config.get("data_seed"))
    bs = int(config.get("batch_size", 2))
    step = FusedTrainStep(model, lr=config.get("learning_rate", 1e-3), weight_decay=config.get("weight_decay", 0.0),
                          topological=bool(config.get("topological", False)),
                          topo_mode=config.get("topo_mode", "first"), process_group=pg)
    hist = {"train_loss": [], "valid_loss": []}
    for epoch in range(int(config.get("epochs", 10))):
        tds.epoch = epoch
        batches = global_batches(len(tds), bs, world, rank, bool(config.get("shuffle", False)),
                                 config.get("data_seed") or 0, epoch)
        epoch_loss = 0.0
        for bi, idx in enumerate(batches):
            if bi == 0:  # training_utils.py:40-44: the first batch of every epoch is skipped
                continue
            n_glob = len(tds) - bi * bs * world if bi == len(batches) - 1 else bs * world
            n_glob = min(n_glob, bs * world)
            items = [tds[i] for i in idx]
            N = _collective_max(_n_prompts(items), pg)
            if idx:
                batch = _batch_for(items, processor, prompt, N, device)
                crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
                orig = tuple(int(v) for v in batch["original_sizes"][0])
                loss = step.forward_backward(batch["pixel_values"], batch["gt_u8"],
                                             input_boxes=batch.get("input_boxes"),
                                             input_points=batch.get("input_points"), crop=crop, orig=orig,
                                             global_batch=n_glob)
                lv = loss[3].double().cpu() * len(idx)
            else:  # nothing on this rank in a ragged last batch: contribute zero gradient
                model.mask_decoder.flat_grad.zero_()
                lv = torch.zeros((), dtype=torch.float64)
            step.allreduce_grads(len(idx), n_glob)
            step.optimizer_step()
            epoch_loss += float(_collective_sum(lv.reshape(1), pg)[0]) / n_glob  # the .item() of :69
        epoch_loss /= len(batches)
        vloss = validate_model(step, vds, processor, bs, config, world, rank, pg, device)
        hist["train_loss"].append(epoch_loss)
        hist["valid_loss"].append(vloss)
        if rank == 0:
            log(f"EPOCH: {epoch}, Train Loss: {epoch_loss}, Valid Loss: {vloss}")
    ckpt = None
    if config.get("checkpoint") and rank == 0:
        os.makedirs(config["checkpoint"], exist_ok=True)
        ckpt = os.path.join(config["checkpoint"], f"{config.get('display_name', 'octsam')}_{config.get('time', '')}.pt")
        torch.save(model.state_dict(), ckpt)  # training_utils.py:77 (HF state-dict keys)
    hist["checkpoint"] = ckpt
    if config.get("evaluate", True):
        conf = evaluate_confusion(model, vds, processor, bs, prompt, world, rank, pg, device)
        hist["dice"] = class_dice(conf)
        hist["mean_dice"] = mean_dice(conf)
        if rank == 0:
            log(f"Mean dice: {hist['mean_dice']}")
    return hist


@torch.no_grad()
def validate_model(step: FusedTrainStep, vds, processor, bs, config, world=1, rank=0, pg=None, device=None):
    """ref:training_utils.py:351-379, including its double accumulation: every batch adds the DiceCE loss
    and then DiceCE (+ topo) again, divided by len(valid_dl)."""
    prompt = config.get("prompt_type", "bboxes")
    batches = global_batches(len(vds), bs, world, rank)
    total = 0.0
    for bi, idx in enumerate(batches):
        n_glob = min(bs * world, len(vds) - bi * bs * world)
        items = [vds[i] for i in idx]
        N = _collective_max(_n_prompts(items), pg)
        lv = torch.zeros((), dtype=torch.float64)
        if idx:
            batch = _batch_for(items, processor, prompt, N, device)
            crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
            orig = tuple(int(v) for v in batch["original_sizes"][0])
            loss = step.forward_backward(batch["pixel_values"], batch["gt_u8"], input_boxes=batch.get("input_boxes"),
                                         input_points=batch.get("input_points"), crop=crop, orig=orig,
                                         global_batch=n_glob, backward=False).cpu()
            dicece = loss[3] - loss[2]
            lv = (dicece + loss[3]) * len(idx)
        total += float(_collective_sum(lv.reshape(1), pg)[0]) / n_glob
    return total / max(len(batches), 1)


@torch.no_grad()
def evaluate_confusion(model, vds, processor, bs, prompt, world=1, rank=0, pg=None, device=None):
    """Pooled per-class (tp, fp, fn) over the validation set (evaluate_metrics, training_utils.py:113-156),
    summed over ranks."""
    conf = torch.zeros(14, 3, dtype=torch.int64)
    for idx in global_batches(len(vds), bs, world, rank):
        if not idx:
            continue
        items = [vds[i] for i in idx]
        batch = _batch_for(items, processor, prompt, _n_prompts(items), device)
        conf += class_confusion(predict_masks(model, batch), batch["gt_u8"], batch["mask_values"])
    return _collective_sum(conf, pg)


def class_dice(conf: torch.Tensor) -> list:
    out = []
    for tp, fp, fn in conf.tolist():
        den = 2 * tp + fp + fn
        out.append(2 * tp / den if den else 0.0)
    return out


def main(argv=None):
    """CLI mirror of ref:octsam/models/training.py (same flags and defaults; W&B, display and pseudocolour
    options are accepted and ignored). --synthetic K trains on K synthetic OCT-like images instead of a
    save_to_disk dataset."""
    import argparse
    import datetime
    p = argparse.ArgumentParser()
    p.add_argument("--project_name", type=str, default="OCT-Mikhail-experiments")
    p.add_argument("--entity", type=str, default="dilab-helmholtz")
    p.add_argument("--base_model", type=str, default="facebook/sam-vit-base")
    p.add_argument("--loss", type=str, default="diceCE")
    p.add_argument("--dataset", type=str, default="custom")
    p.add_argument("--data_directory", type=str, default="/vol/data")
    p.add_argument("--dataset_name", type=str, default="default_preprocessed_at_24-01-10_13.41.28")
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--weight_decay", type=float, default=0)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--bs", type=int, default=2)
    p.add_argument("--shuffle", type=bool, default=False)  # type=bool as in the reference
    p.add_argument("--optimizer", type=str, default="adam")
    p.add_argument("--display_mode", type=str, default="predefined")
    p.add_argument("--display_idx", type=str, default="0, 1, 3")
    p.add_argument("--display_val_nr", type=int, default=1)
    p.add_argument("--display_train_nr", type=int, default=1)
    p.add_argument("--mode", type=int, default=1)
    p.add_argument("--seg_nr", type=int, default=3)
    p.add_argument("--pseudocolor", type=str, default="grayscale")
    p.add_argument("--display_name", type=str, default="")
    p.add_argument("--evaluate", type=bool, default=True)
    p.add_argument("--prompt", type=str, default="bboxes")
    p.add_argument("--top", action="store_true")
    p.add_argument("--synthetic", type=int, default=0, help="train on K synthetic images (no dataset on disk)")
    args = p.parse_args(argv)
    if args.loss != "diceCE" or args.optimizer != "adam":
        raise SystemExit("only --loss diceCE and --optimizer adam exist in the reference")
    if args.pseudocolor != "grayscale":
        raise SystemExit("pseudocolour maps need cv2, which is not available")
    now = datetime.datetime.now().strftime("%y-%m-%d_%H.%M.%S")
    name = args.display_name or (f"{'{:.0e}'.format(args.lr)} lr,{'{:.0e}'.format(args.weight_decay)} wd,"
                                 f"{args.bs} bs, {args.loss} loss, {args.pseudocolor}, {now}")
    config = {"display_name": name, "base_model": args.base_model,
              "dataset": os.path.join(args.data_directory, "datasets", "processed", args.dataset, args.dataset_name),
              "checkpoint": os.path.join(args.data_directory, "models", args.dataset),
              "learning_rate": args.lr, "weight_decay": args.weight_decay, "epochs": args.epochs,
              "batch_size": args.bs, "shuffle": args.shuffle, "optimizer": args.optimizer, "loss": args.loss,
              "time": now, "evaluate": args.evaluate, "topological": args.top, "prompt_type": args.prompt,
              "pseudocolor": None}
    pg = None
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        pg = dist.group.WORLD
    tr = va = None
    if args.synthetic:
        from . import data
        tr = data.synthetic_oct(seed=0, n=args.synthetic)
        va = data.synthetic_oct(seed=1, n=max(1, args.synthetic // 4))
        config["checkpoint"] = None
        config["data_seed"] = 0
    t0 = time.time()
    hist = training(args.base_model, config, tr, va, process_group=pg)
    if pg is None or torch.distributed.get_rank() == 0:
        print(f"done in {time.time() - t0:.1f} s: {hist}")
    if pg is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
