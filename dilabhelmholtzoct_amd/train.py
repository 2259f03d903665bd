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
                         crop=(992, 1024), orig=(496, 512)):
        """Returns a device float64 tensor [4] = (dice, ce, topo, total). Leaves the decoder gradient in
        mask_decoder.flat_grad."""
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
            topo = topo_forward_backward(masks, gt_u8.view(B, N, H, W), dmask, lamda=self.lamda, interp=self.interp,
                                         feat_d=1, loss_q=2, mode=self.topo_mode)
        dlow = postproc_backward(dmask.view(B * N, H, W), 256, crop, orig)
        dec.backward_impl(saved, dlow.view(B, N, 1, 256, 256))
        loss = torch.empty(4, device=loss3.device, dtype=torch.float64)
        loss[0:2] = loss3[0:2]
        loss[2] = topo
        loss[3] = loss3[2] + topo
        return loss

    @torch.no_grad()
    def allreduce_grads(self):
        if self.pg is None:
            return
        import torch.distributed as dist
        g = self.model.mask_decoder.flat_grad
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.pg)
        g.div_(dist.get_world_size(self.pg))

    @torch.no_grad()
    def optimizer_step(self):
        dec = self.model.mask_decoder
        self.t += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.t
        bc2 = 1.0 - b2 ** self.t
        K.adam(dec.flat, dec.flat_grad, self.exp_avg, self.exp_avg_sq, beta1=b1, beta2=b2, eps=self.eps,
               weight_decay=self.wd, step_size=self.lr / bc1, bc2_sqrt=math.sqrt(bc2), params_bf16=dec.flat_b16)

    def step(self, batch: dict):
        """batch: device tensors from data.process_batch/to_device_batch."""
        crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
        orig = tuple(int(v) for v in batch["original_sizes"][0])
        loss = self.forward_backward(batch["pixel_values"], batch["gt_u8"], input_boxes=batch.get("input_boxes"),
                                     input_points=batch.get("input_points"), input_labels=batch.get("input_labels"),
                                     crop=crop, orig=orig)
        self.allreduce_grads()
        self.optimizer_step()
        return loss


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
