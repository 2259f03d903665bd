"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

CPU fp32 restatement of one training step of ref:octsam/models/training_utils.py:46-69 built from the
reference's own model library (transformers SamModel, the dependency the reference pins at 4.36.2;
5.15.0 installed — identical SAM arithmetic up to rounding) and the restated losses of
oracle/losses_ref.py, with torch.optim.Adam on the mask decoder only. Used for loss/gradient parity
and as bench.py's CPU baseline ("port").
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .losses_ref import dicece_ref, topo_loss_ref


def hf_config(base_model: str):
    from transformers import SamConfig
    from dilabhelmholtzoct_amd.config import config_for
    v = config_for(base_model).vision
    return SamConfig(vision_config=dict(hidden_size=v.hidden_size, num_hidden_layers=v.num_hidden_layers,
                                        num_attention_heads=v.num_attention_heads,
                                        global_attn_indexes=list(v.global_attn_indexes)))


def synthetic_state_dict(base_model: str, seed: int = 0):
    """The deterministic synthetic weights (CPU torch only) used on both sides of a parity check."""
    from dilabhelmholtzoct_amd.model import SamModel
    m = SamModel(base_model)
    m.init_weights(seed=seed)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


class CpuReferenceStep:
    def __init__(self, base_model="facebook/sam-vit-base", topological=False, seed=0, lr=1e-3, weight_decay=0.0,
                 topo_mode="first", state_dict=None, device="cpu", loss_device="cpu"):
        """device: where the fp32 SamModel runs (CPU for the bench baseline; a GPU only to speed up the
        val-Dice parity test); loss_device: where the torch post-processing and losses run (fp32 / f64; the
        persistence and the transport plan are always CPU code)."""
        from transformers import SamModel
        self.model = SamModel(hf_config(base_model)).float()
        self.model.load_state_dict(state_dict if state_dict is not None else synthetic_state_dict(base_model, seed))
        self.device = torch.device(device)
        self.model.to(self.device)
        for name, p in self.model.named_parameters():  # training_utils.py:277-279
            if name.startswith("vision_encoder") or name.startswith("prompt_encoder"):
                p.requires_grad_(False)
        self.opt = torch.optim.Adam(self.model.mask_decoder.parameters(), lr=lr, weight_decay=weight_decay)
        self.topological = topological
        self.topo_mode = topo_mode
        self.loss_device = torch.device(loss_device)

    @torch.no_grad()
    def embed(self, batch):
        """Image embeddings of the frozen encoder (the vision encoder has no trainable weight, so a batch's
        embedding is the same at every step: callers may compute it once and pass it to predict/step)."""
        return self.model.get_image_embeddings(batch["pixel_values"].float().to(self.device))

    def predict(self, batch, image_embeddings=None):
        """Post-processed fp32 logits [B, N, H, W] on loss_device (training_utils.py:56-58 / :121-125).
        image_embeddings: the frozen encoder's output for this batch (embed()), or None to run the encoder."""
        dev = self.device
        if image_embeddings is not None:
            inputs = {"image_embeddings": image_embeddings}
        else:
            inputs = {"pixel_values": batch["pixel_values"].float().to(dev)}
        if "input_boxes" in batch:
            inputs["input_boxes"] = batch["input_boxes"].to(dev)
        if "input_points" in batch:
            inputs["input_points"] = batch["input_points"].to(dev)
        out = self.model(**inputs, multimask_output=False)
        masks = F.interpolate(out.pred_masks.squeeze(2).to(self.loss_device), (1024, 1024), mode="bilinear",
                              align_corners=False)
        rh, rw = (int(v) for v in batch["reshaped_input_sizes"][0])
        oh, ow = (int(v) for v in batch["original_sizes"][0])
        masks = masks[..., :rh, :rw]
        return F.interpolate(masks, (oh, ow), mode="bilinear", align_corners=False)

    def forward_loss(self, batch, image_embeddings=None):
        gt = batch["gt_u8"].to(self.loss_device).double()
        masks = self.predict(batch, image_embeddings)
        loss = dicece_ref(masks, gt)
        topo = torch.zeros((), dtype=torch.float64)
        if self.topological:
            topo = topo_loss_ref(torch.sigmoid(masks.float()), gt.float(), 0.1, feat_d=1, interp=50,
                                 mode=self.topo_mode)
            loss = loss + topo
        return loss, topo, masks

    def step(self, batch, image_embeddings=None):
        self.opt.zero_grad()
        loss, topo, _ = self.forward_loss(batch, image_embeddings)
        loss.backward()
        self.opt.step()
        return float(loss.item())
