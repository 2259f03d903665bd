"""SAM configuration mirroring transformers' SamConfig / SamVisionConfig / SamMaskDecoderConfig /
SamPromptEncoderConfig (hf:configuration_sam.py), with the hub presets the reference selects by
name in ``--base_model`` (ref:octsam/models/training.py:27-28). The vit-l / vit-h values are the
public hub configs (not present offline), stated explicitly here."""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class VisionConfig:
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    global_attn_indexes: tuple = (2, 5, 8, 11)
    output_channels: int = 256
    image_size: int = 1024
    patch_size: int = 16
    window_size: int = 14
    layer_norm_eps: float = 1e-6
    num_pos_feats: int = 128
    mlp_ratio: float = 4.0
    initializer_range: float = 0.02

    @property
    def mlp_dim(self) -> int:
        return int(self.hidden_size * self.mlp_ratio)

    @property
    def scale(self) -> int:  # SamPositionalEmbedding init std (hf:configuration_sam.py:125)
        return self.hidden_size // 2


@dataclass
class DecoderConfig:
    hidden_size: int = 256
    mlp_dim: int = 2048
    num_hidden_layers: int = 2
    num_attention_heads: int = 8
    attention_downsample_rate: int = 2
    num_multimask_outputs: int = 3
    iou_head_depth: int = 3
    iou_head_hidden_dim: int = 256
    layer_norm_eps: float = 1e-6


@dataclass
class PromptConfig:
    hidden_size: int = 256
    image_size: int = 1024
    patch_size: int = 16
    mask_input_channels: int = 16
    num_point_embeddings: int = 4
    layer_norm_eps: float = 1e-6

    @property
    def image_embedding_size(self) -> int:
        return self.image_size // self.patch_size


@dataclass
class SamConfig:
    vision: VisionConfig = field(default_factory=VisionConfig)
    decoder: DecoderConfig = field(default_factory=DecoderConfig)
    prompt: PromptConfig = field(default_factory=PromptConfig)
    initializer_range: float = 0.02


PRESETS = {
    "facebook/sam-vit-base": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                  global_attn_indexes=(2, 5, 8, 11)),
    "facebook/sam-vit-large": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                   global_attn_indexes=(5, 11, 17, 23)),
    "facebook/sam-vit-huge": dict(hidden_size=1280, num_hidden_layers=32, num_attention_heads=16,
                                  global_attn_indexes=(7, 15, 23, 31)),
    "wanglab/medsam-vit-base": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                                    global_attn_indexes=(2, 5, 8, 11)),
}


def config_for(name: str, **vision_overrides) -> SamConfig:
    """SamConfig for a hub model name (or a short alias vit-b / vit-l / vit-h)."""
    alias = {"vit-b": "facebook/sam-vit-base", "vit-l": "facebook/sam-vit-large",
             "vit-h": "facebook/sam-vit-huge", "sam-vit-base": "facebook/sam-vit-base",
             "sam-vit-large": "facebook/sam-vit-large", "sam-vit-huge": "facebook/sam-vit-huge"}
    key = alias.get(name, name)
    if key not in PRESETS:
        raise ValueError(f"unknown SAM model {name!r}; known: {sorted(PRESETS)}")
    v = dict(PRESETS[key])
    v.update(vision_overrides)
    return SamConfig(vision=VisionConfig(**v))
