"""Same-process A/B of the pipelined training step (bench.py's loop: hipGraphs + encoder lookahead, B = 8 boxes,
--top=True) for variants of the step / mask decoder set while the graphs are captured (STEP_VARIANTS: default,
wgrad_off = image-side weight gradients by the split-K tile GEMM, tok_off = token-side ones by the split-K tile
GEMM + reductions + column-sum kernels, fork_topo = resampling + persistence forked beside
the DiceCE backward too (the default since round 5; topo_in_f = not forked), ln_sep = the upscaling LayerNorm2d + GELU backward as its own kernel instead of fused into
the mask-head backward, g4res_off = the decoder's [K | Q' | V] projection on the persistent 8-phase GEMM in plain tile
order, octsam_gemm fast path 1 | 1024 | 2048, while capturing; attn_v2 = the global attention with whole rel_h
tables, two workgroups per CU; n192 = octsam_gemm fast path 24 (256x192 tiles where they fill the waves better, the
8-phase kernels otherwise); pp_unfused = the DiceCE backward and the post-processing row pass as two kernels with
the [B, N, H, W] d-mask between them; t2isum_off = the first block's token->image backward per prompt +
prompt group sums instead of octsam_dec_t2i_bwd_sum; dkeys_joint = the mask head's and the final attention's keys
gradients as one product; dkeys_two = the two-product form; tokgroup_off = every token-side weight gradient as its own
launch instead of the deferred grouped launches; tokflush_block = the deferred group flushed at the end of every
two-way block; n192w = the opt-in 256x192 ping-pong tiles; small_chained = the token-side K <= 256 products on the
chained 64x64 kernel instead of the one-shot one). Interleaved rounds, median of 5 rounds x 20 steps.
Diagnostic only."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dilabhelmholtzoct_amd import _lib, data
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    dev = torch.device("cuda", 0)
    sd = data.SAMDataset(data.synthetic_oct(seed=1000, n=8), {"prompt_type": "bboxes"}, epoch_seed=0)
    batch = data.to_device_batch(data.process_batch(data.make_processor(), data.custom_collate(
        [sd[i] for i in range(8)]), "bboxes"), dev)
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(dev)
    variants = {}
    dec = model.mask_decoder
    # (name, attributes of the step, attributes of the mask decoder read while the graphs are captured)
    VARIANTS = {"default": ({}, {}), "wgrad_off": ({}, {"wide_wgrad": False}), "tok_off": ({}, {"tok_wgrad": False}),
                "fork_topo": ({"fork_topo": True}, {}), "topo_in_f": ({"fork_topo": False}, {}), "ln_sep": ({}, {"fused_ln_bwd": False}),
                "g4res_off": ({}, {}), "attn_v2": ({}, {}), "pp_unfused": ({"fused_pp": False}, {}),
                "n192": ({}, {}), "t2isum_off": ({}, {"t2i_sum": False}),
                "dkeys_joint": ({}, {"fuse_dkeys": True}), "dkeys_two": ({}, {"fuse_dkeys": False}),
                "tokgroup_off": ({}, {"tok_group": False}), "g4w_off": ({}, {}),
                "tokflush_block": ({}, {"tok_flush_block": True}), "n192w": ({}, {}), "small_chained": ({}, {}),
                "default2": ({}, {}),
                "combo": ({"fork_topo": False, "fused_pp": False}, {"fuse_dkeys": False}),
                "combo_g4w": ({"fork_topo": False, "fused_pp": False}, {"fuse_dkeys": False}),
                "topo_pp": ({"fork_topo": False, "fused_pp": False}, {})}
    FAST = {"g4res_off": 1 | 1024 | 2048, "n192": 24, "g4w_off": 1 | 512, "n192w": 1 | 262144, "small_chained": 1 | 65536,
            "combo_g4w": 1 | 512}
    ATTN = {"attn_v2": 2}  # global attention variant while capturing (-1: the library default)
    lib = _lib.load()
    for name in os.environ.get("STEP_VARIANTS", "default,wgrad_off").split(","):
        st_attr, dec_attr = VARIANTS[name]
        st = FusedTrainStep(model, lr=1e-3, topological=True, graphs=True,
                            pipeline=os.environ.get("STEP_PIPELINE", "1") == "1")
        for k, v in st_attr.items():
            setattr(st, k, v)
        saved = {k: getattr(dec, k) for k in dec_attr}
        for k, v in dec_attr.items():
            setattr(dec, k, v)
        lib.octsam_gemm_set_fast_path(FAST.get(name, 1))
        lib.octsam_attention_set_variant(ATTN.get(name, -1))
        for i in range(3):  # capture + warm
            st.step(batch, next_batch=batch if i < 2 else None)
        st.flush()
        lib.octsam_gemm_set_fast_path(1)
        lib.octsam_attention_set_variant(-1)
        for k, v in saved.items():
            setattr(dec, k, v)
        variants[name] = st
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    n = 20
    for _ in range(5):
        for name, st in variants.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                st.step(batch, next_batch=batch if i + 1 < n else None)
            st.flush()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e3 / n)
    print(json.dumps({k: {"median_ms": round(statistics.median(v), 3), "all": [round(x, 3) for x in v]}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
