#!/usr/bin/env python3
"""Per-tensor decoder-gradient error of one HIP step against the fp32 oracle fed the SAME image embeddings (the HIP
encoder's), so the comparison sees only the decoder / post-processing / loss path (diagnostics, test infrastructure:
uses the oracle). States: the val-Dice protocol's oracle-made warm decoder and the random synthetic decoder; topo on
and off. Prints the losses, the global cosine, the per-tensor relative Frobenius errors (worst first) and, per
tensor, the error of the oracle against ITSELF with bf16-rounded embeddings (the operand-rounding floor)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import valdice_protocol as P  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    from oracle.step_ref import CpuReferenceStep
    cuda = torch.device("cuda", 0)
    warm_state, _ = P.load_warm()
    states = {"warm": warm_state, "random": P.base_state()}
    batch = P.host_batches(2001, 8, 0)[0]
    bd = {k: (v.to(cuda) if isinstance(v, torch.Tensor) else v) for k, v in batch.items()}
    crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
    orig = tuple(int(v) for v in batch["original_sizes"][0])
    for sname, state in states.items():
        for top in (False, True):
            ours = SamModel(P.NAME)
            ours.load_state_dict(state)
            ours = ours.to(cuda)
            step = FusedTrainStep(ours, topological=top)
            loss = step.forward_backward(bd["pixel_values"], bd["gt_u8"], input_boxes=bd.get("input_boxes"), crop=crop,
                                         orig=orig).cpu()
            with torch.no_grad():
                e = ours.vision_encoder.forward_nhwc(bd["pixel_values"].float())
            emb = e.view(e.shape[0], 64, 64, 256).permute(0, 3, 1, 2).contiguous().float()
            ours.mask_decoder.bind_param_grads()
            got = {n: p.grad.detach().double().cpu() for n, p in ours.mask_decoder.named_parameters()
                   if p.grad is not None}
            del ours, step
            torch.cuda.empty_cache()

            def oracle_grads(embedding):
                with P.oracle_mode():
                    ref = CpuReferenceStep(P.NAME, topological=top, state_dict=state, device=cuda, loss_device=cuda)
                    ref.opt.zero_grad()
                    rl, rtopo, _ = ref.forward_loss(batch, embedding)
                    rl.backward()
                g = {n: p.grad.double().cpu() for n, p in ref.model.mask_decoder.named_parameters() if p.grad is not None}
                out = (float(rl.detach()), float(torch.as_tensor(rtopo).detach()), g)
                del ref
                torch.cuda.empty_cache()
                return out

            rl, rtopo, rg = oracle_grads(emb)
            _, _, rg16 = oracle_grads(emb.bfloat16().float())
            scale = max(g.norm().item() for g in rg.values())
            rows, fg, fw = [], [], []
            for n, r in rg.items():
                if r.norm().item() < 1e-6 * scale:
                    continue
                fg.append(got[n].flatten())
                fw.append(r.flatten())
                rows.append((n, rel(got[n], r), rel(rg16[n], r), r.norm().item() / scale))
            g_, w_ = torch.cat(fg), torch.cat(fw)
            cos = float((g_ @ w_) / (g_.norm() * w_.norm()))
            rows.sort(key=lambda x: -x[1])
            errs = sorted(x[1] for x in rows)
            print(json.dumps({"state": sname, "topo": top, "hip_loss": [round(float(x), 6) for x in loss.tolist()],
                              "oracle_loss_total": round(rl, 6), "oracle_topo": round(rtopo, 6), "cosine": round(cos, 6),
                              "median_rel": round(errs[len(errs) // 2], 5),
                              "worst": [(n, round(a, 4), round(b, 4), round(s, 4)) for n, a, b, s in rows[:12]]}),
                  flush=True)


if __name__ == "__main__":
    main()
