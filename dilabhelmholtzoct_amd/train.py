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

import numpy as np

import torch

from . import kernels as K
from .losses import (dicece_forward_backward, dicece_pp_rows, dicece_pp_rows_supported, postproc_backward,
                     postproc_forward, pp_rows_finish, topo_device_backward, topo_device_forward, topo_host, topo_index, topo_w2_device)
from .model import SamModel


class _Phases:
    """Tensors that flow between the phases of one step (static across graph replays)."""


class FusedTrainStep:
    """One training step of the reference (training_utils.py:46-69) as four phases:

      E  image encoder forward                        (reads no trainable weight)
      F  prompt tokens, decoder forward, post-processing, DiceCE forward, topo resampling + persistence (PH) and,
         with w2="device" (default), the W2 transport, topo loss and d topo / d map on the GPU (octsam_topo_w2)
      F2 DiceCE backward (the W2 of w2="device" forks beside it when fork_topo)
      B  topo backward, post-processing backward, decoder backward, loss assembly
      then (world > 1) the RCCL all-reduce of the flat decoder gradient and Adam. No host work or device sync sits
      inside a step; w2="host" keeps the round-2 path (pairs D2H after F, octsam_topo_host on the host, H2D before B).

    graphs=True captures E, F, F2 and B as hipGraphs (one pool, replayed in capture order) the first time a
    batch shape is seen, after eager warm-up, and replays them afterwards: no per-kernel host launch cost.
    In data-parallel runs (overlap=True) the all-reduce runs on a side stream and Adam is deferred to the
    next step, after that step's encoder forward has been queued: the gradient exchange overlaps the
    encoder; flush() completes a pending update.

    pipeline=True (graph mode): step(batch, next_batch=...) replays the encoder phase E of next_batch on a
    side stream while this step's decoder phases F / F2 / B run, so the MFMA-bound frozen encoder fills the
    CUs the HBM- and latency-bound decoder kernels leave idle. E reads no trainable weight, so the result is
    the sequential one bit for bit. Two graph sets per batch shape (separate memory pools, the image
    embedding double-buffered by set parity); the next step consumes the prefetched embedding if its inputs
    are the tensors next_batch named (same storage and version), else it runs E itself. Every step still
    runs its own E exactly once (the lookahead is the next step's E, moved earlier)."""

    def __init__(self, model: SamModel, lr: float = 1e-3, weight_decay: float = 0.0, topological: bool = False,
                 lamda: float = 0.1, interp: int = 50, betas=(0.9, 0.999), eps: float = 1e-8,
                 topo_mode: str = "first", process_group=None, graphs: bool = False, overlap: bool = True,
                 pipeline: bool = False, w2: str = "device"):
        self.model = model
        if w2 not in ("device", "host"):
            raise ValueError(f"w2 must be 'device' or 'host', got {w2!r}")
        # "device": the diagrams' transport, the topo loss and its gradient on the GPU (octsam_topo_w2): no host
        # round trip inside the step; "host": octsam_topo_host between the forward and backward graphs (A/B)
        self.w2 = w2
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.topological, self.lamda, self.interp, self.topo_mode = topological, lamda, interp, topo_mode
        dec = model.mask_decoder
        self.exp_avg = torch.zeros_like(dec.flat, requires_grad=False)
        self.exp_avg_sq = torch.zeros_like(dec.flat, requires_grad=False)
        self.t = 0
        self.pg = process_group
        self._pe = None
        self.graphs = graphs
        self.overlap = overlap and process_group is not None
        self._graphs = {}       # batch shape -> captured graphs + static input copies (graph mode), LRU order
        self.captures = 0       # graph sets captured (recaptures after an eviction included)
        self.evictions = 0
        self._pending = None    # (event, ) of an all-reduce whose Adam step has not run yet
        self._side = None
        self.pipeline = pipeline and graphs
        self._enc_stream = None
        # lookahead stream priority: equal to the main stream's (measured: a high-priority lookahead 17.8 -> 21.3
        # ms/step, the step on a high-priority stream instead 17.7 -> 18.0; scripts/prio_ab.py)
        self.enc_priority = 0
        # encoder graph sets the lookahead cycles through (2: the encoder of step t+2 waits for the backward of
        # step t; 3 sets measured the same, 17.72 vs 17.76 ms/step: the encoder stream is busy throughout)
        self.pipeline_sets = 2
        self._prefetch = None   # (encoder set, pixel tag) whose E was replayed ahead on the encoder stream
        self._w2_stream = None  # side stream of the device topological forward (forked in F2, joined before B)
        # w2 = "device": the 50x50 resampling, the persistence and the transport fork beside the DiceCE backward
        # (False: only the transport, the resampling + persistence in F). Same-process A/B (scripts/step_ab3.py):
        # round 3 measured the fork slower (profiles/r03/step_ab_fork_tokdw.log, 17.04 vs 17.13 ms/step); with the
        # fused DiceCE / post-processing row pass of round 4 it is faster, 16.31 -> 16.16 ms pipelined and 18.77 ->
        # 18.55 sequential (profiles/r05/fork_topo_ab.log): the 16-workgroup persistence kernel (348 us) no longer
        # runs alone on the main stream
        self.fork_topo = True
        # DiceCE backward fused with the post-processing adjoint's row pass (no [B, N, H, W] d-mask round trip;
        # False: the round-3 octsam_dicece_bwd + octsam_postproc_bwd path, for A/B)
        self.fused_pp = True
        self._parity = {}       # pixel shape -> parity of the graph sets the next step of that shape uses
        self._esets = {}        # (pixel shape, dtype, parity) -> captured encoder graph E

    def image_pe(self):
        G = self.model.shared_image_embedding.positional_embedding
        tag = (G._version, G.data_ptr())
        if self._pe is None or self._pe[0] != tag:
            self._pe = (tag, self.model.image_pe())
        return self._pe[1]

    # ------------------------------------------------------------------ phases
    def _phase_e(self, st):
        st.emb = self.model.vision_encoder.forward_nhwc(st.pixel_values)

    def _phase_f(self, st, backward):
        model = self.model
        dec = model.mask_decoder
        # the prompt tokens start with the decoder's iou / mask tokens (trainable): built here, after the
        # previous step's Adam, not in E (which may run ahead of that update: DP overlap, pipelining)
        st.tokens = model.prompt_tokens(st.input_points, st.input_labels, st.input_boxes)
        B, N = st.tokens.shape[:2]
        H, W = st.orig
        low, _, st.saved = dec.forward_impl(st.emb, self.image_pe(), st.tokens,
                                            model.prompt_encoder.no_mask_embed.weight.detach(), False)
        gt = st.gt_u8.reshape(B * N, H, W)
        masks, dpart = postproc_forward(low.view(B * N, 256, 256), st.crop, st.orig, gt)
        st.masks = masks.view(B, N, H, W)
        st.dpart = dpart
        st.topo_dev = None
        if self.topological and self.lamda != 0.0:
            entries, maps, midx = topo_index(B, N, self.topo_mode, st.global_batch, masks.device)
            if entries:
                st.topo_dev = (entries, maps, midx)
                if self.w2 == "device" and self.fork_topo:
                    # resampling, persistence and transport run in F2, beside the DiceCE backward
                    st.w2_job = (entries, maps, midx, backward, None)
                    return
                pairs, cnt, vals = topo_device_forward(st.masks, st.gt_u8.view(B, N, H, W), midx, interp=self.interp)
                if self.w2 == "device":  # (default: only the transport beside the DiceCE backward)
                    st.w2_job = (entries, maps, midx, backward, (pairs, cnt, vals))
                elif st.pinned is not None:  # graph mode: async copies into fixed pinned buffers
                    for h, d in zip(st.pinned, (pairs, cnt, vals)):
                        h.copy_(d, non_blocking=True)
                else:
                    st.topo_out = (pairs, cnt, vals)

    def _phase_f2(self, st):
        """DiceCE loss and its gradient, and (w2="device") beside it on a forked side stream the diagrams' W2
        transport, topo loss and topo gradient (octsam_topo_w2; with fork_topo also the 50x50 resampling and the
        persistence) — a few latency-bound workgroups that the DiceCE kernels run beside; B joins the two branches. w2="host": the persistence runs in F and the host's W2 overlaps this phase (it
        waits on an event between the graphs)."""
        B, N, H, W = st.masks.shape
        job = getattr(st, "w2_job", None)
        if job is None:
            self._dicece(st)
            return
        entries, maps, midx, want_grad, diagrams = job
        main = torch.cuda.current_stream()
        if self._w2_stream is None:
            self._w2_stream = torch.cuda.Stream(device=main.device)
        side = self._w2_stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            if diagrams is None:
                pairs, cnt, vals = topo_device_forward(st.masks, st.gt_u8.view(B, N, H, W), midx, interp=self.interp)
            else:
                pairs, cnt, vals = diagrams
            st.topo_loss_dev, st.dp = topo_w2_device(pairs, cnt, vals, entries, maps, lamda=self.lamda, feat_d=1,
                                                     loss_q=2, want_grad=want_grad)
        self._dicece(st)
        main.wait_stream(side)
        if not torch.cuda.is_current_stream_capturing():  # (a captured graph owns its memory)
            for t in (st.topo_loss_dev, st.dp):
                if t is not None:
                    t.record_stream(main)

    def _dicece(self, st):
        """DiceCE loss + backward. fused_pp (default): fused with the post-processing adjoint's row pass, the
        topological loss's maps kept as d-masks for B (losses.dicece_pp_rows); else the [B, N, H, W] d-mask."""
        B, N, H, W = st.masks.shape
        # the fused kernel takes at most 32 prompts and W % 4 == 0; other batches (the reference caps neither) take
        # the two-kernel path, chosen per batch shape (so per captured graph set)
        st.fused_pp = self.fused_pp and dicece_pp_rows_supported(B, N, H, W)
        if st.fused_pp:
            maps = st.topo_dev[1] if st.topo_dev is not None else ()
            st.loss3, st.pp_tmp, st.dkeep = dicece_pp_rows(st.masks, st.gt_u8.view(B, N, H, W), st.dpart, st.crop,
                                                           maps=maps)
            st.dmask = None
        else:
            st.loss3, st.dmask = dicece_forward_backward(st.masks, st.gt_u8.view(B, N, H, W), st.dpart)

    def _topo_host(self, st, backward):
        """-> topo loss (float); in backward mode also fills the device (eager) / pinned (graph) gradient.
        w2 = "device": nothing to do on the host (the loss and gradient were formed in F)."""
        if st.topo_dev is None or self.w2 == "device":
            return 0.0
        entries, maps, midx = st.topo_dev
        if st.pinned is not None:
            pairs_h, cnt_h, vals_h = (t.numpy() for t in st.pinned)
        else:
            pairs_h, cnt_h, vals_h = (t.cpu().numpy() for t in st.topo_out)
        loss, dpred = topo_host(pairs_h, cnt_h, vals_h, entries, maps, lamda=self.lamda, feat_d=1, loss_q=2,
                                want_grad=backward)
        if backward:
            if st.pinned is not None:
                st.dp_pinned.numpy()[...] = dpred
            else:
                st.dp = torch.from_numpy(dpred).to(st.masks.device)
        return loss

    def _phase_b(self, st, backward):
        B, N, H, W = st.masks.shape
        if backward:
            if st.topo_dev is not None:
                if self.w2 == "host" and st.pinned is not None:
                    st.dp.copy_(st.dp_pinned, non_blocking=True)
                if st.fused_pp:
                    topo_device_backward(st.masks, st.topo_dev[2], st.dp, st.dkeep, interp=self.interp, compact=True)
                else:
                    topo_device_backward(st.masks, st.topo_dev[2], st.dp, st.dmask, interp=self.interp)
            if st.fused_pp:
                dlow = pp_rows_finish(st.pp_tmp, st.crop, st.orig, dkeep=st.dkeep,
                                      midx=st.topo_dev[2] if st.topo_dev is not None else None)
            else:
                dlow = postproc_backward(st.dmask.view(B * N, H, W), 256, st.crop, st.orig)
            self.model.mask_decoder.backward_impl(st.saved, dlow.view(B, N, 1, 256, 256))
        loss = st.loss_out
        loss[0:2] = st.loss3[0:2]
        if self.w2 == "device":
            if st.topo_dev is not None:
                loss[2:3].copy_(st.topo_loss_dev)
            else:
                loss[2:3].zero_()
        elif st.pinned is not None:
            loss[2:3].copy_(st.topo_pinned, non_blocking=True)
        else:
            loss[2] = st.topo_val
        loss[3] = st.loss3[2] + loss[2]

    # ------------------------------------------------------------------ eager / graph drivers
    def _state(self, pixel_values, gt_u8, input_boxes, input_points, input_labels, crop, orig, global_batch):
        st = _Phases()
        st.pixel_values, st.gt_u8 = pixel_values, gt_u8
        st.input_boxes, st.input_points, st.input_labels = input_boxes, input_points, input_labels
        st.crop, st.orig, st.global_batch = tuple(crop), tuple(orig), global_batch
        st.pinned = None
        st.loss_out = torch.empty(4, device=pixel_values.device, dtype=torch.float64)
        return st

    @torch.no_grad()
    def forward_backward(self, pixel_values, gt_u8, input_boxes=None, input_points=None, input_labels=None,
                         crop=(992, 1024), orig=(496, 512), global_batch=None, backward=True, between=None,
                         next_inputs=None):
        """Returns a device float64 tensor [4] = (dice, ce, topo, total). With backward=True leaves the
        decoder gradient in mask_decoder.flat_grad. global_batch: images in the global (all-rank) batch,
        which fixes the topological loss's batch nesting. between: optional callable run on
        the host while the GPU works on the step (after the forward is queued)."""
        if self.graphs and backward:
            return self._graph_forward_backward(pixel_values, gt_u8, input_boxes, input_points, input_labels, crop,
                                                orig, global_batch, between, next_inputs)
        out = self._eager_forward_backward(pixel_values, gt_u8, input_boxes, input_points, input_labels, crop, orig,
                                           global_batch, backward)
        if between is not None:
            between()
        return out

    def _eager_forward_backward(self, pixel_values, gt_u8, input_boxes, input_points, input_labels, crop, orig,
                                global_batch, backward):
        st = self._state(pixel_values, gt_u8, input_boxes, input_points, input_labels, crop, orig, global_batch)
        self._phase_e(st)
        self._finish_pending()
        self._phase_f(st, backward)
        self._phase_f2(st)
        st.topo_val = self._topo_host(st, backward)
        self._phase_b(st, backward)
        return st.loss_out

    def _graph_key(self, *ts):
        return tuple((None if t is None else (tuple(t.shape), t.dtype)) for t in ts)

    # captured step graphs kept, least recently used evicted (one set per batch shape: B, the prompt count N, prompt
    # kind; x2 encoder-lookahead parities). N is the batch's largest component count and cannot be bucketed: the
    # collate's zero-padded prompts enter the reference's DiceCE mean, so padding N further would change the loss.
    # A set's private pool holds the step's activations, ~1.5-2 GB at B = 8, N ~ 21 (vit-b), so 32 sets stay far
    # below 288 GB; `captures` / `evictions` count recaptures (a capture = one eager pass + 3 captures + a sync).
    MAX_GRAPHS = 32

    def _encoder_set(self, ekey, pixel_values):
        """Captured encoder graph E for one pixel shape and parity: its own memory pool, a static pixel input and
        the image embedding it writes (read by every decoder graph set of that parity)."""
        es = self._esets.get(ekey)
        if es is not None:
            return es
        px = pixel_values.detach().to(pixel_values.device, copy=True)
        st = _Phases()
        st.pixel_values = px
        ge = torch.cuda.CUDAGraph()
        dev = px.device
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(ge, stream=s, capture_error_mode="relaxed"):
                self._phase_e(st)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        es = {"graph": ge, "pixel": px, "emb": st.emb, "src": None, "e_done": torch.cuda.Event(),
              "b_done": torch.cuda.Event()}
        es["b_done"].record()
        self._esets[ekey] = es
        return es

    def _capture(self, key, inputs, crop, orig, global_batch, ekey):
        """Capture F / F2 / B for one batch shape (and E for its pixel shape if not captured yet). The graphs
        read their own static copies of the inputs (``inputs`` is cloned), so any later batch of the same shape
        is replayed after a copy-in."""
        dev = inputs[0].device
        # device copies (prompts may come as host tensors from the data path; the graphs read device memory)
        pixel_values, gt_u8, input_boxes, input_points, input_labels = (
            None if t is None else t.detach().to(dev, copy=True) for t in inputs)
        # one eager pass first: lazily built operand caches, tables and kernel attributes exist before capture
        self._eager_forward_backward(pixel_values, gt_u8, input_boxes, input_points, input_labels, crop, orig,
                                     global_batch, True)
        torch.cuda.synchronize()
        es = self._encoder_set(ekey, pixel_values)
        st = self._state(es["pixel"], gt_u8, input_boxes, input_points, input_labels, crop, orig, global_batch)
        st.emb = es["emb"]
        B, N = gt_u8.shape[:2]
        if self.topological and self.lamda != 0.0 and self.w2 == "host":
            entries, maps, midx = topo_index(B, N, self.topo_mode, global_batch, dev)
            Kn = len(maps)
            if Kn:
                mp = K.ph_max_pairs(self.interp, self.interp)
                st.pinned = (torch.empty((2 * Kn, mp, 2), dtype=torch.int32, pin_memory=True),
                             torch.empty((2 * Kn, 3), dtype=torch.int32, pin_memory=True),
                             torch.empty((2 * Kn, self.interp * self.interp), dtype=torch.float32, pin_memory=True))
                st.dp_pinned = torch.zeros((Kn, self.interp * self.interp), dtype=torch.float32, pin_memory=True)
                st.dp = torch.zeros((Kn, self.interp * self.interp), dtype=torch.float32, device=dev)
        if st.pinned is None:  # no host phase: the pinned topo scalar stays 0
            st.pinned = ()
        st.topo_pinned = torch.zeros(1, dtype=torch.float64, pin_memory=True)
        gf, gf2, gb = (torch.cuda.CUDAGraph() for _ in range(3))
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(gf, stream=s, capture_error_mode="relaxed"):
                self._phase_f(st, True)
            pool = gf.pool()
            with torch.cuda.graph(gf2, stream=s, pool=pool, capture_error_mode="relaxed"):
                self._phase_f2(st)
            with torch.cuda.graph(gb, stream=s, pool=pool, capture_error_mode="relaxed"):
                self._phase_b(st, True)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        if st.pinned == ():
            st.pinned = None
            st.topo_dev = None
        static = (None, gt_u8, input_boxes, input_points, input_labels)  # pixels: the encoder set's input
        g = {"graphs": (gf, gf2, gb), "eset": es, "st": st, "ev": torch.cuda.Event(), "static": static}
        self._graphs[key] = g
        self.captures += 1
        while len(self._graphs) > self.MAX_GRAPHS:
            self._graphs.pop(next(iter(self._graphs)))
            self.evictions += 1
        return g

    @staticmethod
    def _src_tag(t):
        """Identity of an input as last copied: the tensor itself (held, so its storage cannot be handed to a
        later batch while the tag lives — a (data_ptr, version) tag matched a new batch that the caching
        allocator placed at a freed batch's address) and its version counter (in-place writes)."""
        return None if t is None else (t, t._version)

    @staticmethod
    def _same(a, b):
        if a is None or b is None:
            return a is None and b is None
        return a[0] is b[0] and a[1] == b[1]

    def _copy_in(self, g, inputs):
        """Copy the batch into the captured graphs' static inputs — every step: an unchanged tensor object is no
        proof of unchanged contents (the library's kernels write through raw pointers without bumping torch's
        version counter), and the copies cost ~10 us of HBM time per step."""
        for dst, src in zip(g["static"], inputs):
            if dst is not None and src is not None:
                dst.copy_(src, non_blocking=True)

    @staticmethod
    def _pixel_in(es, px):
        es["pixel"].copy_(px, non_blocking=True)
        es["src"] = FusedTrainStep._src_tag(px)

    def _graph_forward_backward(self, pixel_values, gt_u8, input_boxes, input_points, input_labels, crop, orig,
                                global_batch, between=None, next_inputs=None):
        inputs = (pixel_values, gt_u8, input_boxes, input_points, input_labels)
        key = self._graph_key(*inputs) + (tuple(crop), tuple(orig), global_batch)
        ekey0 = (tuple(pixel_values.shape), pixel_values.dtype)
        par = self._parity.get(ekey0, 0) if self.pipeline else 0
        ekey = ekey0 + (par,)
        g = self._graphs.pop(key + (par,), None)
        if g is None:
            g = self._capture(key + (par,), inputs, crop, orig, global_batch, ekey)
        else:
            self._graphs[key + (par,)] = g  # most recently used last
        es = g["eset"]
        gf, gf2, gb = g["graphs"]
        st, ev = g["st"], g["ev"]
        main = torch.cuda.current_stream()
        pre = self._prefetch
        self._prefetch = None
        if pre is not None and pre[0] is es and self._same(pre[1], self._src_tag(pixel_values)):
            main.wait_event(es["e_done"])  # this batch's E ran ahead on the encoder stream
        else:
            if pre is not None:
                main.wait_event(pre[0]["e_done"])  # a lookahead for other pixels: let it finish, then redo E
            self._pixel_in(es, pixel_values)
            es["graph"].replay()
        self._copy_in(g, inputs)
        if self.pipeline and next_inputs is not None:
            # queued before the deferred update and F: the next E may also overlap a pending all-reduce
            self._launch_lookahead(ekey0, par, next_inputs[0])
        self._finish_pending()
        gf.replay()
        if st.pinned is not None:
            ev.record()
        gf2.replay()  # DiceCE backward runs on the GPU while the host computes W2 below
        if between is not None:
            between()  # host work overlapped with the step (e.g. building the next batch on a side stream)
        if st.pinned is not None:
            ev.synchronize()  # the persistence pairs are in the pinned buffers
        loss = self._topo_host(st, True) if st.pinned is not None else 0.0
        if st.pinned is not None:
            st.topo_pinned.numpy()[0] = loss
        gb.replay()
        if self.pipeline:
            es["b_done"].record(main)
            self._parity[ekey0] = (par + 1) % self.pipeline_sets
        return st.loss_out

    def _launch_lookahead(self, ekey0, par, next_px):
        """Replay E of the next batch's pixels on the encoder stream (encoder set of the other parity) once that
        set's previous step (its B, which reads the embedding) has finished; the pixel copy-in runs on the same
        stream. Any prompt count: only the pixel shape has to match."""
        if (tuple(next_px.shape), next_px.dtype) != ekey0:
            return  # another pixel shape: its first step runs E itself
        es = self._esets.get(ekey0 + ((par + 1) % self.pipeline_sets,))
        if es is None:
            return  # the other set is captured when a step first needs it
        main = torch.cuda.current_stream()
        if self._enc_stream is None:
            self._enc_stream = torch.cuda.Stream(device=main.device, priority=self.enc_priority)
        enc = self._enc_stream
        enc.wait_event(es["b_done"])
        ready = torch.cuda.Event()
        ready.record(main)  # the next pixels were produced on (or handed to) the main stream
        enc.wait_event(ready)
        with torch.cuda.stream(enc):
            self._pixel_in(es, next_px)
            es["graph"].replay()
            es["e_done"].record(enc)
        if next_px.is_cuda:
            next_px.record_stream(enc)
        self._prefetch = (es, self._src_tag(next_px))

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

    @torch.no_grad()
    def optimizer_state(self) -> dict:
        """Adam state with HF names: "exp_avg.mask_decoder.<param>" / "exp_avg_sq.mask_decoder.<param>" (fp32, CPU,
        the parameters' HF shapes) and "step" (torch.optim.Adam's per-parameter step count; one shared count here)."""
        self.flush()
        dec = self.model.mask_decoder
        out = {"step": torch.tensor(float(self.t))}
        for name in dec._order:
            for key, buf in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                out[f"{key}.mask_decoder.{name}"] = dec._param_view(buf, name).detach().float().cpu().contiguous()
        return out

    @torch.no_grad()
    def load_optimizer_state(self, state: dict):
        """Resume Adam from optimizer_state()'s layout (e.g. a torch.optim.Adam run converted by name), so a
        continued run takes the same update as the optimizer it replaces instead of a cold first step."""
        self.flush()
        dec = self.model.mask_decoder
        for name in dec._order:
            for key, buf in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                src = state[f"{key}.mask_decoder.{name}"]
                view = dec._param_view(buf, name)
                if tuple(src.shape) != tuple(view.shape):
                    raise ValueError(f"{key} of {name}: shape {tuple(src.shape)} != {tuple(view.shape)}")
                view.copy_(src.to(device=buf.device, dtype=torch.float32))
        self.t = int(float(state["step"]))

    def _launch_update(self, n_local, n_global):
        """All-reduce (side stream when overlapping) then Adam, now or at the next _finish_pending."""
        if self.pg is None or not self.overlap:
            self.allreduce_grads(n_local, n_global)
            self.optimizer_step()
            return
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(device=main.device)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            self.allreduce_grads(n_local, n_global)
            done = torch.cuda.Event()
            done.record(self._side)
        self._pending = done

    def _finish_pending(self):
        if self._pending is None:
            return
        torch.cuda.current_stream().wait_event(self._pending)
        self._pending = None
        self.optimizer_step()

    def flush(self):
        """Apply a deferred (overlapped) parameter update."""
        self._finish_pending()

    def step(self, batch: dict, n_global=None, between=None, next_batch: dict | None = None):
        """batch: device tensors from data.process_batch/to_device_batch. n_global: images in the global
        batch (data parallel; None = this rank's batch is the whole batch). between: host work to overlap
        with the step (see forward_backward). next_batch (pipeline=True): the batch the next step() gets; its
        encoder phase runs during this step's decoder."""
        crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
        orig = tuple(int(v) for v in batch["original_sizes"][0])
        n_local = int(batch["pixel_values"].shape[0])
        nxt = None
        if next_batch is not None:
            nxt = (next_batch["pixel_values"], next_batch["gt_u8"], next_batch.get("input_boxes"),
                   next_batch.get("input_points"), next_batch.get("input_labels"))
        loss = self.forward_backward(batch["pixel_values"], batch["gt_u8"], input_boxes=batch.get("input_boxes"),
                                     input_points=batch.get("input_points"), input_labels=batch.get("input_labels"),
                                     crop=crop, orig=orig, global_batch=n_global, between=between, next_inputs=nxt)
        self._launch_update(n_local, n_global)
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
    background-valued prompt follows the first one (training_utils.py:126-134). int64 [C, 3]. The counts
    of every prompt come from the HIP kernel octsam_confusion (metrics.prompt_confusion)."""
    from .metrics import included_prompts, prompt_confusion
    B, N = masks.shape[:2]
    per = prompt_confusion(masks, gt_u8).view(B, N, 4).cpu()
    mv = mask_values.cpu()
    conf = torch.zeros(num_classes, 3, dtype=torch.int64)
    for b, c in included_prompts(mv):
        conf[int(mv[b, c])] += per[b, c, :3]
    return conf


def mean_dice(conf: torch.Tensor) -> float:
    """'Mean dice' of training_utils.py:156,246: mean over classes of 2tp/(2tp+fp+fn) (0 if empty)."""
    d = []
    for tp, fp, fn in conf[:, :3].tolist():
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
    from .preprocess import DeviceProcessor
    if isinstance(processor, DeviceProcessor):
        b = data.process_batch_device(processor, data.custom_collate(items), prompt)
    else:
        b = data.process_batch(processor, data.custom_collate(items), prompt)
    b = data.pad_prompts(b, n_target)
    return data.to_device_batch(b, device)


def _prep(ds, idx, prompt, device, device_data):
    """Phase 1 of a batch: the reference's host items (SAMDataset, scipy components), or — with the HIP data
    path — device components (components.collate_device_begin, with SAMDataset's per-item seeding replayed).
    Returns (kind, state, local N)."""
    from . import data
    if device_data and idx:
        from .components import ComponentLimitError, collate_device_begin
        its = [ds.dataset[i] for i in idx]
        imgs = np.stack([np.array(it["image"]) for it in its])
        if ds.config.get("pseudocolor") is not None:  # as SAMDataset.__getitem__ (a host gather per pixel)
            from .colormaps import apply_colormap, colormap_lut
            lut = colormap_lut(ds.config["pseudocolor"])
            imgs = np.stack([apply_colormap(im, lut) for im in imgs])
        if imgs.ndim == 3:  # grayscale scans: the processor's convert_rgb replicates the channel
            imgs = np.repeat(imgs[..., None], 3, -1)
        labs = np.stack([np.array(it["label"]) for it in its]).astype(np.uint8)
        hooks = None
        if ds.epoch_seed is not None:
            hooks = [(lambda i=i: data.seed_sample(ds.epoch, i, ds.epoch_seed)) for i in idx]
        try:
            st = collate_device_begin(imgs, labs, prompt, device, hooks)
            return "dev", st, max(st["cc"]["ncomp"])
        except ComponentLimitError:
            pass  # beyond the device path's limits: the reference's host path below (same draws, same batch)
    items = [ds[i] for i in idx]
    return "host", items, _n_prompts(items)


def _finish(prep, processor, prompt, n_target, device):
    """Phase 2: the device batch of _prep, padded to the global N."""
    kind, state, _ = prep
    if kind == "dev":
        from .components import collate_device_end
        from .preprocess import DeviceProcessor
        b = collate_device_end(state, n_target, processor if isinstance(processor, DeviceProcessor) else None)
        b.pop("prompt_raw")
        return b
    return _batch_for(state, processor, prompt, n_target, device)


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
    if device is None:
        if not torch.cuda.is_available():
            # the reference falls back to the CPU (training_utils.py:33); this loop's arithmetic is the HIP library
            # (no CPU fallback by design: a silent CPU path would not be the measured product), so say so up front
            raise RuntimeError("training() needs an MI355X (liboctsam_hip.so runs every op of the step as a HIP kernel); "
                               "no GPU is visible. The reference's CPU step is restated as test infrastructure in "
                               "oracle/step_ref.py (bench.py's cpu_baseline), not as a product path.")
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError(f"training() runs on a GPU device (liboctsam_hip.so), got {device}")
    model = SamModel.from_pretrained(base_model, **({"seed": config["seed"]} if "seed" in config else {})).to(device)
    if config.get("encoder_dtype", "bf16") == "fp16":  # BASELINE configs[4]
        model.set_encoder_dtype(torch.float16)
    if device.type == "cuda" and config.get("gpu_processor", True):  # image path as a HIP kernel (§8(f)1)
        from .preprocess import DeviceProcessor
        processor = DeviceProcessor(device)
    else:
        processor = data.make_processor()
    # components / prompts / gt on the GPU too (§8(f)1), with the HIP image processor
    device_data = device.type == "cuda" and config.get("gpu_processor", True) and config.get("gpu_components", True)
    train_data = train_data if train_data is not None else _load_split(config, "train")
    valid_data = valid_data if valid_data is not None else _load_split(config, "test")
    prompt = config.get("prompt_type", "bboxes")
    tds = data.SAMDataset(train_data, config, epoch_seed=config.get("data_seed"))
    vds = data.SAMDataset(valid_data, config, epoch_seed=config.get("data_seed"))
    bs = int(config.get("batch_size", 2))
    # config "graphs" / "pipeline" (default on for a GPU; the CLI's --graphs / --pipeline): hipGraph replay per
    # batch shape, and the encoder lookahead (the next batch is built before this step so its encoder runs during
    # this step's decoder) — the path bench.py times
    graphs = _bool_flag(config.get("graphs", True)) and device.type == "cuda"
    step = FusedTrainStep(model, lr=config.get("learning_rate", 1e-3), weight_decay=config.get("weight_decay", 0.0),
                          topological=bool(config.get("topological", False)),
                          topo_mode=config.get("topo_mode", "first"), process_group=pg, graphs=graphs,
                          pipeline=graphs and _bool_flag(config.get("pipeline", True)))
    hist = {"train_loss": [], "valid_loss": [], "train_time_s": []}
    # the data path (host RNG draws, device components / processor, their host syncs) runs on a side stream, so
    # building the next batches overlaps the queued steps on the main stream
    main = torch.cuda.current_stream(device) if device.type == "cuda" else None
    side = torch.cuda.Stream(device=device) if device.type == "cuda" else None

    def build(bi, idx):
        n_glob = len(tds) - bi * bs * world if bi == len(batches) - 1 else bs * world
        n_glob = min(n_glob, bs * world)
        if side is None:
            prep = _prep(tds, idx, prompt, device, device_data)
            N = _collective_max(prep[2], pg)
            return n_glob, (_finish(prep, processor, prompt, N, device) if idx else None), None
        with torch.cuda.stream(side):  # allocations come from the side stream's pool (no wait on queued steps)
            prep = _prep(tds, idx, prompt, device, device_data)
            N = _collective_max(prep[2], pg)
            b = _finish(prep, processor, prompt, N, device) if idx else None
            ev = torch.cuda.Event()
            ev.record(side)
        for v in (b or {}).values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(main)
        return n_glob, b, ev

    def inputs_of(b):
        return (b["pixel_values"], b["gt_u8"], b.get("input_boxes"), b.get("input_points"), b.get("input_labels"))

    for epoch in range(int(config.get("epochs", 10))):
        tds.epoch = epoch
        batches = global_batches(len(tds), bs, world, rank, bool(config.get("shuffle", False)),
                                 config.get("data_seed") or 0, epoch)
        t_epoch = time.perf_counter()
        # sum over steps of loss * images / global images on the device: no per-step host sync (the reference's
        # .item() of :69 only feeds this sum); one read per epoch
        loss_acc = torch.zeros(1, dtype=torch.float64, device=device)
        # batches are built two ahead, in loader order (same RNG draws as building each at its own step): batch
        # bi + 1 must exist when step bi is queued (its encoder runs during step bi's decoder), and batch bi + 2 is
        # built on the host while the GPU runs step bi (forward_backward's `between`)
        ready = {j: build(j, batches[j]) for j in (1, 2) if j < len(batches)}
        for bi, idx in enumerate(batches):
            if bi == 0:  # training_utils.py:40-44: the first batch of every epoch is skipped
                continue
            n_glob, batch, ev = ready.pop(bi)
            nxt = ready.get(bi + 1)

            def ahead(j=bi + 2):
                if j < len(batches):
                    ready[j] = build(j, batches[j])
            if idx:
                if ev is not None:
                    main.wait_event(ev)
                crop = tuple(int(v) for v in batch["reshaped_input_sizes"][0])
                orig = tuple(int(v) for v in batch["original_sizes"][0])
                nb = nxt[1] if (nxt is not None and step.pipeline) else None
                if nb is not None and nxt[2] is not None:
                    main.wait_event(nxt[2])
                loss = step.forward_backward(*inputs_of(batch)[:2], input_boxes=batch.get("input_boxes"),
                                             input_points=batch.get("input_points"), crop=crop, orig=orig,
                                             global_batch=n_glob, next_inputs=None if nb is None else inputs_of(nb),
                                             between=ahead)
                loss_acc += loss[3:4].double() * len(idx) / n_glob
            else:  # nothing on this rank in a ragged last batch: contribute zero gradient
                model.mask_decoder.flat_grad.zero_()
                ahead()
            step._launch_update(len(idx), n_glob)  # all-reduce (overlapped with the next encoder forward) + Adam
        step.flush()
        epoch_loss = float(_collective_sum(loss_acc, pg)[0]) / len(batches)
        hist["train_time_s"].append(time.perf_counter() - t_epoch)
        hist.setdefault("graph_captures", []).append(step.captures)  # cumulative; > 2 per shape = recaptures
        vloss = validate_model(step, vds, processor, bs, config, world, rank, pg, device, device_data)
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
        conf, metrics = evaluate_model(model, vds, processor, bs, prompt, world, rank, pg, device, device_data)
        hist["dice"] = class_dice(conf)
        hist["mean_dice"] = mean_dice(conf)
        hist["metrics"] = metrics
        if rank == 0:
            m = metrics["mean"]
            log(f"Mean_accuracy:{m['accuracy']}\nMean_iou:{m['iou']}\nMean specificity: {m['specificity']}\n"
                f"Mean sensitivity: {m['sensitivity']}\nMean dice: {hist['mean_dice']}\nMean mAP: {m['ap']}")
    return hist


@torch.no_grad()
def validate_model(step: FusedTrainStep, vds, processor, bs, config, world=1, rank=0, pg=None, device=None,
                   device_data=False):
    """ref:training_utils.py:351-379, including its double accumulation: every batch adds the DiceCE loss
    and then DiceCE (+ topo) again, divided by len(valid_dl)."""
    prompt = config.get("prompt_type", "bboxes")
    batches = global_batches(len(vds), bs, world, rank)
    total = 0.0
    for bi, idx in enumerate(batches):
        n_glob = min(bs * world, len(vds) - bi * bs * world)
        prep = _prep(vds, idx, prompt, device, device_data)
        N = _collective_max(prep[2], pg)
        lv = torch.zeros((), dtype=torch.float64)
        if idx:
            batch = _finish(prep, processor, prompt, N, device)
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
def evaluate_model(model, vds, processor, bs, prompt, world=1, rank=0, pg=None, device=None, device_data=False):
    """evaluate_metrics (training_utils.py:113-270) over the validation set on the GPU: per-prompt confusion
    counts (HIP), per-class pooled and per-sample IoU / accuracy / specificity / sensitivity / F1 / Dice / AP
    (metrics.EvalAccumulator). Data parallel: the per-sample counts of all ranks are gathered, so every
    confusion-based metric is the single-process one; the pooled AP needs every score and is computed only
    when world == 1 (NaN otherwise). Returns (pooled (tp, fp, fn) int64 [14, 3], metrics dict)."""
    from .metrics import EvalAccumulator
    acc = EvalAccumulator(keep_scores=(world == 1))
    for idx in global_batches(len(vds), bs, world, rank):
        if not idx:
            continue
        prep = _prep(vds, idx, prompt, device, device_data)
        batch = _finish(prep, processor, prompt, prep[2], device)
        acc.add(predict_masks(model, batch), batch["gt_u8"], batch["mask_values"], image_index=idx)
    if pg is not None:
        import torch.distributed as dist
        got = [None] * world
        dist.all_gather_object(got, (acc.counts, acc.samples), group=pg)
        acc.counts = [sum((g[0][v] for g in got), []) for v in range(acc.C)]
        acc.samples = [sum((g[1][v] for g in got), []) for v in range(acc.C)]
    return acc.pooled_confusion()[:, :3], acc.compute()


@torch.no_grad()
def evaluate_confusion(model, vds, processor, bs, prompt, world=1, rank=0, pg=None, device=None,
                       device_data=False):
    """Pooled per-class (tp, fp, fn) over the validation set (training_utils.py:113-156), all ranks."""
    return evaluate_model(model, vds, processor, bs, prompt, world, rank, pg, device, device_data)[0]


def class_dice(conf: torch.Tensor) -> list:
    out = []
    for tp, fp, fn in conf.tolist():
        den = 2 * tp + fp + fn
        out.append(2 * tp / den if den else 0.0)
    return out


def _bool_flag(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("true", "1", "yes", "y", "on"):
        return True
    if s in ("false", "0", "no", "n", "off"):
        return False
    import argparse
    raise argparse.ArgumentTypeError(f"expected True or False, got {v!r}")


def build_parser():
    """argparse of ref:octsam/models/training.py:20-93 (same flags and defaults)."""
    import argparse
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
    p.add_argument("--top", nargs="?", const=True, default=False, type=_bool_flag,
                   help="topological loss: --top, --top=True or --top=False (README usage; the reference's "
                        "store_true flag rejects --top=True)")
    p.add_argument("--synthetic", type=int, default=0, help="train on K synthetic images (no dataset on disk)")
    p.add_argument("--precision", type=str, default="bf16", choices=["bf16", "fp16"],
                   help="16-bit operand type of the frozen image encoder (build extension; fp16 = configs[4])")
    p.add_argument("--graphs", nargs="?", const=True, default=True, type=_bool_flag,
                   help="replay each batch shape's step as hipGraphs (default on; --graphs=False: eager launches)")
    p.add_argument("--pipeline", nargs="?", const=True, default=True, type=_bool_flag,
                   help="encoder lookahead: the next batch's frozen encoder runs during this step's decoder "
                        "(default on; needs --graphs)")
    return p


def main(argv=None):
    """CLI mirror of ref:octsam/models/training.py (same flags and defaults; W&B, display and pseudocolour
    options are accepted and ignored). --synthetic K trains on K synthetic OCT-like images instead of a
    save_to_disk dataset."""
    import datetime
    args = build_parser().parse_args(argv)
    if args.loss != "diceCE" or args.optimizer != "adam":
        raise SystemExit("only --loss diceCE and --optimizer adam exist in the reference")
    from .colormaps import colormap_lut
    try:  # the reference's OCV_COLORMAPS[args.pseudocolor] (ref:octsam/models/training.py:123)
        pseudocolor = colormap_lut(args.pseudocolor)
    except (KeyError, NotImplementedError) as e:
        raise SystemExit(f"--pseudocolor: {e}")
    now = datetime.datetime.now().strftime("%y-%m-%d_%H.%M.%S")
    name = args.display_name or (f"{'{:.0e}'.format(args.lr)} lr,{'{:.0e}'.format(args.weight_decay)} wd,"
                                 f"{args.bs} bs, {args.loss} loss, {args.pseudocolor}, {now}")
    config = {"display_name": name, "base_model": args.base_model,
              "dataset": os.path.join(args.data_directory, "datasets", "processed", args.dataset, args.dataset_name),
              "checkpoint": os.path.join(args.data_directory, "models", args.dataset),
              "learning_rate": args.lr, "weight_decay": args.weight_decay, "epochs": args.epochs,
              "batch_size": args.bs, "shuffle": args.shuffle, "optimizer": args.optimizer, "loss": args.loss,
              "time": now, "evaluate": args.evaluate, "topological": args.top, "prompt_type": args.prompt,
              "pseudocolor": pseudocolor, "encoder_dtype": args.precision, "graphs": args.graphs, "pipeline": args.pipeline}
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
