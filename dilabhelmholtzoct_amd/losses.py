"""Post-processing, DiceCE and topological loss of the OCT-SAM step on liboctsam_hip.so.

Drop-in callables for the reference's loss surface:
  * ``postprocess_masks(pred_masks, reshaped_input_sizes, original_sizes)`` — the two F.interpolate
    calls + crop of ref:octsam/models/training_utils.py:57-59, fused (autograd-aware).
  * ``DiceCELoss(sigmoid=True)`` — monai 1.3.0 DiceCELoss as called at training_utils.py:32,62
    (monai is not installed; its published algorithm is restated in postproc_loss.hip).
  * ``topo_loss(pred_obj, true_obj, lamda, interp, feat_d, loss_q, loss_r)`` — ref:octsam/models/
    topological_loss.py:11-96 with torch_topological's CubicalComplex (HIP persistence kernel) and
    WassersteinDistance (host exact assignment, like POT's host ot.emd2).
The fused training step (train.py) calls the same kernels directly without autograd.
"""
from __future__ import annotations

import functools
import math

import numpy as np
import torch

from . import kernels as K
from . import _lib


# ------------------------------------------------------------------------ post-processing
def _lin_acf_np(dst: int, in_size: int, scale: np.float32):
    r = np.float32(scale) * (np.float32(dst) + np.float32(0.5)) - np.float32(0.5)
    if r < 0:
        r = np.float32(0.0)
    i0 = int(r)
    i1 = i0 + (1 if i0 < in_size - 1 else 0)
    l1 = np.float32(r - np.float32(i0))
    return i0, i1, np.float32(1.0) - l1, l1


def _composite_1d(S: int, mid: int, crop: int, out: int) -> np.ndarray:
    """[out, S] weights of interp(S->mid) -> crop -> interp(crop->out), torch index arithmetic."""
    W = np.zeros((out, S), np.float64)
    s1 = np.float32(S) / np.float32(mid)
    s2 = np.float32(crop) / np.float32(out)
    for i in range(out):
        r0, r1, l0, l1 = _lin_acf_np(i, crop, s2)
        for r, lr in ((r0, l0), (r1, l1)):
            a0, a1, m0, m1 = _lin_acf_np(r, S, s1)
            W[i, a0] += float(lr) * float(m0)
            W[i, a1] += float(lr) * float(m1)
    return W.astype(np.float32)


@functools.lru_cache(maxsize=16)
def _pp_tables_host(S, mid, ch, cw, oh, ow):
    Wy = _composite_1d(S, mid, ch, oh)   # [oh, S]
    Wx = _composite_1d(S, mid, cw, ow)   # [ow, S]

    def csr_by_source(Wm):
        ptr, idx, w = [0], [], []
        for a in range(S):
            nz = np.nonzero(Wm[:, a])[0]
            idx.extend(nz.tolist())
            w.extend(Wm[nz, a].tolist())
            ptr.append(len(idx))
        return (np.asarray(ptr, np.int32), np.asarray(idx, np.int32), np.asarray(w, np.float32))

    return csr_by_source(Wx), csr_by_source(Wy)


_DEV_TABLES: dict = {}


def pp_tables(S, mid, ch, cw, oh, ow, device):
    key = (S, mid, ch, cw, oh, ow, str(device))
    if key not in _DEV_TABLES:
        cols, rows = _pp_tables_host(S, mid, ch, cw, oh, ow)
        _DEV_TABLES[key] = tuple(torch.from_numpy(a).to(device) for a in cols + rows)
    return _DEV_TABLES[key]


def postproc_forward(low: torch.Tensor, crop, orig, gt_u8=None):
    """low fp32 [M, 256, 256] -> masks fp32 [M, oh, ow]; with gt also the Dice partials (one per 4 output rows)."""
    M, S, _ = low.shape
    (ch, cw), (oh, ow) = crop, orig
    nblk = (oh + 3) // 4
    out = torch.empty(M, oh, ow, device=low.device, dtype=torch.float32)
    part = torch.empty(M, nblk, 3, device=low.device, dtype=torch.float32) if gt_u8 is not None else None
    _lib.call("octsam_postproc_fwd", K.ptr(low), M, S, 1024, ch, cw, oh, ow, K.ptr(out), K.ptr(gt_u8), K.ptr(part),
              nblk)
    return out, part


def postproc_backward(dout: torch.Tensor, S: int, crop, orig) -> torch.Tensor:
    M, oh, ow = dout.shape
    (ch, cw) = crop
    cptr, cidx, cw_, rptr, ridx, rw = pp_tables(S, 1024, ch, cw, oh, ow, dout.device)
    tmp = torch.empty(M, oh, S, device=dout.device, dtype=torch.float32)
    dlow = torch.empty(M, S, S, device=dout.device, dtype=torch.float32)
    _lib.call("octsam_postproc_bwd", K.ptr(dout), M, S, oh, ow, K.ptr(cptr), K.ptr(cidx), K.ptr(cw_), K.ptr(rptr),
              K.ptr(ridx), K.ptr(rw), K.ptr(tmp), K.ptr(dlow))
    return dlow


class _PostProcFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, low, crop, orig):
        B, N = low.shape[:2]
        out, _ = postproc_forward(low.reshape(B * N, low.shape[-2], low.shape[-1]).float().contiguous(), crop, orig)
        ctx.meta = (B, N, low.shape[-1], crop, orig)
        return out.view(B, N, orig[0], orig[1])

    @staticmethod
    def backward(ctx, dout):
        B, N, S, crop, orig = ctx.meta
        dlow = postproc_backward(dout.reshape(B * N, orig[0], orig[1]).float().contiguous(), S, crop, orig)
        return dlow.view(B, N, S, S), None, None


def postprocess_masks(pred_masks: torch.Tensor, reshaped_input_sizes, original_sizes) -> torch.Tensor:
    """training_utils.py:57-59: pred_masks [B,N,1,256,256] -> [B,N,oh,ow] (sizes of sample 0, as the
    reference indexes [0])."""
    low = pred_masks.squeeze(2)
    crop = (int(reshaped_input_sizes[0][0]), int(reshaped_input_sizes[0][1]))
    orig = (int(original_sizes[0][0]), int(original_sizes[0][1]))
    return _PostProcFn.apply(low, crop, orig)


# ------------------------------------------------------------------------ DiceCE
def dicece_forward_backward(masks: torch.Tensor, gt_u8: torch.Tensor, dice_part: torch.Tensor | None = None,
                            w_dice: float = 1.0, w_ce: float = 1.0, nblk: int = 1024):
    """masks fp32 [B,N,H,W], gt uint8 [B,N,H,W] -> (loss double [3] = dice, ce, total; dmask fp32).
    dice_part (from postproc_forward) avoids a second pass over masks."""
    B, N, H, W = masks.shape
    M = B * N
    dev = masks.device
    if dice_part is None:
        raise ValueError("dice partial sums required (octsam_postproc_fwd with gt)")
    nb_d = dice_part.shape[1]
    dice_map = torch.empty(M, device=dev, dtype=torch.float64)
    coef = torch.empty(M, 2, device=dev, dtype=torch.float32)
    _lib.call("octsam_dice_reduce", K.ptr(dice_part), M, nb_d, K.ptr(dice_map), K.ptr(coef))
    dmask = torch.empty_like(masks)
    ce_part = torch.empty(nblk, device=dev, dtype=torch.float64)
    _lib.call("octsam_dicece_bwd", K.ptr(masks), K.ptr(gt_u8), K.ptr(coef), B, N, H * W, w_dice, w_ce, K.ptr(dmask),
              K.ptr(ce_part), nblk)
    loss = torch.empty(3, device=dev, dtype=torch.float64)
    _lib.call("octsam_loss_finalize", K.ptr(dice_map), M, K.ptr(ce_part), nblk, B, H * W, w_dice, w_ce, K.ptr(loss))
    return loss, dmask


_KEEP: dict = {}


def _keep_table(B: int, N: int, maps, device):
    """keep [B*N] int32: position k of map m in the topological loss's map list, else -1 (cached: fixed address for
    captured graphs)."""
    key = (B, N, tuple(maps), str(device))
    if key not in _KEEP:
        keep = torch.full((B * N,), -1, dtype=torch.int32)
        for k, m in enumerate(maps):
            keep[m] = k
        _KEEP[key] = keep.to(device)
    return _KEEP[key]


def dicece_pp_rows_supported(B: int, N: int, H: int, W: int) -> bool:
    """Whether octsam_dicece_pp_rows (and octsam_pp_bwd_rows_maps) take a [B, N, H, W] batch: at most 32 prompts whose
    rows fit 160 KB of LDS, W % 4 == 0, W <= 1024. The reference puts no cap on the prompt count (one prompt per
    8-connected component of every label value, training_utils.py:389-415), so callers fall back to
    dicece_forward_backward + postproc_backward when this is False."""
    return (0 < N <= 32 and N * W * 4 <= 160 * 1024 and W % 4 == 0 and 0 < W <= 1024 and B * H * W < (1 << 31)
            and B <= 65535)


def dicece_pp_rows(masks: torch.Tensor, gt_u8: torch.Tensor, dice_part: torch.Tensor, crop, *, maps=(),
                   w_dice: float = 1.0, w_ce: float = 1.0, S: int = 256):
    """The DiceCE loss and its backward fused with the post-processing adjoint's row pass (octsam_dicece_pp_rows):
    no [B, N, H, W] d-mask in HBM. Returns (loss double [3] = dice, ce, total; tmp fp32 [B*N, H, S] (the row pass of
    every map not in `maps`); dkeep fp32 [len(maps), H, W] (the d-mask of the topological loss's maps, whose topo
    gradient joins in pp_rows_finish) or None). dice_part from postproc_forward with gt (training_utils.py:56-62)."""
    B, N, H, W = masks.shape
    M = B * N
    dev = masks.device
    dice_map = torch.empty(M, device=dev, dtype=torch.float64)
    coef = torch.empty(M, 2, device=dev, dtype=torch.float32)
    _lib.call("octsam_dice_reduce", K.ptr(dice_part), M, dice_part.shape[1], K.ptr(dice_map), K.ptr(coef))
    cptr, cidx, cw_, _, _, _ = pp_tables(S, 1024, crop[0], crop[1], H, W, dev)
    tmp = torch.empty(M, H, S, device=dev, dtype=torch.float32)
    keep = _keep_table(B, N, maps, dev) if maps else None
    dkeep = torch.empty(len(maps), H, W, device=dev, dtype=torch.float32) if maps else None
    ce_part = torch.empty(B * H, device=dev, dtype=torch.float64)
    _lib.call("octsam_dicece_pp_rows", K.ptr(masks), K.ptr(gt_u8), K.ptr(coef), B, N, H, W, w_dice, w_ce, S,
              K.ptr(cptr), K.ptr(cidx), K.ptr(cw_), K.ptr(keep), K.ptr(dkeep), K.ptr(tmp), K.ptr(ce_part))
    loss = torch.empty(3, device=dev, dtype=torch.float64)
    _lib.call("octsam_loss_finalize", K.ptr(dice_map), M, K.ptr(ce_part), B * H, B, H * W, w_dice, w_ce, K.ptr(loss))
    return loss, tmp, dkeep


def pp_rows_finish(tmp: torch.Tensor, crop, orig, *, dkeep: torch.Tensor | None = None,
                   midx: torch.Tensor | None = None, S: int = 256) -> torch.Tensor:
    """Second half of the fused post-processing adjoint: the row pass of the kept maps (dkeep -> tmp[midx]) and the
    column pass of every map -> d low-res masks fp32 [B*N, S, S]."""
    M, H, _ = tmp.shape
    W = orig[1]
    dev = tmp.device
    cptr, cidx, cw_, rptr, ridx, rw = pp_tables(S, 1024, crop[0], crop[1], H, W, dev)
    if dkeep is not None and dkeep.shape[0]:
        _lib.call("octsam_pp_bwd_rows_maps", K.ptr(dkeep), K.ptr(midx), dkeep.shape[0], S, H, W, K.ptr(cptr),
                  K.ptr(cidx), K.ptr(cw_), K.ptr(tmp))
    dlow = torch.empty(M, S, S, device=dev, dtype=torch.float32)
    _lib.call("octsam_pp_bwd_cols", K.ptr(tmp), M, S, H, K.ptr(rptr), K.ptr(ridx), K.ptr(rw), K.ptr(dlow))
    return dlow


def _dice_partials(masks, gt_u8, nblk=64):
    """Dice partial sums of an already post-processed fp32 mask tensor (drop-in path): octsam_dice_partials."""
    B, N, H, W = masks.shape
    part = torch.empty(B * N, nblk, 3, device=masks.device, dtype=torch.float32)
    _lib.call("octsam_dice_partials", K.ptr(masks), K.ptr(gt_u8), B * N, H * W, K.ptr(part), nblk)
    return part


class _DiceCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, masks, gt_u8, w_dice, w_ce):
        x = masks.float().contiguous()
        part = _dice_partials(x, gt_u8)
        loss, dmask = dicece_forward_backward(x, gt_u8, part, w_dice, w_ce)
        ctx.save_for_backward(dmask)
        return loss[2]

    @staticmethod
    def backward(ctx, g):
        (dmask,) = ctx.saved_tensors
        return dmask * g.to(dmask.dtype), None, None, None


def _binary_u8(target: torch.Tensor, who: str) -> torch.Tensor:
    """0/1 targets as uint8 (the kernels' gt format); any other value raises (one device reduction + sync).
    The reference's gt is the 0/1 component indicator (training_utils.py:389-434)."""
    if target.dtype == torch.bool:
        return target.to(torch.uint8).contiguous()
    if bool(((target != 0) & (target != 1)).any()):
        raise ValueError(f"{who}: targets must be binary (0/1); soft targets are not supported by the HIP kernels")
    return target.to(torch.uint8).contiguous()


class DiceCELoss:
    """monai.losses.DiceCELoss(sigmoid=True) drop-in for binary (0/1) targets (anything else raises
    ValueError); float64 result like the reference (training_utils.py:62 promotes to the float64 gt dtype).
    N == 1: monai 1.3.0's CE is nn.CrossEntropyLoss over the single channel, i.e. 0 (the BCE branch for
    one channel arrived in a later monai release)."""

    def __init__(self, sigmoid: bool = True, lambda_dice: float = 1.0, lambda_ce: float = 1.0, **kw):
        if not sigmoid or kw.get("softmax") or kw.get("to_onehot_y") or kw.get("include_background") is False:
            raise NotImplementedError("only DiceCELoss(sigmoid=True) as used by the reference")
        self.lambda_dice, self.lambda_ce = lambda_dice, lambda_ce

    def __call__(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if input.shape != target.shape:
            raise ValueError(f"the number of dimensions for input and target should be the same, got "
                             f"shape {input.shape} and {target.shape}.")
        gt = _binary_u8(target, "DiceCELoss")
        return _DiceCEFn.apply(input, gt, self.lambda_dice, self.lambda_ce)


# ------------------------------------------------------------------------ topological loss
def topo_entries(B: int, N: int, mode: str = "first", global_batch: int | None = None):
    """Which (b, n) maps each loss entry of topo_loss covers, after `.squeeze()` + CubicalComplex
    nesting + torch_topological.batch_iter(dim=feat_d) (topological_loss.py:62-76):
      B == 1           -> one entry per prompt (nesting level 2)
      N == 1           -> one entry per image  (nesting level 2)
      B > 1 and N > 1  -> one entry per image (nesting level 3); mode "first": only prompt 0 of the
                          image (the upstream handler keeps the first channel),
                          mode "all": every prompt of the image (costs summed before the 1/q power).
    batch_iter's nesting semantics are unpinned (torch_topological absent).
    global_batch: the batch the single-process reference would see (data parallel: the sum over
    ranks); the nesting level follows it, so a rank holding one image of a larger global batch still
    uses the per-image rule."""
    GB = B if global_batch is None else global_batch
    if GB == 1:
        return [[n] for n in range(N)]
    if N == 1:
        return [[b] for b in range(B)]
    if mode == "all":
        return [[b * N + n for n in range(N)] for b in range(B)]
    return [[b * N] for b in range(B)]


_TOPO_INDEX: dict = {}


def topo_index(B: int, N: int, mode: str, global_batch: int | None, device):
    """(entries, maps, device int32 map index) of the topological loss for a [B, N] mask batch (cached: the
    index tensor's address stays fixed, so captured graphs may read it)."""
    key = (B, N, mode, global_batch, str(device))
    if key not in _TOPO_INDEX:
        entries = topo_entries(B, N, mode, global_batch)
        maps = sorted({m for e in entries for m in e})
        midx = torch.tensor(maps, dtype=torch.int32, device=device) if maps else None
        _TOPO_INDEX[key] = (entries, maps, midx)
    return _TOPO_INDEX[key]


def topo_device_forward(masks: torch.Tensor, gt_u8: torch.Tensor, midx: torch.Tensor, *, interp=50, feat_d=1,
                        max_pairs=None, logits=True):
    """Device half of the topological loss forward (no host sync; capturable): 50x50 align-corners
    resampling of sigmoid(pred) and gt (topological_loss.py:33-46; interp=0: the maps as they are, :48-52)
    and cubical persistence of both (:55-63). Returns (pairs [2Kn, max_pairs, 2] of dim feat_d, counts
    [2Kn, 3], maps [2Kn, side^2]); max_pairs defaults to kernels.ph_max_pairs(side, side), which no map can
    overflow. feat_d = 0 appends the essential class paired with the argmax pixel, as torch_topological's
    CubicalComplex does with gudhi's infinite pairs."""
    B, N, H, W = masks.shape
    oh, ow = (interp, interp) if interp else (H, W)
    Kn = midx.numel()
    dev = masks.device
    both = torch.empty(2 * Kn, oh, ow, device=dev, dtype=torch.float32)
    _lib.call("octsam_topo_down", K.ptr(masks), K.ptr(gt_u8), K.ptr(midx), Kn, H, W, oh, ow, int(logits),
              K.ptr(both[:Kn]), K.ptr(both[Kn:]))
    p0, p1, ess, cnt = K.cubical_ph(both, max_pairs=max_pairs)
    if feat_d == 0:
        # one more row for the essential pair: a map whose finite H0 pairs fill max_pairs (count saturated at
        # max_pairs) must not scatter past the buffer
        p0 = torch.cat([p0, torch.zeros((2 * Kn, 1, 2), dtype=p0.dtype, device=dev)], 1)
        rows = torch.arange(2 * Kn, device=dev)
        p0[rows, cnt[:, 0].long()] = ess
        cnt = cnt.clone()
        cnt[:, 0] += 1
    return (p0 if feat_d == 0 else p1), cnt, both.view(2 * Kn, oh * ow)


@functools.lru_cache(maxsize=64)
def _entry_csr(entries, maps):
    """Loss entries as CSR over map positions (int32 map indices, offsets) for octsam_topo_host."""
    pos = {m: i for i, m in enumerate(maps)}
    flat = np.array([pos[m] for e in entries for m in e], dtype=np.int32)
    off = np.zeros(len(entries) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(e) for e in entries])
    return flat, off


@functools.lru_cache(maxsize=64)
def _entry_tables(entries, maps):
    """_entry_csr plus map_entry [Kn]: the loss entry holding each map position (-1 = none)."""
    flat, off = _entry_csr(entries, maps)
    pos = {m: i for i, m in enumerate(maps)}
    map_entry = np.full(len(maps), -1, np.int32)
    for e, ms in enumerate(entries):
        for m in ms:
            map_entry[pos[m]] = e
    return flat, off, map_entry


_DEV_ENTRY: dict = {}


def _entry_tables_device(entries, maps, device):
    """Device copies of _entry_tables (cached: fixed addresses, so captured graphs may read them)."""
    key = (tuple(tuple(e) for e in entries), tuple(maps), str(device))
    if key not in _DEV_ENTRY:
        _DEV_ENTRY[key] = tuple(torch.from_numpy(a).to(device) for a in _entry_tables(key[0], key[1]))
    return _DEV_ENTRY[key]


def topo_w2_device(pairs: torch.Tensor, cnt: torch.Tensor, vals: torch.Tensor, entries, maps, *, lamda=0.1,
                   feat_d=1, loss_q=2, want_grad=True):
    """Device half of topo_loss's forward and backward (topological_loss.py:68-96): the exact
    W_q transport per map on the GPU (octsam_topo_w2, bit-identical to octsam_topo_host at q = 2), the loss and
    d loss / d pred-map values — no host sync, capturable. pairs / cnt / vals as topo_device_forward returns
    them. Returns (loss float64 [1] device, dpred fp32 [Kn, nvals] device or None); the loss is NaN if a pair
    count exceeded max_pairs (impossible at the default kernels.ph_max_pairs)."""
    Kn = len(maps)
    dev = pairs.device
    mp, nvals = int(pairs.shape[1]), int(vals.shape[1])
    flat, off, map_entry = _entry_tables_device(entries, maps, dev)
    lib = _lib.load()
    ws_bytes = int(lib.octsam_topo_w2_workspace(Kn, mp))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    loss = torch.empty(1, dtype=torch.float64, device=dev)
    dpred = torch.empty((Kn, nvals), dtype=torch.float32, device=dev) if want_grad else None
    _lib.call("octsam_topo_w2", K.ptr(pairs), K.ptr(cnt), K.ptr(vals), Kn, mp, nvals, K.ptr(flat), K.ptr(off),
              K.ptr(map_entry), len(entries), 0 if feat_d == 0 else 1, float(loss_q), float(lamda), int(want_grad),
              K.ptr(ws), ws_bytes, K.ptr(loss), K.ptr(dpred))
    return loss, dpred


def topo_host(pairs_h: np.ndarray, cnt_h: np.ndarray, vals_h: np.ndarray, entries, maps, *, lamda=0.1, feat_d=1,
              loss_q=2, want_grad=True):
    """Host half: W2 between the H_feat_d diagrams of pred and gt per loss entry (topological_loss.py:68-96,
    torch_topological WassersteinDistance(q) -> exact OT, restated in octsam_w2_host), all entries in one
    C call (octsam_topo_host). Returns the loss (float) and d loss / d pred-map values [Kn, interp^2]
    (float32; None without want_grad)."""
    Kn = len(maps)
    if cnt_h[:, 2].any():
        raise RuntimeError("persistence pair buffer overflow: max_pairs below kernels.ph_max_pairs(interp, interp)")
    flat, off = _entry_csr(tuple(tuple(e) for e in entries), tuple(maps))
    pairs_c = np.ascontiguousarray(pairs_h, dtype=np.int32)
    cnt_c = np.ascontiguousarray(cnt_h, dtype=np.int32)
    vals_c = np.ascontiguousarray(vals_h, dtype=np.float32)
    loss = np.zeros(1, np.float64)
    dpred = np.zeros((Kn, vals_c.shape[1]), np.float32) if want_grad else None
    rc = _lib.load().octsam_topo_host(pairs_c.ctypes.data, cnt_c.ctypes.data, vals_c.ctypes.data, Kn,
                                      pairs_c.shape[1], vals_c.shape[1], flat.ctypes.data, off.ctypes.data,
                                      len(entries), 0 if feat_d == 0 else 1, float(loss_q), float(lamda),
                                      int(want_grad), loss.ctypes.data,
                                      dpred.ctypes.data if want_grad else None)
    _lib.check(rc, "octsam_topo_host")
    return float(loss[0]), dpred


def topo_device_backward(masks: torch.Tensor, midx: torch.Tensor, dp: torch.Tensor, dmask: torch.Tensor, *,
                         interp=50, logits=True, compact=False):
    """dmask += d topo / d masks, given d topo / d (resampled sigmoid map) dp [Kn, side^2] (capturable).
    compact: dmask is [Kn, H, W], the Kn maps themselves (dicece_pp_rows' dkeep)."""
    B, N, H, W = masks.shape
    oh, ow = (interp, interp) if interp else (H, W)
    _lib.call("octsam_topo_bwd_compact" if compact else "octsam_topo_bwd", K.ptr(masks), K.ptr(midx), midx.numel(),
              H, W, oh, ow, int(logits), K.ptr(dp), 1.0, K.ptr(dmask))


def total_persistence_host(pairs_h, cnt_h, vals_h, entries, maps, *, col, q, lamda, dpred=None):
    """loss_r of topological_loss.py:88-94: lamda * mean over the pred diagrams of every entry of
    torch_topological.utils.total_persistence(diagram, p=q) = sum |death - birth|^q; its gradient is added
    into dpred [Kn, nvals]. Off the reference's path (loss_r=False there); host numpy."""
    pos = {m: i for i, m in enumerate(maps)}
    ks = [pos[m] for e in entries for m in e]
    if not ks:
        return 0.0
    total = 0.0
    for k in ks:
        pr = pairs_h[k, : cnt_h[k, col]]
        b = vals_h[k][pr[:, 0]].astype(np.float64)
        d = vals_h[k][pr[:, 1]].astype(np.float64)
        diff = d - b
        total += float(np.sum(np.abs(diff) ** q))
        if dpred is not None and len(pr):
            g = (lamda / len(ks)) * q * np.abs(diff) ** (q - 1) * np.sign(diff)
            np.add.at(dpred[k], pr[:, 1], g.astype(np.float32))
            np.add.at(dpred[k], pr[:, 0], (-g).astype(np.float32))
    return lamda * total / len(ks)


def topo_forward_backward(masks: torch.Tensor, gt_u8: torch.Tensor, dmask: torch.Tensor | None, *, lamda=0.1,
                          interp=50, feat_d=1, loss_q=2, mode="first", max_pairs=None, logits=True,
                          global_batch: int | None = None, loss_r=False, as_tensor=False):
    """Topological loss value (float; as_tensor: a float64 [1] device tensor, no host sync) and, when dmask is
    given, its gradient added into dmask. masks fp32 [B,N,H,W] (logits; sigmoid applied inside like
    training_utils.py:64). feat_d = 2 (the reference's default) selects no pairs of a 2-D map: the loss is 0, as
    gudhi reports no H2 there. The transport runs on the device (octsam_topo_w2); loss_r (total persistence,
    off the reference's path) adds a host pass."""
    zero = (lambda: torch.zeros(1, dtype=torch.float64, device=masks.device)) if as_tensor else (lambda: 0.0)
    if lamda == 0.0:
        return zero()
    if not 0 <= feat_d <= 2:
        raise NotImplementedError("feat_d outside [0, 2] (unfiltered dimensions) is not supported")
    if feat_d == 2:
        return zero()
    B, N, H, W = masks.shape
    if not interp and (H * W > 4096 or (H + 1) * (W + 1) + H * W > 8192):
        raise NotImplementedError(f"interp=0 needs maps the persistence kernel accepts (<= 64x63), got {H}x{W}")
    entries, maps, midx = topo_index(B, N, mode, global_batch, masks.device)
    if not entries:
        return zero()
    pairs, cnt, both = topo_device_forward(masks, gt_u8, midx, interp=interp, feat_d=feat_d, max_pairs=max_pairs,
                                           logits=logits)
    if not loss_r:
        loss, dpred = topo_w2_device(pairs, cnt, both, entries, maps, lamda=lamda, feat_d=feat_d, loss_q=loss_q,
                                     want_grad=dmask is not None)
        if dmask is not None:
            topo_device_backward(masks, midx, dpred, dmask, interp=interp, logits=logits)
        if as_tensor:
            return loss
        v = float(loss.cpu()[0])
        if math.isnan(v):
            raise RuntimeError("persistence pair buffer overflow: max_pairs below kernels.ph_max_pairs(interp, interp)")
        return v
    host = [t.cpu() for t in (pairs, cnt, both)]  # one D2H sync per step (diagrams are tiny)
    ph, ch, vh = (t.numpy() for t in host)
    loss, dpred = topo_host(ph, ch, vh, entries, maps, lamda=lamda, feat_d=feat_d, loss_q=loss_q,
                            want_grad=dmask is not None)
    if loss_r:
        loss += total_persistence_host(ph, ch, vh, entries, maps, col=0 if feat_d == 0 else 1, q=loss_q,
                                       lamda=lamda, dpred=dpred)
    if dmask is not None:
        topo_device_backward(masks, midx, torch.from_numpy(dpred).to(masks.device), dmask, interp=interp,
                             logits=logits)
    return torch.tensor([loss], dtype=torch.float64, device=masks.device) if as_tensor else loss


class _TopoFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, maps, gt_u8, lamda, interp, feat_d, loss_q, mode, logits, loss_r):
        x = maps.float().contiguous()
        dmask = torch.zeros_like(x)
        loss = topo_forward_backward(x, gt_u8, dmask, lamda=lamda, interp=interp, feat_d=feat_d, loss_q=loss_q,
                                     mode=mode, logits=logits, loss_r=loss_r, as_tensor=True)
        ctx.save_for_backward(dmask)
        ctx.in_dtype = maps.dtype
        return loss.to(torch.float32).reshape(())

    @staticmethod
    def backward(ctx, g):
        (dmask,) = ctx.saved_tensors
        return (dmask * g).to(ctx.in_dtype), None, None, None, None, None, None, None, None


def _as_u8(t):
    return _binary_u8(t, "topo_loss")


def topo_loss_from_logits(masks, gt, lamda, interp=50, feat_d=1, loss_q=2, mode="first"):
    """topo_loss(sigmoid(masks.float()), gt.float(), ...) of training_utils.py:64, sigmoid fused."""
    return _TopoFn.apply(masks, _as_u8(gt), lamda, interp, feat_d, loss_q, mode, True, False)


def topo_loss(pred_obj, true_obj, lamda, interp=0, feat_d=2, loss_q=2, loss_r=False, mode="first"):
    """Signature of ref:octsam/models/topological_loss.py:11 on [B, N, H, W] probability maps and
    binary targets (anything else raises ValueError). interp=0 runs the persistence on the maps as they
    are (the kernel takes up to 64x63; larger maps raise NotImplementedError); loss_r adds the total-
    persistence regulariser of :88-94. Returns a 0-dim float32 tensor (0.0 when lamda == 0, as :30-31)."""
    if lamda == 0.0:
        return 0.0
    if pred_obj.dim() != 4:
        raise ValueError("expected [B, C, H, W] maps")
    return _TopoFn.apply(pred_obj, _as_u8(true_obj), lamda, interp, feat_d, loss_q, mode, False, loss_r)
