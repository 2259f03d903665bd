"""Thin, typed Python wrappers over the C ABI (no autograd). Every function launches HIP work
on torch's current stream and raises OctsamError on any failure; there is no CPU path."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import GemmArgs, ptr


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("octsam kernels take device tensors only")


def gemm(A: torch.Tensor, B: torch.Tensor, *, M: int, N: int, K: int, out: torch.Tensor,
         a_mode: int = 0, b_mode: int = 0, lda: int | None = None, ldb: int | None = None,
         ldc: int | None = None, bias: torch.Tensor | None = None, residual: torch.Tensor | None = None,
         ldr: int | None = None, act: int = 0, pre_out: torch.Tensor | None = None,
         row_map: torch.Tensor | None = None, alpha: float = 1.0, beta: float = 0.0, batch: int = 1,
         stride_a: int = 0, stride_b: int = 0, stride_c: int = 0, stride_r: int = 0,
         A2: torch.Tensor | None = None, B2: torch.Tensor | None = None, a2_rows: int = 0,
         b2_rows: int = 0, conv_c: int = 0, a_remap: tuple[int, int] = (0, 1),
         b_remap: tuple[int, int] = (0, 1), r_remap: tuple[int, int] = (0, 1)) -> torch.Tensor:
    """C[b] = epi(alpha * A[b] @ B[b]^T); see octsam_gemm in include/octsam.h."""
    _require_cuda(A, B, out, bias, residual, pre_out, row_map, A2, B2)
    if a_mode in (0, 4):
        lda = K if lda is None else lda
    elif a_mode == 1:
        lda = M if lda is None else lda
    else:
        lda = 0 if lda is None else lda
    if ldb is None:
        ldb = K if b_mode == 0 else N
    ldc = N if ldc is None else ldc
    ldr = ldc if ldr is None else ldr
    if bias is not None and bias.dtype != torch.float32:
        raise ValueError("bias must be fp32")
    args = GemmArgs(
        A=ptr(A), B=ptr(B), C=ptr(out), bias=ptr(bias), R=ptr(residual), C_pre=ptr(pre_out),
        row_map=ptr(row_map), A2=ptr(A2), B2=ptr(B2),
        M=M, N=N, K=K, batch=batch, lda=lda, ldb=ldb, ldc=ldc, ldr=ldr,
        stride_a=stride_a, stride_b=stride_b, stride_c=stride_c, stride_r=stride_r,
        alpha=alpha, beta=beta, act=act, a_mode=a_mode, b_mode=b_mode,
        c_f32=int(out.dtype == torch.float32),
        r_f32=int(residual is not None and residual.dtype == torch.float32),
        pre_f32=int(pre_out is not None and pre_out.dtype == torch.float32),
        conv_c=conv_c, a2_rows=a2_rows, b2_rows=b2_rows, a_blk=a_remap[0], a_rep=a_remap[1],
        b_blk=b_remap[0], b_rep=b_remap[1], r_blk=r_remap[0], r_rep=r_remap[1])
    _lib.call("octsam_gemm", ctypes.byref(args))
    return out


def splitk_reduce(partials: torch.Tensor, out: torch.Tensor, splits: int, beta: float = 0.0) -> torch.Tensor:
    _require_cuda(partials, out)
    _lib.call("octsam_splitk_reduce", ptr(partials), ptr(out), out.numel(), splits, beta)
    return out


def cubical_ph(maps: torch.Tensor, max_pairs: int = 1024):
    """Persistence pairs of every [H, W] map in ``maps`` ([nmaps, H, W] fp32, device).

    Returns (pairs0, pairs1, essential, counts) int32 device tensors; see octsam_cubical_ph."""
    _require_cuda(maps)
    maps = maps.contiguous().float()
    nmaps, H, W = maps.shape
    dev = maps.device
    pairs0 = torch.empty((nmaps, max_pairs, 2), dtype=torch.int32, device=dev)
    pairs1 = torch.empty((nmaps, max_pairs, 2), dtype=torch.int32, device=dev)
    essential = torch.empty((nmaps, 2), dtype=torch.int32, device=dev)
    counts = torch.empty((nmaps, 3), dtype=torch.int32, device=dev)
    _lib.call("octsam_cubical_ph", ptr(maps), nmaps, H, W, max_pairs, ptr(pairs0), ptr(pairs1),
              ptr(essential), ptr(counts))
    return pairs0, pairs1, essential, counts


def layernorm_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float, out: torch.Tensor, *,
                  rows: int | None = None, src_rows: torch.Tensor | None = None, act: int = 0,
                  out2_f32: torch.Tensor | None = None, mean: torch.Tensor | None = None,
                  rstd: torch.Tensor | None = None) -> torch.Tensor:
    """LayerNorm over the last dim; see octsam_layernorm_fwd."""
    _require_cuda(x, w, b, out, src_rows, out2_f32, mean, rstd)
    D = w.numel()
    if rows is None:
        rows = out.numel() // D
    _lib.call("octsam_layernorm_fwd", ptr(x), int(x.dtype == torch.float32), ptr(src_rows), rows, D, ptr(w),
              ptr(b), eps, ptr(out), int(out.dtype == torch.float32), ptr(out2_f32), act, ptr(mean), ptr(rstd))
    return out


def layernorm_bwd(dy: torch.Tensor, x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, w: torch.Tensor,
                  b: torch.Tensor, dx: torch.Tensor, *, act: int = 0, beta: float = 0.0, nblocks: int = 512):
    """Returns (dx, dw, db); dw/db reduced deterministically from per-block partials."""
    _require_cuda(dy, x, mean, rstd, w, b, dx)
    D = w.numel()
    rows = mean.numel()
    nblocks = max(1, min(nblocks, (rows + 3) // 4))
    part = torch.empty((2, nblocks, D), device=dy.device, dtype=torch.float32)
    _lib.call("octsam_layernorm_bwd", ptr(dy), int(dy.dtype == torch.float32), ptr(x),
              int(x.dtype == torch.float32), ptr(mean), ptr(rstd), ptr(w), ptr(b), act, rows, D, ptr(dx),
              int(dx.dtype == torch.float32), beta, ptr(part[0]), ptr(part[1]), nblocks)
    dw = torch.empty(D, device=dy.device, dtype=torch.float32)
    db = torch.empty(D, device=dy.device, dtype=torch.float32)
    splitk_reduce(part[0], dw, nblocks)
    splitk_reduce(part[1], db, nblocks)
    return dx, dw, db


def vit_attention(qkv: torch.Tensor, out: torch.Tensor, rel_pos_h: torch.Tensor, rel_pos_w: torch.Tensor, *,
                  nseq: int, side: int, heads: int) -> torch.Tensor:
    """Fused SAM ViT attention with decomposed rel-pos bias; see octsam_vit_attention."""
    _require_cuda(qkv, out, rel_pos_h, rel_pos_w)
    if qkv.dtype != torch.bfloat16 or out.dtype != torch.bfloat16:
        raise ValueError("vit_attention expects bf16 qkv/out")
    if qkv.numel() != nseq * side * side * 3 * heads * 64:
        raise ValueError("qkv shape does not match nseq/side/heads")
    _lib.call("octsam_vit_attention", ptr(qkv), ptr(out), ptr(rel_pos_h.float().contiguous()),
              ptr(rel_pos_w.float().contiguous()), nseq, side, heads, 64)
    return out
