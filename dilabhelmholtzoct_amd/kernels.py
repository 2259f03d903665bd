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
         b_remap: tuple[int, int] = (0, 1), r_remap: tuple[int, int] = (0, 1), k_total: int = 0,
         a_colsum: torch.Tensor | None = None, b_colsum: torch.Tensor | None = None) -> torch.Tensor:
    """C[b] = epi(alpha * A[b] @ B[b]^T); see octsam_gemm in include/octsam.h. The 16-bit operand type (bf16 or
    fp16: octsam_gemm_f16) is B's; every other 16-bit operand must match it. a_colsum / b_colsum (fp32
    [batch, M] / [batch, N], k-major operands only): per-batch column sums of A / B, fused."""
    _require_cuda(A, B, out, bias, residual, pre_out, row_map, A2, B2, a_colsum, b_colsum)
    for name, t, n in (("a_colsum", a_colsum, M), ("b_colsum", b_colsum, N)):
        if t is not None and (t.dtype != torch.float32 or t.numel() < batch * n or not t.is_contiguous()):
            raise ValueError(f"{name} must be contiguous fp32 with batch * {n} elements")
    e16 = B.dtype
    if e16 not in (torch.bfloat16, torch.float16):
        raise ValueError(f"B must be bf16 or fp16, got {e16}")
    for name, t in (("A", A), ("out", out), ("residual", residual), ("pre_out", pre_out), ("A2", A2), ("B2", B2)):
        if t is not None and t.dtype not in (e16, torch.float32):
            raise ValueError(f"{name} is {t.dtype}; the GEMM's 16-bit type is {e16}")
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
        b_blk=b_remap[0], b_rep=b_remap[1], r_blk=r_remap[0], r_rep=r_remap[1], k_total=k_total,
        c_rows=_mapped_rows(out, ldc, residual, ldr, pre_out) if row_map is not None else 0,
        a_colsum=ptr(a_colsum), b_colsum=ptr(b_colsum))
    _lib.call("octsam_gemm_f16" if e16 == torch.float16 else "octsam_gemm", ctypes.byref(args))
    return out


def _span_rows(t: torch.Tensor, ld: int) -> int:
    """Rows of leading dimension ld addressable from t's first element to the end of its storage (a column-sliced
    or offset view included)."""
    return (t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()) // ld


def _mapped_rows(out, ldc, residual, ldr, pre_out) -> int:
    """c_rows of a row-mapped GEMM: the rows every row-mapped operand (C, R, C_pre) can hold; the lean epilogue
    range-checks C, R and C_pre against c_rows * ld."""
    rows = _span_rows(out, ldc)
    if residual is not None:
        rows = min(rows, _span_rows(residual, ldr))
    if pre_out is not None:
        rows = min(rows, _span_rows(pre_out, ldc))
    return min(rows, 2 ** 31 - 1)


def splitk_reduce(partials: torch.Tensor, out: torch.Tensor, splits: int, beta: float = 0.0) -> torch.Tensor:
    _require_cuda(partials, out)
    _lib.call("octsam_splitk_reduce", ptr(partials), ptr(out), out.numel(), splits, beta)
    return out


def wgrad_supported(M: int, O: int, I: int) -> bool:
    return bool(_lib.load().octsam_wgrad_supported(M, O, I))


def wgrad(dy: torch.Tensor, x: torch.Tensor, M: int, out: torch.Tensor, *, ldy: int | None = None,
          ldx: int | None = None, beta: float = 0.0, db: torch.Tensor | None = None, dbx: torch.Tensor | None = None,
          dbx_fold: int = 1) -> torch.Tensor:
    """out[O, I] = beta * out + dy[M, O]^T x[M, I] (bf16 operands with row strides ldy / ldx, fp32 out), db = column
    sums of dy, dbx = column sums of x folded over dbx_fold column groups (octsam_wgrad)."""
    _require_cuda(dy, x, out, db, dbx)
    O, I = out.shape
    ldy = O if ldy is None else ldy
    ldx = I if ldx is None else ldx
    if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or out.dtype != torch.float32:
        raise ValueError("wgrad: bf16 operands and an fp32 output")
    if not out.is_contiguous():
        raise ValueError("wgrad: out must be contiguous (the final reduction writes O*I floats from its base)")
    for name, t in (("db", db), ("dbx", dbx)):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError(f"wgrad: {name} must be contiguous fp32")
    lib = _lib.load()
    nbytes = lib.octsam_wgrad_workspace(M, O, I)
    ws = torch.empty(max(nbytes, 16), device=out.device, dtype=torch.uint8)
    _lib.call("octsam_wgrad", ptr(dy), ldy, ptr(x), ldx, M, O, I, ptr(out), beta, ptr(db), ptr(dbx), dbx_fold,
              ptr(ws), nbytes)
    return out


def wgrad_tok(dy: torch.Tensor, x: torch.Tensor, M: int, out: torch.Tensor, *, ldy: int | None = None,
              ldx: int | None = None, beta: float = 0.0, db: torch.Tensor | None = None) -> torch.Tensor:
    """Token-side weight gradient in one launch: out[O, I] = beta * out + dy[M, O]^T x[M, I], db = column sums of dy
    (octsam_wgrad_tok; bf16 operands with row strides ldy / ldx, fp32 out / db)."""
    _require_cuda(dy, x, out, db)
    O, I = out.shape
    ldy = O if ldy is None else ldy
    ldx = I if ldx is None else ldx
    if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("wgrad_tok: bf16 operands and a contiguous fp32 output")
    if db is not None and (db.dtype != torch.float32 or not db.is_contiguous()):
        raise ValueError("wgrad_tok: db must be contiguous fp32")
    _lib.call("octsam_wgrad_tok", ptr(dy), ldy, ptr(x), ldx, M, O, I, ptr(out), beta, ptr(db))
    return out


TOK_GROUP_MAX = 24


def wgrad_tok_group(problems) -> None:
    """Several wgrad_tok problems in one launch (octsam_wgrad_tok_group): problems = [(dy, x, M, out, ldy, ldx, beta,
    db)], at most TOK_GROUP_MAX, no two sharing an output; each gives the same bits as its own wgrad_tok call."""
    n = len(problems)
    if not 0 < n <= TOK_GROUP_MAX:
        raise ValueError(f"wgrad_tok_group: 1..{TOK_GROUP_MAX} problems, got {n}")
    arrs = {k: (t * n)() for k, t in (("dy", ctypes.c_void_p), ("x", ctypes.c_void_p), ("out", ctypes.c_void_p),
                                       ("db", ctypes.c_void_p), ("ldy", ctypes.c_int64), ("ldx", ctypes.c_int64),
                                       ("M", ctypes.c_int64), ("O", ctypes.c_int32), ("I", ctypes.c_int32),
                                       ("beta", ctypes.c_float))}
    for k, (dy, x, M, out, ldy, ldx, beta, db) in enumerate(problems):
        _require_cuda(dy, x, out, db)
        if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("wgrad_tok_group: bf16 operands and contiguous fp32 outputs")
        if db is not None and (db.dtype != torch.float32 or not db.is_contiguous()):
            raise ValueError("wgrad_tok_group: db must be contiguous fp32")
        O, I = out.shape
        arrs["dy"][k], arrs["x"][k], arrs["out"][k], arrs["db"][k] = ptr(dy), ptr(x), ptr(out), ptr(db)
        arrs["ldy"][k], arrs["ldx"][k], arrs["M"][k] = O if ldy is None else ldy, I if ldx is None else ldx, M
        arrs["O"][k], arrs["I"][k], arrs["beta"][k] = O, I, beta
    a = {k: ctypes.cast(v, ctypes.c_void_p) for k, v in arrs.items()}
    _lib.call("octsam_wgrad_tok_group", n, a["dy"], a["ldy"], a["x"], a["ldx"], a["M"], a["O"], a["I"], a["out"],
              a["beta"], a["db"])


def ph_max_pairs(H: int, W: int) -> int:
    """Pair-buffer length that no [H, W] map can overflow: finite H0 pairs are born at regional minima
    (pairwise non-8-adjacent, <= ceil(H/2)*ceil(W/2)) and H1 pairs die at regional maxima (pairwise
    non-4-adjacent, <= ceil(H*W/2)); the kernel's record capacities cover both for every accepted size."""
    return (H * W + 1) // 2


def cubical_ph(maps: torch.Tensor, max_pairs: int | None = None):
    """Persistence pairs of every [H, W] map in ``maps`` ([nmaps, H, W] fp32, device).
    max_pairs defaults to ph_max_pairs(H, W) (cannot overflow).

    Returns (pairs0, pairs1, essential, counts) int32 device tensors; see octsam_cubical_ph."""
    _require_cuda(maps)
    maps = maps.contiguous().float()
    nmaps, H, W = maps.shape
    if max_pairs is None:
        max_pairs = ph_max_pairs(H, W)
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
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("layernorm input must be fp32 or bf16")
    yty = {torch.bfloat16: 0, torch.float32: 1, torch.float16: 2}[out.dtype]
    _lib.call("octsam_layernorm_fwd", ptr(x), int(x.dtype == torch.float32), ptr(src_rows), rows, D, ptr(w),
              ptr(b), eps, ptr(out), yty, ptr(out2_f32), act, ptr(mean), ptr(rstd))
    return out


def layernorm_bwd(dy: torch.Tensor, x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, w: torch.Tensor,
                  b: torch.Tensor, dx: torch.Tensor, *, act: int = 0, beta: float = 0.0, nblocks: int = 512,
                  dx2_bf16: torch.Tensor | None = None, dw: torch.Tensor | None = None,
                  db: torch.Tensor | None = None):
    """Returns (dx, dw, db); dw/db reduced deterministically from per-block partials (written into the
    given dw/db views when provided)."""
    _require_cuda(dy, x, mean, rstd, w, b, dx, dx2_bf16)
    D = w.numel()
    rows = mean.numel()
    if D <= 64:
        nblocks = max(nblocks, 4096)
    elif rows >= 65536:
        nblocks = max(nblocks, 1280)  # image-side rows: 5 waves per SIMD (the kernel's occupancy) in flight
    nblocks = max(1, min(nblocks, (rows + 3) // 4))
    part = torch.empty((2, nblocks, D), device=dy.device, dtype=torch.float32)
    _lib.call("octsam_layernorm_bwd", ptr(dy), int(dy.dtype == torch.float32), ptr(x),
              int(x.dtype == torch.float32), ptr(mean), ptr(rstd), ptr(w), ptr(b), act, rows, D, ptr(dx),
              int(dx.dtype == torch.float32), beta, ptr(dx2_bf16), ptr(part[0]), ptr(part[1]), nblocks)
    if dw is None:
        dw = torch.empty(D, device=dy.device, dtype=torch.float32)
    if db is None:
        db = torch.empty(D, device=dy.device, dtype=torch.float32)
    splitk_reduce(part[0], dw, nblocks)
    splitk_reduce(part[1], db, nblocks)
    return dx, dw, db


def vit_attention(qkv: torch.Tensor, out: torch.Tensor, rel_pos_h: torch.Tensor, rel_pos_w: torch.Tensor, *,
                  nseq: int, side: int, heads: int, grid: int = 0,
                  pad_row: torch.Tensor | None = None) -> torch.Tensor:
    """Fused SAM ViT attention with decomposed rel-pos bias; see octsam_vit_attention. head_dim from the
    rel-pos tables (64 or 80), element type from qkv (bf16 or fp16). grid > 0 (windowed layers): qkv / out are
    token-ordered over images of grid x grid tokens and pad_row ([3 * heads * head_dim], the qkv bias in qkv's
    type) stands for window_partition's padding tokens."""
    _require_cuda(qkv, out, rel_pos_h, rel_pos_w, pad_row)
    if qkv.dtype not in (torch.bfloat16, torch.float16) or out.dtype != qkv.dtype:
        raise ValueError("vit_attention expects bf16 or fp16 qkv / out of the same type")
    hd = rel_pos_h.shape[-1]
    tokens = nseq * side * side
    if grid:
        nw = (grid + side - 1) // side
        if side != 14 or nseq % (nw * nw):
            raise ValueError("token-ordered windows need side 14 and nseq = images * windows per image")
        if pad_row is None or pad_row.dtype != qkv.dtype or pad_row.numel() != 3 * heads * hd:
            raise ValueError("token-ordered windows need pad_row [3 * heads * head_dim] of qkv's type")
        tokens = nseq // (nw * nw) * grid * grid
    if qkv.numel() != tokens * 3 * heads * hd or out.numel() != tokens * heads * hd:
        raise ValueError("qkv / out shape does not match nseq / side / heads / head_dim")
    rh = rel_pos_h.float().contiguous()  # (named, so a converted copy outlives the launch)
    rw = rel_pos_w.float().contiguous()
    _lib.call("octsam_vit_attention", ptr(qkv), ptr(out), ptr(rh), ptr(rw), nseq, side, heads, hd,
              int(qkv.dtype == torch.float16), grid, ptr(pad_row))
    return out


def _f32(t):
    return int(t.dtype == torch.float32)


def axpby(a, b, out, *, alpha=1.0, beta=1.0, b_period=0, out2_f32=None, n=None):
    """out = alpha*a + beta*b (b broadcast with period b_period); a or b may be None."""
    n = out.numel() if n is None else n
    _lib.call("octsam_axpby", ptr(a), _f32(a) if a is not None else 0, ptr(b), _f32(b) if b is not None else 0,
              b_period, alpha, beta, ptr(out), _f32(out), ptr(out2_f32), n)
    return out


def patchify_bf16(px, out):
    """pixel_values fp32 [B, 3, 1024, 1024] -> patch rows [B*4096, 768] (k = c, ky, kx), bf16 or fp16 (out's
    type)."""
    _require_cuda(px, out)
    _lib.call("octsam_patchify_f16" if out.dtype == torch.float16 else "octsam_patchify_bf16", ptr(px), px.shape[0],
              ptr(out))
    return out


def cast_bf16(x, out):
    """fp32 -> out's 16-bit type (bf16 or fp16)."""
    _lib.call("octsam_cast_f16" if out.dtype == torch.float16 else "octsam_cast_bf16", ptr(x), ptr(out), x.numel())
    return out


def colsum(x, rows, cols, out, *, beta=0.0, nblocks=None):
    """out[c] = beta*out[c] + sum_r x[r, c] (x contiguous [rows, cols]); deterministic."""
    if nblocks is None:
        lanes = max(1, 256 // max(1, cols // 8))
        nblocks = max(1, min(1024, (rows + lanes * 16 - 1) // (lanes * 16)))
    part = torch.empty((nblocks, cols), device=x.device, dtype=torch.float32)
    _lib.call("octsam_colsum", ptr(x), _f32(x), rows, cols, ptr(part), nblocks)
    splitk_reduce(part, out, nblocks, beta=beta)
    return out


def relu_bwd(dy, y, out, *, ldy, cols):
    _lib.call("octsam_relu_bwd", ptr(dy), ptr(y), ldy, cols, ptr(out), out.numel())
    return out


def group_sum(x, out, *, ld_in, cols, groups, nper, rows_per):
    _lib.call("octsam_group_sum", ptr(x), ld_in, cols, groups, nper, rows_per, ptr(out))
    return out


def prompt_tokens(boxes, points, labels, P, npts, G, point_embed, not_a_point, out_tokens, input_size, tokens):
    _lib.call("octsam_prompt_tokens", ptr(boxes), ptr(points), ptr(labels), P, npts, ptr(G), ptr(point_embed),
              ptr(not_a_point), ptr(out_tokens), input_size, ptr(tokens))
    return tokens


def image_pe(G, size, out):
    _lib.call("octsam_image_pe", ptr(G), size, ptr(out))
    return out


def tok_attn_fwd(q, k, v, P, T, out, probs):
    _lib.call("octsam_dec_tok_attn_fwd", ptr(q), ptr(k), ptr(v), P, T, ptr(out), ptr(probs))


def tok_attn_bwd(q, k, v, probs, dout, P, T, dq, dk, dv):
    _lib.call("octsam_dec_tok_attn_bwd", ptr(q), ptr(k), ptr(v), ptr(probs), ptr(dout), P, T, ptr(dq), ptr(dk), ptr(dv))


def _t2i_workspace(P, L, device):
    n = _lib.load().octsam_dec_t2i_workspace(P, L)
    return torch.empty(n, device=device, dtype=torch.float32)


def _opt(t):
    return ptr(t) if t is not None else None


def t2i_fwd(q, k, v, ldkv, kv_rep, P, Tq, L, out, lse, score_bias=None, out_f32=None):
    """score_bias: fp32 [P, L] added to the logits (attention_similarity), or None. out_f32: fp32 [P, Tq, 128] that
    also receives the unrounded O (for the backward's delta), or None (octsam_dec_t2i_fwd2)."""
    _require_cuda(q, k, v, out, lse)
    ws = _t2i_workspace(P, L, q.device)
    if score_bias is not None and (score_bias.dtype != torch.float32 or score_bias.numel() != P * L
                                   or not score_bias.is_contiguous()):
        raise ValueError("t2i_fwd: score_bias must be contiguous fp32 [P, L]")
    if out_f32 is not None:
        _require_cuda(out_f32)
        if out_f32.dtype != torch.float32 or out_f32.numel() != P * Tq * 128 or not out_f32.is_contiguous():
            raise ValueError("t2i_fwd: out_f32 must be contiguous fp32 [P, Tq, 128]")
    _lib.call("octsam_dec_t2i_fwd2", ptr(q), ptr(k), ptr(v), ldkv, kv_rep, P, Tq, L, _opt(score_bias), ptr(out),
              _opt(out_f32), ptr(lse), ptr(ws))


def _check_out_f32(out_f32, P, Tq):
    if out_f32 is not None:
        _require_cuda(out_f32)
        if out_f32.dtype != torch.float32 or out_f32.numel() != P * Tq * 128 or not out_f32.is_contiguous():
            raise ValueError("t2i backward: out_f32 must be contiguous fp32 [P, Tq, 128]")


def t2i_bwd(q, k, v, ldkv, kv_rep, P, Tq, L, out, dout, lse, dq, dk, dv, lddkv, out_f32=None):
    """out_f32: the forward's fp32 O (t2i_fwd(out_f32=...)) for delta = dO . O, or None (from the bf16 out)."""
    _require_cuda(q, k, v, out, dout, lse, dq, dk, dv)
    _check_out_f32(out_f32, P, Tq)
    ws = _t2i_workspace(P, L, q.device)
    _lib.call("octsam_dec_t2i_bwd2", ptr(q), ptr(k), ptr(v), ldkv, kv_rep, P, Tq, L, ptr(out), _opt(out_f32),
              ptr(dout), ptr(lse), ptr(dq), ptr(dk), ptr(dv), lddkv, ptr(ws))


def t2i_bwd_sum(q, k, v, ldkv, kv_rep, P, Tq, L, out, dout, lse, dq, dk, dv, lddkv, out_f32=None):
    """t2i_bwd for K / V shared by kv_rep prompts per image with the prompt sum fused in: dk, dv are the image rows
    [(P / kv_rep) * L, lddkv] (octsam_dec_t2i_bwd_sum2)."""
    _require_cuda(q, k, v, out, dout, lse, dq, dk, dv)
    _check_out_f32(out_f32, P, Tq)
    n = _lib.load().octsam_dec_t2i_bwd_sum_workspace(P, Tq, L)
    ws = torch.empty(n, device=q.device, dtype=torch.float32)
    _lib.call("octsam_dec_t2i_bwd_sum2", ptr(q), ptr(k), ptr(v), ldkv, kv_rep, P, Tq, L, ptr(out), _opt(out_f32),
              ptr(dout), ptr(lse), ptr(dq), ptr(dk), ptr(dv), lddkv, ptr(ws))


def i2t_fwd(q, ldq, q_rep, k, v, P, Tk, L, out, ldo):
    _lib.call("octsam_dec_i2t_fwd", ptr(q), ldq, q_rep, ptr(k), ptr(v), P, Tk, L, ptr(out), ldo)


def i2t_bwd(q, ldq, q_rep, k, v, P, Tk, L, dout, lddo, dq, lddq):
    """Returns dk, dv fp32 [P, Tk, 128] each."""
    n = _lib.load().octsam_dec_i2t_bwd_partials(P, Tk, L)
    nb = n // (P * 2 * Tk * 128)
    part = torch.empty(n, device=k.device, dtype=torch.float32)
    _lib.call("octsam_dec_i2t_bwd", ptr(q), ldq, q_rep, ptr(k), ptr(v), P, Tk, L, ptr(dout), lddo, ptr(dq), lddq,
              ptr(part))
    red = torch.empty(P * 2 * Tk * 128, device=k.device, dtype=torch.float32)
    splitk_reduce(part.view(nb, -1), red, nb)
    red = red.view(P, 2, Tk, 128)
    return red[:, 0], red[:, 1]


def i2t_bwd_sum(q, ldq, q_rep, k, v, P, Tk, L, dout, lddo, dq, lddq):
    """i2t_bwd for queries shared by q_rep prompts per image with the prompt sum of dQ fused in: dq holds the image
    rows [(P / q_rep) * L, lddq] (octsam_dec_i2t_bwd_sum). Returns dk, dv fp32 [P, Tk, 128] each."""
    _require_cuda(q, k, v, dout, dq)
    n = _lib.load().octsam_dec_i2t_bwd_sum_partials(P, Tk, L)
    nb = n // (P * 2 * Tk * 128)
    part = torch.empty(n, device=k.device, dtype=torch.float32)
    _lib.call("octsam_dec_i2t_bwd_sum", ptr(q), ldq, q_rep, ptr(k), ptr(v), P, Tk, L, ptr(dout), lddo, ptr(dq), lddq,
              ptr(part))
    red = torch.empty(P * 2 * Tk * 128, device=k.device, dtype=torch.float32)
    splitk_reduce(part.view(nb, -1), red, nb)
    red = red.view(P, 2, Tk, 128)
    return red[:, 0], red[:, 1]


def upmask_fwd(up1, w2, b2, hyper, P, ntok, masks):
    """Fused ConvT2 + GELU + mask head (octsam_upmask_fwd): masks [P, ntok, 256, 256] fp32."""
    _require_cuda(up1, w2, b2, hyper, masks)
    _lib.call("octsam_upmask_fwd", ptr(up1), ptr(w2), ptr(b2), ptr(hyper), P, ntok, ptr(masks))
    return masks


def upmask_bwd(up1, w2, b2, hyper, dmask, P, ntok, dup1, dw2, db2, dhyper, ln=None, ldd=256):
    """Backward of upmask_fwd: writes d up1 (bf16) and overwrites d w2, d b2, d hyper (fp32).
    ln = (x, mean, rstd, ln_w, ln_b, dln_w, dln_b): the LayerNorm2d + GELU that produced up1 from x is
    differentiated in the same pass (octsam_upmask_ln_bwd); dup1 then receives d x, and dln_w / dln_b are overwritten.
    ldd (with ln): elements between the rows of d x's [P * 4096, 256] view (octsam_upmask_ln_bwd_strided)."""
    _require_cuda(up1, w2, b2, hyper, dmask, dup1, dw2, db2, dhyper)
    n = _lib.load().octsam_upmask_bwd_workspace(P, ntok)
    ws = torch.empty(n, device=up1.device, dtype=torch.float32)
    if ln is None:
        _lib.call("octsam_upmask_bwd", ptr(up1), ptr(w2), ptr(b2), ptr(hyper), ptr(dmask), P, ntok, ptr(dup1),
                  ptr(dw2), ptr(db2), ptr(dhyper), ptr(ws))
        return dup1
    x, mean, rstd, lw, lb, dlw, dlb = ln
    _require_cuda(x, mean, rstd, lw, lb, dlw, dlb)
    if ldd != 256:
        _lib.call("octsam_upmask_ln_bwd_strided", ptr(up1), ptr(w2), ptr(b2), ptr(hyper), ptr(dmask), P, ntok, ptr(x),
                  ptr(mean), ptr(rstd), ptr(lw), ptr(lb), ptr(dup1), ldd, ptr(dw2), ptr(db2), ptr(dhyper), ptr(dlw),
                  ptr(dlb), ptr(ws))
        return dup1
    _lib.call("octsam_upmask_ln_bwd", ptr(up1), ptr(w2), ptr(b2), ptr(hyper), ptr(dmask), P, ntok, ptr(x), ptr(mean),
              ptr(rstd), ptr(lw), ptr(lb), ptr(dup1), ptr(dw2), ptr(db2), ptr(dhyper), ptr(dlw), ptr(dlb), ptr(ws))
    return dup1


def mask_embed(masks: torch.Tensor, packed: torch.Tensor, eps: float, out: torch.Tensor) -> torch.Tensor:
    """SamMaskEmbedding forward (octsam_mask_embed): masks fp32 [B, 256, 256] -> out fp32 [B, 4096, 256]."""
    _require_cuda(masks, packed, out)
    B = masks.shape[0]
    if masks.dtype != torch.float32 or masks.numel() != B * 65536 or out.numel() != B * 4096 * 256:
        raise ValueError("mask_embed: masks fp32 [B, 256, 256], out fp32 [B, 4096, 256]")
    _lib.call("octsam_mask_embed", ptr(masks.contiguous()), B, ptr(packed), float(eps), ptr(out))
    return out


def adam(params, grads, exp_avg, exp_avg_sq, *, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt,
         params_bf16=None):
    _lib.call("octsam_adam", ptr(params), ptr(grads), ptr(exp_avg), ptr(exp_avg_sq), params.numel(), beta1, beta2,
              eps, weight_decay, step_size, bc2_sqrt, ptr(params_bf16))


def w2_host(d1: "np.ndarray", d2: "np.ndarray", q: float = 2.0):
    """Host exact q-Wasserstein transport cost and d cost / d d1 (see octsam_w2_host)."""
    import numpy as np
    d1 = np.ascontiguousarray(d1, dtype=np.float32).reshape(-1, 2)
    d2 = np.ascontiguousarray(d2, dtype=np.float32).reshape(-1, 2)
    cost = np.zeros(1, np.float64)
    grad = np.zeros_like(d1)
    rc = _lib.load().octsam_w2_host(d1.ctypes.data if len(d1) else None, len(d1),
                                    d2.ctypes.data if len(d2) else None, len(d2), q, cost.ctypes.data,
                                    grad.ctypes.data if len(d1) else None)
    _lib.check(rc, "octsam_w2_host")
    return float(cost[0]), grad
