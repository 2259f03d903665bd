"""LayerNorm and ViT-attention kernels vs plain PyTorch fp32 references of the same ops
(hf:modeling_sam.py:729-882 restated in fp32 on the same bf16-rounded inputs)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


@pytest.mark.parametrize("D", [64, 256, 768])
@pytest.mark.parametrize("act", [0, 2])
def test_layernorm_fwd_bwd(cuda, D, act):
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(D + act)
    rows = 1000
    x = torch.randn(rows, D, generator=g).to(cuda) * 3 + 1
    w = torch.randn(D, generator=g).to(cuda)
    b = torch.randn(D, generator=g).to(cuda)
    y = torch.empty(rows, D, device=cuda)
    mean = torch.empty(rows, device=cuda)
    rstd = torch.empty(rows, device=cuda)
    kernels.layernorm_fwd(x, w, b, 1e-6, y, act=act, mean=mean, rstd=rstd)
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    br = b.clone().requires_grad_()
    ref = F.layer_norm(xr, (D,), wr, br, 1e-6)
    if act == 2:
        ref = F.gelu(ref)
    assert _rel(y, ref) < 1e-5
    dy = torch.randn(rows, D, generator=g).to(cuda)
    ref.backward(dy)
    dx = torch.empty_like(x)
    _, dw, db = kernels.layernorm_bwd(dy, x, mean, rstd, w, b, dx, act=act)
    assert _rel(dx, xr.grad) < 1e-4
    assert _rel(dw, wr.grad) < 1e-4
    assert _rel(db, br.grad) < 1e-4


@pytest.mark.parametrize("D", [64, 256, 768])
@pytest.mark.parametrize("rows", [37, 4099])
def test_layernorm_bf16_beta_dual(cuda, D, rows):
    """bf16 input / fp32 second output (decoder residual stream), ragged row counts; backward with bf16 dy,
    beta-accumulated fp32 dx and the bf16 dx copy."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(D * 3 + rows)
    x = (torch.randn(rows, D, generator=g) * 2 - 0.5).to(cuda, torch.bfloat16)
    w = torch.randn(D, generator=g).to(cuda)
    b = torch.randn(D, generator=g).to(cuda)
    y = torch.empty(rows, D, device=cuda, dtype=torch.bfloat16)
    y2 = torch.empty(rows, D, device=cuda)
    mean = torch.empty(rows, device=cuda)
    rstd = torch.empty(rows, device=cuda)
    kernels.layernorm_fwd(x, w, b, 1e-6, y, out2_f32=y2, mean=mean, rstd=rstd)
    xr = x.float().requires_grad_()
    ref = F.layer_norm(xr, (D,), w, b, 1e-6)
    assert _rel(y2, ref) < 1e-5 and _rel(y, ref) < 8e-3
    dy = torch.randn(rows, D, generator=g).to(cuda, torch.bfloat16)
    ref.backward(dy.float())
    dx0 = torch.randn(rows, D, generator=g).to(cuda)
    dx = dx0.clone()
    dx2 = torch.empty(rows, D, device=cuda, dtype=torch.bfloat16)
    kernels.layernorm_bwd(dy, x, mean, rstd, w, b, dx, beta=1.0, dx2_bf16=dx2)
    want = xr.grad + dx0
    assert _rel(dx, want) < 1e-4 and _rel(dx2, want) < 8e-3


def test_layernorm_gather_rows(cuda):
    from dilabhelmholtzoct_amd import kernels
    x = torch.randn(10, 768, device=cuda)
    w = torch.ones(768, device=cuda)
    b = torch.zeros(768, device=cuda)
    src = torch.tensor([3, -1, 0, 9, -1], dtype=torch.int32, device=cuda)
    y = torch.empty(5, 768, device=cuda, dtype=torch.bfloat16)
    kernels.layernorm_fwd(x, w, b, 1e-6, y, src_rows=src)
    ref = F.layer_norm(x, (768,), eps=1e-6)
    assert _rel(y[0], ref[3]) < 1e-2 and _rel(y[2], ref[0]) < 1e-2 and _rel(y[3], ref[9]) < 1e-2
    assert torch.all(y[1] == 0) and torch.all(y[4] == 0)


def _ref_attention(qkv, Rh, Rw, nseq, side, heads, hd=64):
    """HF SamVisionAttention math (eager path) in fp32."""
    T = side * side
    qkv = qkv.float().reshape(nseq, T, 3, heads, hd).permute(2, 0, 3, 1, 4).reshape(3, nseq * heads, T, hd)
    q, k, v = qkv.unbind(0)
    attn = (q * hd ** -0.5) @ k.transpose(-2, -1)
    idx = (torch.arange(side)[:, None] - torch.arange(side)[None, :] + side - 1).to(q.device)
    Rh_ = Rh.float()[idx]  # [side, side, hd]
    Rw_ = Rw.float()[idx]
    rq = q.reshape(-1, side, side, hd)
    rel_h = torch.einsum("bhwc,hkc->bhwk", rq, Rh_)
    rel_w = torch.einsum("bhwc,wkc->bhwk", rq, Rw_)
    bias = (rel_h[:, :, :, :, None] + rel_w[:, :, :, None, :]).reshape(-1, T, T)
    attn = torch.softmax(attn + bias, dim=-1)
    o = (attn @ v).reshape(nseq, heads, side, side, hd).permute(0, 2, 3, 1, 4).reshape(nseq, T, heads * hd)
    return o


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hd", [64, 80])
@pytest.mark.parametrize("side,nseq,heads", [(14, 6, 3), (64, 2, 2)])
def test_vit_attention(cuda, side, nseq, heads, hd, dtype):
    """Global (side 64) and windowed (side 14) attention, head_dim 64 (vit-b/l) and 80 (vit-h), bf16 and fp16
    operands, vs fp32 attention on the same rounded inputs (rel-pos tables rounded like the kernel's)."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(side + hd)
    T = side * side
    qkv = torch.randn(nseq, T, 3 * heads * hd, generator=g).to(cuda, dtype)
    Rh = (0.3 * torch.randn(2 * side - 1, hd, generator=g)).to(cuda)
    Rw = (0.3 * torch.randn(2 * side - 1, hd, generator=g)).to(cuda)
    Rh_b, Rw_b = Rh.to(dtype).float(), Rw.to(dtype).float()
    out = torch.empty(nseq, T, heads * hd, device=cuda, dtype=dtype)
    kernels.vit_attention(qkv, out, Rh, Rw, nseq=nseq, side=side, heads=heads)
    ref = _ref_attention(qkv, Rh_b, Rw_b, nseq, side, heads, hd)
    err = (out.float() - ref).abs().max().item()
    assert err < (2e-2 if dtype == torch.bfloat16 else 4e-3), err


@pytest.mark.parametrize("hd", [64, 80])
@pytest.mark.parametrize("side,nseq", [(14, 64), (64, 8)])
def test_vit_attention_deterministic(cuda, side, nseq, hd):
    """Windowed (side 14) and global (side 64) attention at the encoder's shapes: repeated launches give
    identical bits (graph replay must reproduce eager steps exactly; an early read of an MFMA result
    register once made the global kernel's row max, and so its rounding, vary run to run)."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(side + nseq)
    T = side * side
    heads = 768 // 64 if hd == 64 else 16
    qkv = (0.5 * torch.randn(nseq * T, 3 * heads * hd, generator=g)).to(cuda, torch.bfloat16)
    Rh = (0.1 * torch.randn(2 * side - 1, hd, generator=g)).to(cuda)
    Rw = (0.1 * torch.randn(2 * side - 1, hd, generator=g)).to(cuda)
    outs = []
    for _ in range(3):
        o = torch.empty(nseq * T, heads * hd, device=cuda, dtype=torch.bfloat16)
        kernels.vit_attention(qkv, o, Rh, Rw, nseq=nseq, side=side, heads=heads)
        outs.append(o)
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def _window_partition(x, grid, ws, pad):
    """[B*grid*grid, C] token rows -> [B*nw*nw*ws*ws, C] window rows, padding rows = pad (hf:modeling_sam.py:900-929
    pads with zeros after layer_norm1, so a padding row's qkv is the bias)."""
    B = x.shape[0] // (grid * grid)
    nw = (grid + ws - 1) // ws
    xp = pad.view(1, 1, 1, -1).expand(B, nw * ws, nw * ws, x.shape[1]).clone()
    xp[:, :grid, :grid] = x.view(B, grid, grid, -1)
    return xp.view(B, nw, ws, nw, ws, -1).permute(0, 1, 3, 2, 4, 5).reshape(-1, x.shape[1])


def _window_unpartition(xw, B, grid, ws):
    nw = (grid + ws - 1) // ws
    x = xw.view(B, nw, nw, ws, ws, -1).permute(0, 1, 3, 2, 4, 5).reshape(B, nw * ws, nw * ws, -1)
    return x[:, :grid, :grid].reshape(B * grid * grid, -1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hd,heads", [(64, 12), (80, 4)])
@pytest.mark.parametrize("grid,B", [(64, 2), (23, 3), (14, 1)])
def test_vit_attention_token_ordered_windows(cuda, grid, B, hd, heads, dtype):
    """Windowed attention on token-ordered qkv (grid > 0: the partition / unpartition and the padding tokens'
    bias row inside the kernel) is bit-identical to the window-ordered launch on the explicitly partitioned
    tensor (which test_vit_attention checks against fp32), including ragged grids (23 = 14 + 9) and a grid
    with no padding (14)."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(grid * 7 + hd + B)
    D = heads * hd
    ws = 14
    nw = (grid + ws - 1) // ws
    qkv = (0.5 * torch.randn(B * grid * grid, 3 * D, generator=g)).to(cuda, dtype)
    pad = (0.5 * torch.randn(3 * D, generator=g)).to(cuda, dtype)
    Rh = (0.2 * torch.randn(2 * ws - 1, hd, generator=g)).to(cuda)
    Rw = (0.2 * torch.randn(2 * ws - 1, hd, generator=g)).to(cuda)
    qkv_w = _window_partition(qkv, grid, ws, pad)
    out_w = torch.empty(qkv_w.shape[0], D, device=cuda, dtype=dtype)
    kernels.vit_attention(qkv_w, out_w, Rh, Rw, nseq=B * nw * nw, side=ws, heads=heads)
    out = torch.full((B * grid * grid, D), float("nan"), device=cuda, dtype=dtype)
    kernels.vit_attention(qkv, out, Rh, Rw, nseq=B * nw * nw, side=ws, heads=heads, grid=grid, pad_row=pad)
    assert torch.equal(out, _window_unpartition(out_w, B, grid, ws))


def test_patchify_bf16(cuda):
    """Patch-embedding operand: rows (b, patch row, patch col), k = (c, ky, kx), bf16-rounded pixels."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(12)
    B = 2
    px = torch.randn(B, 3, 1024, 1024, generator=g).to(cuda)
    out = torch.empty(B * 4096, 768, device=cuda, dtype=torch.bfloat16)
    kernels.patchify_bf16(px, out)
    ref = px.view(B, 3, 64, 16, 64, 16).permute(0, 2, 4, 1, 3, 5).reshape(B * 4096, 768).to(torch.bfloat16)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("ld,cols,off,nper", [(256, 128, 0, 5), (256, 128, 128, 5), (128, 128, 0, 5), (24, 12, 0, 5),
                                             (256, 256, 0, 21), (256, 128, 128, 16)])
def test_group_sum(cuda, ld, cols, off, nper):
    """out[g] = sum over the nper prompt blocks of image g (fixed order), strided column window; bf16 out. The
    8-column kernel keeps 8 loads in flight but adds in block order: bit-identical to a sequential fp32 sum."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(ld + cols + off + nper)
    G, rows = 3, 4096
    x = torch.randn(G * nper * rows, ld, generator=g).to(cuda, torch.bfloat16)
    out = torch.empty(G * rows, cols, device=cuda, dtype=torch.bfloat16)
    kernels.group_sum(x[:, off:], out, ld_in=ld, cols=cols, groups=G, nper=nper, rows_per=rows)
    ref = x[:, off:off + cols].float().view(G, nper, rows, cols).sum(1).reshape(G * rows, cols)
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    blocks = x[:, off:off + cols].float().view(G, nper, rows, cols)
    seq = blocks[:, 0].clone()
    for j in range(1, nper):
        seq += blocks[:, j]
    assert torch.equal(out, seq.reshape(G * rows, cols).to(torch.bfloat16))


@pytest.mark.parametrize("rows,cols,dt", [(688128, 256, torch.bfloat16), (4097, 256, torch.float32),
                                          (1176, 64, torch.bfloat16), (33, 128, torch.float32)])
def test_colsum(cuda, rows, cols, dt):
    """Column sums (bias gradients) over many rows: fixed-order partials (deterministic), against torch fp64."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(rows + cols)
    x = torch.randn(rows, cols, generator=g).to(cuda, dt)
    outs = []
    for _ in range(2):
        out = torch.empty(cols, device=cuda)
        kernels.colsum(x, rows, cols, out)
        outs.append(out)
    ref = x.double().sum(0)
    assert torch.equal(outs[0], outs[1])
    assert (outs[0].double() - ref).abs().max().item() < 1e-4 * max(1.0, rows ** 0.5)
