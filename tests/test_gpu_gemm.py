"""GEMM parity: octsam_gemm (MFMA bf16, fp32 accumulate) vs a plain PyTorch fp32 reference on the
same bf16-rounded operands, for every operand mode the model uses."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(300, 200, 136), (128, 128, 64), (4096, 768, 768), (7, 40, 256)])
@pytest.mark.parametrize("b_mode", [0, 1])
def test_gemm_nt_nn(cuda, M, N, K, b_mode):
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator(device="cpu").manual_seed(M + N + K + b_mode)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    Bw = torch.randn(N, K, generator=g).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda)
    Bop = Bw if b_mode == 0 else Bw.t().contiguous()
    out = torch.empty(M, N, device=cuda)
    pre = torch.empty(M, N, device=cuda)
    kernels.gemm(A, Bop, M=M, N=N, K=K, out=out, b_mode=b_mode, bias=bias, residual=R, act=2, pre_out=pre)
    ref_pre = A.float() @ Bw.float().t() + bias
    ref = F.gelu(ref_pre) + R
    assert _rel(pre, ref_pre) < 1e-5
    assert _rel(out, ref) < 1e-5


@pytest.mark.parametrize("b_mode", [0, 1])
def test_gemm_transposed_a(cuda, b_mode):
    from dilabhelmholtzoct_amd import kernels
    M, N, K = 256, 136, 520
    g = torch.Generator().manual_seed(3)
    At = torch.randn(K, M, generator=g).to(cuda, torch.bfloat16)  # A stored [K, M]
    Bw = torch.randn(N, K, generator=g).to(cuda, torch.bfloat16)
    Bop = Bw if b_mode == 0 else Bw.t().contiguous()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    kernels.gemm(At, Bop, M=M, N=N, K=K, out=out, a_mode=1, b_mode=b_mode, act=1)
    ref = torch.relu(At.float().t() @ Bw.float().t())
    assert _rel(out, ref) < 8e-3


def test_gemm_batched_beta_rowmap(cuda):
    from dilabhelmholtzoct_amd import kernels
    Bt, M, N, K = 3, 130, 72, 64
    g = torch.Generator().manual_seed(4)
    A = torch.randn(Bt, M, K, generator=g).to(cuda, torch.bfloat16)
    W = torch.randn(Bt, N, K, generator=g).to(cuda, torch.bfloat16)
    C0 = torch.randn(Bt, M, N, generator=g).to(cuda)
    out = C0.clone()
    kernels.gemm(A, W, M=M, N=N, K=K, out=out, batch=Bt, stride_a=M * K, stride_b=N * K, stride_c=M * N,
                 alpha=0.5, beta=2.0)
    ref = 0.5 * torch.bmm(A.float(), W.float().transpose(1, 2)) + 2.0 * C0
    assert _rel(out, ref) < 1e-5
    # row_map: reverse rows and drop every third
    rm = torch.arange(M - 1, -1, -1, dtype=torch.int32)
    rm[::3] = -1
    rm = rm.to(cuda)
    out2 = torch.zeros(M, N, device=cuda)
    kernels.gemm(A[0], W[0], M=M, N=N, K=K, out=out2, row_map=rm)
    full = A[0].float() @ W[0].float().t()
    ref2 = torch.zeros(M, N, device=cuda)
    keep = (rm >= 0).nonzero().flatten()
    ref2[rm[keep].long()] = full[keep]
    assert _rel(out2, ref2) < 1e-5


def test_gemm_patch16(cuda):
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(5)
    px = torch.randn(2, 3, 1024, 1024, generator=g).to(cuda)
    W = (0.05 * torch.randn(96, 3, 16, 16, generator=g)).to(cuda, torch.bfloat16)
    out = torch.empty(2 * 4096, 96, device=cuda)
    kernels.gemm(px, W.reshape(96, 768), M=2 * 4096, N=96, K=768, out=out, a_mode=2)
    ref = F.conv2d(px.to(torch.bfloat16).float(), W.float(), stride=16).permute(0, 2, 3, 1).reshape(-1, 96)
    assert _rel(out, ref) < 1e-5


def test_gemm_conv3x3(cuda):
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(6)
    C, Co = 32, 48
    x = torch.randn(2, 64, 64, C, generator=g).to(cuda, torch.bfloat16)  # NHWC
    W = (0.1 * torch.randn(Co, C, 3, 3, generator=g)).to(cuda, torch.bfloat16)
    Wr = W.permute(0, 2, 3, 1).reshape(Co, 9 * C).contiguous()  # k = (ky,kx,c)
    out = torch.empty(2 * 4096, Co, device=cuda)
    kernels.gemm(x, Wr, M=2 * 4096, N=Co, K=9 * C, out=out, a_mode=3, conv_c=C)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), W.float(), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    assert _rel(out, ref) < 1e-5


def test_gemm_broadcast_addends(cuda):
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(7)
    P, L, C, N = 3, 256, 64, 40
    keys = torch.randn(P * L, C, generator=g).to(cuda, torch.bfloat16)
    pe = torch.randn(L, C, generator=g).to(cuda, torch.bfloat16)
    W = torch.randn(N, C, generator=g).to(cuda, torch.bfloat16)
    out = torch.empty(P * L, N, device=cuda)
    kernels.gemm(keys, W, M=P * L, N=N, K=C, out=out, a_mode=4, A2=pe, a2_rows=L)
    summed = (keys.float().view(P, L, C) + pe.float()).to(torch.bfloat16).float().view(P * L, C)
    assert _rel(out, summed @ W.float().t()) < 1e-5
    # dW = dY^T (keys + pe): A = dY stored [M, N] (transposed mode), B = keys + pe stored [M, C]
    dY = torch.randn(P * L, N, generator=g).to(cuda, torch.bfloat16)
    dW = torch.empty(N, C, device=cuda)
    kernels.gemm(dY, keys, M=N, N=C, K=P * L, out=dW, a_mode=1, b_mode=2, B2=pe, b2_rows=L)
    assert _rel(dW, dY.float().t() @ summed) < 1e-5


def test_splitk_reduce(cuda):
    from dilabhelmholtzoct_amd import kernels
    part = torch.randn(5, 1000, device=cuda)
    out = torch.ones(1000, device=cuda)
    kernels.splitk_reduce(part, out, 5, beta=1.0)
    assert torch.allclose(out, part.sum(0) + 1, atol=1e-5)


@pytest.mark.parametrize("c_f32", [False, True])
@pytest.mark.parametrize("resid", [None, "bf16", "f32"])
@pytest.mark.parametrize("beta", [0.0, 1.5])
@pytest.mark.parametrize("pre", [None, "bf16", "f32"])
def test_gemm_fast_path_epilogues(cuda, c_f32, resid, beta, pre):
    """The persistent LDS-DMA kernel (a_mode = b_mode = 0, M >= 1024, K % 64 == 0) with every epilogue
    option, ragged M/N tiles, batch strides and a row map; the generic kernel and torch fp32 as references."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    Bt, M, N, K = 2, 1100, 392, 192
    g = torch.Generator().manual_seed(int(c_f32) * 100 + int(beta * 10) + len(str(resid)) + len(str(pre)))
    A = torch.randn(Bt, M, K, generator=g).to(cuda, torch.bfloat16)
    W = torch.randn(Bt, N, K, generator=g).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    cdt = torch.float32 if c_f32 else torch.bfloat16
    C0 = torch.randn(Bt, M, N, generator=g).to(cuda, cdt)
    R = None if resid is None else torch.randn(Bt, M, N, generator=g).to(cuda, torch.float32 if resid == "f32"
                                                                          else torch.bfloat16)
    rm = torch.randperm(M, generator=g).to(torch.int32)
    rm[::7] = -1
    rm = rm.to(cuda)
    outs = []
    # 1: default (a row map -> the 8-phase kernel, one tile per workgroup, register epilogue; beta != 0 goes to
    # the ring kernel), 11: same, forced, 8: 8-phase with the LDS-staged epilogue, 5: persistent ring kernel,
    # 0: generic
    for fast in (1, 11, 8, 5, 0):
        lib.octsam_gemm_set_fast_path(fast | 256)  # 256: keep this shape off the small-problem path
        out = C0.clone()
        pout = None if pre is None else torch.zeros(Bt, M, N, device=cuda,
                                                    dtype=torch.float32 if pre == "f32" else torch.bfloat16)
        kw = dict(M=M, N=N, K=K, out=out, batch=Bt, stride_a=M * K, stride_b=N * K, stride_c=M * N, bias=bias,
                  act=2, beta=beta, alpha=0.75, pre_out=pout, row_map=rm)
        if R is not None:
            kw.update(residual=R, stride_r=M * N)
        kernels.gemm(A, W, **kw)
        p8 = 2 if beta == 0.0 else 1
        assert lib.octsam_gemm_last_path() == {1: p8, 11: p8, 8: p8, 5: 1, 0: 0}[fast]
        outs.append((out, pout))
    lib.octsam_gemm_set_fast_path(1)
    keep = (rm >= 0).nonzero().flatten()
    dst = rm[keep].long()
    pre_ref = 0.75 * torch.bmm(A.float(), W.float().transpose(1, 2))[:, keep] + beta * C0.float()[:, dst] + bias
    ref = F.gelu(pre_ref) + (R.float()[:, dst] if R is not None else 0.0)
    tol = 1e-5 if c_f32 else 8e-3
    for out, pout in outs:
        assert _rel(out[:, dst], ref) < tol
        if pout is not None:
            assert _rel(pout[:, dst], pre_ref) < (1e-5 if pre == "f32" else 8e-3)
    # rows dropped by the row map keep their previous contents
    drop = torch.ones(M, dtype=torch.bool, device=cuda)
    drop[dst] = False
    for out, _ in outs:
        assert torch.equal(out[:, drop], C0[:, drop])
    assert all(_rel(o[0], outs[-1][0]) < tol for o in outs[:-1])


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(4096, 2304, 768), (1100, 264, 128), (70000, 512, 64), (9000, 768, 3072), (20000, 2304, 192)])
def test_gemm8_register_epilogue_act(cuda, act, M, N, K):
    """8-phase kernel, register epilogue, each activation against torch fp32 (bf16 out, bf16 residual)."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(act * 7 + M)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda, torch.bfloat16)
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    lib.octsam_gemm_set_fast_path(1 | 256)
    kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=bias, act=act, residual=R)
    assert lib.octsam_gemm_last_path() == 2
    lib.octsam_gemm_set_fast_path(1)
    pre = A.float() @ W.float().t() + bias
    ref = {0: pre, 1: F.relu(pre), 2: F.gelu(pre)}[act] + R.float()
    assert _rel(out, ref) < 8e-3


@pytest.mark.parametrize("act", [0, 2])
@pytest.mark.parametrize("M,N,K,Bt", [(39200, 2304, 768, 1), (4096, 768, 64, 1), (1100, 392, 128, 3),
                                      (70000, 256, 192, 1), (20000, 3072, 768, 1)])
@pytest.mark.parametrize("variant", ["bias", "nobias", "f32out", "pre"])
def test_gemm8_persistent(cuda, act, M, N, K, Bt, variant):
    """Persistent 8-phase kernel (bias from LDS, epilogue overlapped with the next tile's prefetch, relaxed
    waits after full e16 tiles): several tiles per workgroup, K = 64 (one K-step per tile), ragged M/N,
    batch strides, fp32 output and a pre-activation copy (conservative waits) against torch fp32 and the
    one-tile-per-workgroup kernel."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K + act + len(variant))
    A = torch.randn(Bt, M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(Bt, N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = None if variant == "nobias" else torch.randn(N, generator=g).to(cuda)
    cdt = torch.float32 if variant == "f32out" else torch.bfloat16
    outs = []
    for fast in (23, 11):  # 23: the persistent kernel for bias / activation kinds (opt-in), 11: one tile per WG
        lib.octsam_gemm_set_fast_path(fast | 256)
        out = torch.full((Bt, M, N), float("nan"), device=cuda, dtype=cdt)
        pout = torch.zeros(Bt, M, N, device=cuda, dtype=torch.bfloat16) if variant == "pre" else None
        kernels.gemm(A, W, M=M, N=N, K=K, out=out, batch=Bt, stride_a=M * K, stride_b=N * K, stride_c=M * N,
                     bias=bias, act=act, pre_out=pout)
        assert lib.octsam_gemm_last_path() == 2
        outs.append((out, pout))
    lib.octsam_gemm_set_fast_path(1)
    pre = torch.bmm(A.float(), W.float().transpose(1, 2)) + (bias if bias is not None else 0.0)
    ref = F.gelu(pre) if act == 2 else pre
    tol = 1e-5 if variant == "f32out" else 8e-3
    for out, pout in outs:
        assert not torch.isnan(out).any()
        assert _rel(out, ref) < tol
        if pout is not None:
            assert _rel(pout, pre) < 8e-3
    assert torch.equal(outs[0][0], outs[1][0])  # same MFMA order, same epilogue arithmetic


@pytest.mark.parametrize("kind", ["e16", "f32", "e16_res", "f32_res", "f32_res_rowmap", "e16_bres"])
@pytest.mark.parametrize("act", [0, 2])
@pytest.mark.parametrize("N", [512, 392])
def test_gemm8_lean_epilogue_kinds(cuda, kind, act, N):
    """The lean buffer-descriptor epilogue for every output kind the encoder and decoder use — e16 or fp32 C,
    a residual of C's type read in place, a row map with dropped rows (windowed attention's projection), a
    broadcast residual (r_remap: the decoder's per-prompt positional projection) — against torch fp32 and
    against the general register epilogue (fast path 18): ragged M, a ragged last column tile, batch strides."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    rowmap = kind.endswith("rowmap")
    bres = kind.endswith("bres")
    Bt = 1 if (rowmap or bres) else 2
    M, K = 1100, 192
    g = torch.Generator().manual_seed(len(kind) * 10 + act)
    A = torch.randn(Bt, M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(Bt, N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    cdt = torch.float32 if kind.startswith("f32") else torch.bfloat16
    Mc = 1500 if rowmap else M  # rows of C (the row map scatters into a larger output)
    C0 = torch.randn(Bt, Mc, N, generator=g).to(cuda, cdt)
    P = torch.randn(100, N, generator=g).to(cuda, cdt) if bres else None
    rm = None
    if rowmap:
        rm = torch.randperm(Mc, generator=g)[:M].to(torch.int32)
        rm[::5] = -1
        rm = rm.to(cuda)
    outs = []
    for fast in (1, 18):
        lib.octsam_gemm_set_fast_path(fast | 256)
        out = C0.clone()
        kw = dict(M=M, N=N, K=K, out=out, batch=Bt, stride_a=M * K, stride_b=N * K, stride_c=Mc * N, bias=bias,
                  act=act, row_map=rm)
        if bres:
            kw.update(residual=P, r_remap=(100, 11))  # residual row = m % 100 (M = 100 * 11)
        elif "res" in kind:
            kw.update(residual=out, stride_r=Mc * N)
        kernels.gemm(A, W, **kw)
        assert lib.octsam_gemm_last_path() == 2
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    pre = torch.bmm(A.float(), W.float().transpose(1, 2)) + bias
    y = F.gelu(pre) if act == 2 else pre
    keep = torch.arange(M, device=cuda) if rm is None else (rm >= 0).nonzero().flatten()
    dst = keep if rm is None else rm[keep].long()
    ref = C0.float().clone()
    if bres:
        ref[:, dst] = y[:, keep] + P.float()[torch.arange(M, device=cuda) % 100]
    else:
        ref[:, dst] = y[:, keep] + (C0.float()[:, dst] if "res" in kind else 0.0)
    tol = 1e-5 if cdt == torch.float32 else 8e-3
    for out in outs:
        assert _rel(out.float(), ref) < tol
        untouched = torch.ones(Mc, dtype=torch.bool, device=cuda)
        untouched[dst] = False
        assert torch.equal(out[:, untouched], C0[:, untouched])
    assert _rel(outs[0].float(), outs[1].float()) < 1e-6 if cdt == torch.float32 else torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K,kind", [(32768, 768, 3072, "f32_res"), (32768, 768, 768, "f32_res"),
                                         (1100, 768, 192, "f32_res"), (1100, 768, 128, "e16"),
                                         (32768, 2304, 768, "e16")])
@pytest.mark.parametrize("act", [0, 2])
def test_gemm8_n192_tiles(cuda, M, N, K, kind, act):
    """256x192 tiles (opt-in, fast path 24: chosen when they fill the chip's waves better, MLP2 / proj at
    M = 32768): against torch fp32 and bit-identical to the 256x256 kernel (the default), ragged M, in-place fp32
    residual."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K + act)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    f32 = kind == "f32_res"
    X0 = torch.randn(M, N, generator=g).to(cuda, torch.float32 if f32 else torch.bfloat16)
    outs = []
    for fast in (24, 1):  # 24: 256x192 tiles where they quantise better; 1: the default 256x256 tiles
        lib.octsam_gemm_set_fast_path(fast | 256)
        out = X0.clone()
        kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=bias, act=act, residual=out if f32 else None)
        assert lib.octsam_gemm_last_path() == 2
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    pre = A.float() @ W.float().t() + bias
    ref = (F.gelu(pre) if act == 2 else pre) + (X0.float() if f32 else 0.0)
    for out in outs:
        assert _rel(out.float(), ref) < (1e-5 if f32 else 8e-3)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("a_mode,b_mode", [(1, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("shape", [(1104, 392, 192, 2), (256, 256, 128, 64), (128, 264, 64, 40)])
def test_gemm_fast_path_kmajor(cuda, a_mode, b_mode, shape):
    """k-major operands (a_mode 1: A stored [K][M]; b_mode 1: B stored [K][N]) through the persistent
    kernel's LDS transpose reads, incl. the split-K weight-gradient shape (small M x N, many batches)."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    M, N, K, Bt = shape
    g = torch.Generator().manual_seed(M + N + K + 7 * a_mode + 3 * b_mode)
    A = torch.randn(Bt, M, K, generator=g).to(torch.bfloat16)
    W = torch.randn(Bt, N, K, generator=g).to(torch.bfloat16)
    Aop = (A if a_mode == 0 else A.transpose(1, 2)).contiguous().to(cuda)
    Bop = (W if b_mode == 0 else W.transpose(1, 2)).contiguous().to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(Bt, M, N, generator=g).to(cuda, torch.bfloat16)
    ref = F.relu(torch.bmm(A.float(), W.float().transpose(1, 2)).to(cuda) + bias) + R.float()
    for fast in (1, 0):
        lib.octsam_gemm_set_fast_path(fast | 256)
        out = torch.empty(Bt, M, N, device=cuda, dtype=torch.float32)
        kernels.gemm(Aop, Bop, M=M, N=N, K=K, out=out, a_mode=a_mode, b_mode=b_mode, batch=Bt, stride_a=M * K,
                     stride_b=N * K, stride_c=M * N, stride_r=M * N, bias=bias, act=1, residual=R)
        assert (lib.octsam_gemm_last_path() > 0) == bool(fast)
        assert _rel(out, ref) < 1e-5, (fast, _rel(out, ref))
    lib.octsam_gemm_set_fast_path(1)


@pytest.mark.parametrize("Mtok,O,I", [(1176, 256, 256), (168, 32, 256), (1176, 2048, 256), (1176, 128, 256)])
def test_dw_ragged_splitk(cuda, Mtok, O, I):
    """Weight gradient over a ragged token count (P*7 rows): 64-row split-K chunks, the last chunk's tail
    zero-filled by the k-major loaders (k_total), fixed-order combine."""
    from dilabhelmholtzoct_amd.decoder import MaskDecoder
    g = torch.Generator().manual_seed(Mtok + O)
    dy = torch.randn(Mtok, O, generator=g).to(cuda, torch.bfloat16)
    x = torch.randn(Mtok, I, generator=g).to(cuda, torch.bfloat16)
    out = torch.empty(O, I, device=cuda)
    split, ks = MaskDecoder._pick_split(Mtok, O, I)
    assert split * ks >= Mtok and (split - 1) * ks < Mtok and ks % 64 == 0
    MaskDecoder._dw(MaskDecoder, dy, x, Mtok, out)
    ref = dy.float().t() @ x.float()
    assert _rel(out, ref) < 1e-5


@pytest.mark.parametrize("Mrows,O,I,ragged", [(32768, 384, 256, False), (65536 + 640, 256, 128, True),
                                               (32768, 128, 256, False), (24576, 200, 136, True)])
@pytest.mark.parametrize("f16", [False, True])
def test_dw_fused_colsums(cuda, Mrows, O, I, ragged, f16):
    """Weight gradient with the bias gradients fused (a_colsum = sum_m dy[m, o], b_colsum = sum_m x[m, i]):
    dW unchanged bit for bit against the same GEMM without them, the sums against fp32 column sums of the same
    16-bit values (incl. a split-K tail zero-filled through k_total, ragged O / I, both 16-bit types)."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    dt = torch.float16 if f16 else torch.bfloat16
    g = torch.Generator().manual_seed(Mrows + O + I + f16)
    dy = torch.randn(Mrows, O, generator=g).to(cuda, dt)
    x = torch.randn(Mrows, I, generator=g).to(cuda, dt)
    ks = 512 if not ragged else 576
    split = -(-Mrows // ks)
    kt = Mrows if split * ks != Mrows else 0
    if kt:  # the operands must hold split * ks rows; the tail rows are never read
        pad = split * ks - Mrows
        dy = torch.cat([dy, torch.full((pad, O), float("nan"), device=cuda, dtype=dt)])
        x = torch.cat([x, torch.full((pad, I), float("nan"), device=cuda, dtype=dt)])
    outs, paths = [], []
    pa = torch.empty(split, O, device=cuda)
    pb = torch.empty(split, I, device=cuda)
    for cs in (False, True):
        part = torch.empty(split, O, I, device=cuda)
        kernels.gemm(dy, x, M=O, N=I, K=ks, out=part, a_mode=1, b_mode=1, lda=O, ldb=I, batch=split,
                     stride_a=ks * O, stride_b=ks * I, stride_c=O * I, k_total=kt,
                     a_colsum=pa if cs else None, b_colsum=pb if cs else None)
        paths.append(lib.octsam_gemm_last_path())
        outs.append(part)
    assert paths[1] == 1  # the sums force the LDS-DMA k-major kernel (few tiles would take the small path)
    if paths[0] == 1:
        assert torch.equal(outs[0], outs[1])
    else:
        assert _rel(outs[1], outs[0]) < 1e-5
    ref_a = dy[:Mrows].float().sum(0)
    ref_b = x[:Mrows].float().sum(0)
    assert _rel(pa.sum(0), ref_a) < 1e-5 and _rel(pb.sum(0), ref_b) < 1e-5
    per_split = dy[:Mrows].float()
    assert _rel(pa[0], per_split[:ks].sum(0)) < 1e-5


def test_dw_colsum_needs_kmajor_path(cuda):
    from dilabhelmholtzoct_amd import kernels
    from dilabhelmholtzoct_amd._lib import OctsamError
    A = torch.randn(256, 256, device=cuda).to(torch.bfloat16)
    out = torch.empty(256, 256, device=cuda)
    with pytest.raises(OctsamError, match="a_mode = b_mode = 1"):
        kernels.gemm(A, A, M=256, N=256, K=256, out=out, a_colsum=torch.empty(256, device=cuda))


@pytest.mark.parametrize("a_mode,b_mode", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("shape", [(1120, 256, 256, 1), (160, 32, 256, 1), (256, 256, 64, 18), (72, 200, 136, 3)])
def test_gemm_small_path(cuda, a_mode, b_mode, shape):
    """Small problems (token-side decoder GEMMs, split-K weight gradients) on the 64x64-tile kernel: every
    operand mode, batches, bias/ReLU/fp32 residual epilogue, against torch fp32."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    M, N, K, Bt = shape
    g = torch.Generator().manual_seed(M * 3 + N + K + a_mode * 5 + b_mode)
    A = torch.randn(Bt, M, K, generator=g).to(torch.bfloat16)
    W = torch.randn(Bt, N, K, generator=g).to(torch.bfloat16)
    Aop = (A if a_mode == 0 else A.transpose(1, 2)).contiguous().to(cuda)
    Bop = (W if b_mode == 0 else W.transpose(1, 2)).contiguous().to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(Bt, M, N, generator=g).to(cuda)
    out = torch.empty(Bt, M, N, device=cuda, dtype=torch.float32)
    kernels.gemm(Aop, Bop, M=M, N=N, K=K, out=out, a_mode=a_mode, b_mode=b_mode, batch=Bt, stride_a=M * K,
                 stride_b=N * K, stride_c=M * N, stride_r=M * N, bias=bias, act=1, residual=R)
    assert lib.octsam_gemm_last_path() == 3
    ref = F.relu(torch.bmm(A.float(), W.float().transpose(1, 2)).to(cuda) + bias) + R
    assert _rel(out, ref) < 1e-5


@pytest.mark.parametrize("M,N,K,kind,act", [
    (32768, 768, 3072, "f32_res", 0),    # vit-b MLP2: x += A W^T + b on the fp32 residual stream (LDS-staged residual)
    (32768, 2304, 768, "e16", 0),        # QKV
    (32768, 3072, 768, "e16", 2),        # MLP1 with the exact-erf GELU
    (16384, 1024, 4096, "f32_res", 0),   # vit-l MLP2
    (5000, 520, 192, "f32_res", 0),      # ragged M and N
    (9000, 392, 320, "e16", 2),          # ragged, GELU
    (4500, 768, 128, "f32", 0),          # fp32 C, two K-steps
    (8192, 768, 768, "f32_res_rowmap", 0),
    (16384, 384, 256, "e16", 0),         # 256x192 tiles: N = 384 as two 192-column tiles
    (8000, 768, 256, "f32_res", 0),      # 256x192 tiles, ragged M, register residual epilogue
    (8192, 576, 320, "e16", 2)])         # 256x192 tiles with GELU
def test_gemm8w_pingpong(cuda, M, N, K, kind, act):
    """The ping-pong 8-wave GEMM (gemm8w: two segments per K-step, the wave rows one segment apart; octsam_gemm's
    default for the 256x256-tile shapes, fast path bit 8192 = the 8-phase gemm8 instead; fast path bit 262144 = its
    opt-in 256x192-tile form where 256-column tiles quantise badly — MLP2, QKV, N = 384 / 576 here):
    against torch fp32, bit-identical to the 8-phase kernel and across tile widths (all chain the same 16x16x32 MFMAs
    over K in the same order) and run to run; the encoder's kinds (vit-b / vit-l shapes) and ragged tiles, the
    row-mapped residual kind."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + act)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    b = torch.randn(N, generator=g).to(cuda)
    X0 = torch.randn(M + 300, N, generator=g).to(cuda)
    rmap = None
    if kind == "f32_res_rowmap":  # rows scattered to a permutation of M + 300 rows, every 7th row dropped
        perm = torch.randperm(M + 300, generator=g)[:M].to(torch.int32)
        perm[::7] = -1
        rmap = perm.to(cuda)
    outs = []
    for fast in (1, 1, 1 | 8192, 1 | 262144):
        lib.octsam_gemm_set_fast_path(fast | 256)
        if kind == "e16":
            out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
            kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=b, act=act)
        elif kind == "f32":
            out = torch.empty(M, N, device=cuda)
            kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=b, act=act)
        elif kind == "f32_res":
            out = X0[:M].clone()
            kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=b, residual=out, act=act)
        else:
            out = X0.clone()
            kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=b, residual=out, row_map=rmap, act=act)
        assert lib.octsam_gemm_last_path() == 2
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    y = A.float() @ W.float().t() + b
    if act == 2:
        y = F.gelu(y)
    if kind == "f32_res":
        ref = y + X0[:M]
    elif kind == "f32_res_rowmap":
        ref = X0.clone()
        keep = rmap >= 0
        ref[rmap[keep].long()] += y[keep]
    else:
        ref = y
    assert _rel(outs[0], ref) < (8e-3 if kind == "e16" else 1e-5)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])
    assert torch.equal(outs[0], outs[3])


@pytest.mark.parametrize("am,bm", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1176, 256, 256), (1176, 2048, 128), (168, 256, 64), (304, 72, 200)])
def test_gemm_small_oneshot_matches_chained(cuda, am, bm, M, N, K):
    """The one-shot K <= 256 small-problem kernel (gemm_small_kernel, default) is bit-identical to the chained 64x64
    kernel it replaces (fast path bit 65536) and matches torch fp32."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + am * 2 + bm)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    Aop = A if am == 0 else A.t().contiguous()
    Bop = W if bm == 0 else W.t().contiguous()
    b = torch.randn(N, generator=g).to(cuda)
    outs = []
    for fast in (1, 1 | 65536):
        lib.octsam_gemm_set_fast_path(fast)
        out = torch.empty(M, N, device=cuda)
        kernels.gemm(Aop, Bop, M=M, N=N, K=K, out=out, a_mode=am, b_mode=bm, bias=b)
        assert lib.octsam_gemm_last_path() == 3
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    assert _rel(outs[0], A.float() @ W.float().t() + b) < 1e-5
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("b_mode", [0, 1])
@pytest.mark.parametrize("kind", ["bias_f32", "relu_b16", "beta_acc", "residual"])
@pytest.mark.parametrize("M,N,K", [(1176, 256, 256), (1176, 256, 2048), (1176, 2048, 256)])
def test_gemm_token_side(cuda, M, N, K, b_mode, kind):
    """The decoder's token-side GEMMs (M = prompts x 7 tokens) on the hand-written small-problem kernel (path 3):
    NT and k-major weights, fp32 D + bias, bf16 D + bias + ReLU, beta = 1 accumulation into D, a separate fp32
    residual; against torch fp32 and bit-identical run to run."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N * 3 + K * 7 + b_mode + len(kind))
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    Bop = W if b_mode == 0 else W.t().contiguous()
    b = torch.randn(N, generator=g).to(cuda)
    D0 = torch.randn(M, N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda)
    pre = A.float() @ W.float().t()
    outs = []
    for _ in range(2):
        if kind == "bias_f32":
            out = torch.empty(M, N, device=cuda)
            kernels.gemm(A, Bop, M=M, N=N, K=K, out=out, b_mode=b_mode, bias=b)
            ref, tol = pre + b, 1e-5
        elif kind == "relu_b16":
            out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
            kernels.gemm(A, Bop, M=M, N=N, K=K, out=out, b_mode=b_mode, bias=b, act=1)
            ref, tol = F.relu(pre + b), 8e-3
        elif kind == "beta_acc":
            out = D0.clone()
            kernels.gemm(A, Bop, M=M, N=N, K=K, out=out, b_mode=b_mode, beta=1.0)
            ref, tol = pre + D0, 1e-5
        else:
            out = torch.empty(M, N, device=cuda)
            kernels.gemm(A, Bop, M=M, N=N, K=K, out=out, b_mode=b_mode, bias=b, residual=R)
            ref, tol = pre + b + R, 1e-5
        assert lib.octsam_gemm_last_path() == 3
        outs.append(out)
    assert _rel(outs[0], ref) < tol
    assert torch.equal(outs[0], outs[1])


def test_gemm_small_path_ktotal(cuda):
    """Split-K with a ragged total (k_total): rows past k_total read as zero on the small-problem path."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    rows, O, I, ks = 1130, 256, 128, 64
    splits = -(-rows // ks)
    g = torch.Generator().manual_seed(11)
    dy = torch.randn(splits * ks, O, generator=g)
    x = torch.randn(splits * ks, I, generator=g)
    dy[rows:] = float("nan")  # must never be read
    x[rows:] = float("nan")
    dyb, xb = dy.to(cuda, torch.bfloat16), x.to(cuda, torch.bfloat16)
    part = torch.empty(splits, O, I, device=cuda)
    kernels.gemm(dyb, xb, M=O, N=I, K=ks, out=part, a_mode=1, b_mode=1, lda=O, ldb=I, batch=splits,
                 stride_a=ks * O, stride_b=ks * I, stride_c=O * I, k_total=rows)
    assert lib.octsam_gemm_last_path() == 3
    ref = dyb[:rows].float().t() @ xb[:rows].float()
    assert _rel(part.sum(0), ref) < 1e-5


# ------------------------------------------------------------------ fp16 operands (octsam_gemm_f16)
@pytest.mark.parametrize("M,N,K,res16", [(300, 200, 136, False), (4096, 768, 768, False), (8192, 3840, 1280, True),
                                          (32768, 1280, 5120, False), (7, 40, 256, True)])
def test_gemm_f16_encoder_paths(cuda, M, N, K, res16):
    """The fp16 encoder's NT GEMMs (small 64-tile path, persistent LDS-DMA kernel, 8-phase kernel with the
    register epilogue; fp32 or fp16 residual, GELU, fp16 / fp32 outputs) vs fp32 on the same fp16 operands.
    fp16 keeps 11 significant bits: fp16 outputs are checked at 2e-3, fp32 outputs at 1e-5."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = (0.5 * torch.randn(M, K, generator=g)).to(cuda, torch.float16)
    W = (0.5 * torch.randn(N, K, generator=g)).to(cuda, torch.float16)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda, torch.float16 if res16 else torch.float32)
    ref_pre = A.float() @ W.float().t() + bias
    out32 = torch.empty(M, N, device=cuda)
    kernels.gemm(A, W, M=M, N=N, K=K, out=out32, bias=bias, residual=R)
    assert _rel(out32, ref_pre + R.float()) < (2e-3 if res16 else 1e-5)
    out16 = torch.empty(M, N, device=cuda, dtype=torch.float16)
    kernels.gemm(A, W, M=M, N=N, K=K, out=out16, bias=bias, act=2)
    assert _rel(out16, F.gelu(ref_pre)) < 2e-3


def test_gemm_f16_conv3x3_and_mixed_types_rejected(cuda):
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(8)
    C = 256
    x = (0.5 * torch.randn(1, 64, 64, C, generator=g)).to(cuda, torch.float16)
    w = (0.05 * torch.randn(C, C, 3, 3, generator=g)).to(cuda)
    wk = w.permute(0, 2, 3, 1).reshape(C, 9 * C).to(torch.float16)
    out = torch.empty(4096, C, device=cuda)
    kernels.gemm(x.reshape(4096, C), wk, M=4096, N=C, K=9 * C, out=out, a_mode=3, conv_c=C)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wk.float().reshape(C, 3, 3, C).permute(0, 3, 1, 2), padding=1)
    assert _rel(out, ref.permute(0, 2, 3, 1).reshape(4096, C)) < 1e-5
    with pytest.raises(ValueError):
        kernels.gemm(x.reshape(4096, C).to(torch.bfloat16), wk, M=4096, N=C, K=9 * C, out=out, a_mode=3, conv_c=C)


def test_fp16_encoder_pieces(cuda):
    """patchify, LayerNorm and the fp32 -> 16-bit cast with fp16 outputs."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(9)
    px = torch.randn(1, 3, 1024, 1024, generator=g).to(cuda)
    out = torch.empty(4096, 768, device=cuda, dtype=torch.float16)
    kernels.patchify_bf16(px, out)
    ref = px.view(1, 3, 64, 16, 64, 16).permute(0, 2, 4, 1, 3, 5).reshape(4096, 768).to(torch.float16)
    assert torch.equal(out, ref)
    x = torch.randn(1000, 1280, generator=g).to(cuda)
    w, b = torch.randn(1280, generator=g).to(cuda), torch.randn(1280, generator=g).to(cuda)
    y = torch.empty(1000, 1280, device=cuda, dtype=torch.float16)
    kernels.layernorm_fwd(x, w, b, 1e-6, y)
    assert _rel(y, F.layer_norm(x, (1280,), w, b, 1e-6)) < 1e-3
    c = torch.empty(1000, 1280, device=cuda, dtype=torch.float16)
    kernels.cast_bf16(x, c)
    assert torch.equal(c, x.to(torch.float16))


@pytest.mark.parametrize("n", [32768 * 768, 4096 * 8 + 8, 1000 * 8, 37, 8 * 3 + 5])
def test_cast_vectorized(cuda, n):
    """fp32 -> bf16 / fp16 casts: the 8-per-thread kernel (n % 8 == 0, aligned) and the scalar fallback
    (ragged n, offset views) round exactly like torch's casts, special values included."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(n % 1000)
    x = (torch.randn(n + 1, generator=g) * 100).to(cuda)
    x[:4] = torch.tensor([float("inf"), -0.0, 1e-40, 65519.0])
    for dt in (torch.bfloat16, torch.float16):
        for src in (x[:n], x[1:n + 1]):  # aligned, and 4-B offset (scalar path)
            out = torch.empty(n, device=cuda, dtype=dt)
            kernels.cast_bf16(src, out)
            assert torch.equal(out, src.to(dt))


@pytest.mark.parametrize("M,O,I,ldy_pad,ldx_pad,db,fold,beta", [
    (688128, 384, 256, 0, 0, True, 0, 0.0),    # the bench's K|Q'|V dW (P = 168 prompts)
    (70000, 384, 128, 8, 0, True, 1, 0.0),     # ragged rows (not a multiple of 32 x workgroups), strided dY
    (65536, 256, 256, 0, 128, False, 4, 0.0),  # ConvT1: bias of x folded over 4 taps, strided X
    (100003, 256, 128, 0, 0, True, 0, 1.0),    # accumulate into out
    (66000, 128, 256, 0, 0, False, 0, 0.0),
    (2000, 128, 128, 0, 0, True, 2, 0.0),      # fewer rows than workgroups x 32
])
def test_wgrad(cuda, M, O, I, ldy_pad, ldx_pad, db, fold, beta):
    """octsam_wgrad (image-side dW = dY^T X, whole output per workgroup) vs torch fp32 on the same bf16 operands,
    with the fused bias column sums; fixed-order combine: bitwise repeatable."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(M + O + I)
    ldy, ldx = O + ldy_pad, I + ldx_pad
    dy = torch.randn(M, ldy, generator=g).to(cuda, torch.bfloat16)
    x = torch.randn(M, ldx, generator=g).to(cuda, torch.bfloat16)
    out0 = torch.randn(O, I, generator=g).to(cuda)
    out = out0.clone()
    gdb = torch.empty(O, device=cuda) if db else None
    gdbx = torch.empty(I // max(fold, 1), device=cuda) if fold else None
    kernels.wgrad(dy, x, M, out, ldy=ldy, ldx=ldx, beta=beta, db=gdb, dbx=gdbx, dbx_fold=max(fold, 1))
    ref = dy[:, :O].float().t() @ x[:, :I].float() + beta * out0
    assert _rel(out, ref) < 1e-5
    if db:
        assert _rel(gdb, dy[:, :O].float().sum(0)) < 1e-5
    if fold:
        assert _rel(gdbx, x[:, :I].float().sum(0).view(fold, -1).sum(0)) < 1e-5
    again = out0.clone()
    kernels.wgrad(dy, x, M, again, ldy=ldy, ldx=ldx, beta=beta, db=None, dbx=None)
    assert torch.equal(again, out)


def test_wgrad_rejects_unsupported(cuda):
    from dilabhelmholtzoct_amd import kernels
    from dilabhelmholtzoct_amd._lib import OctsamError
    assert not kernels.wgrad_supported(1000, 192, 256)
    dy = torch.zeros(1000, 192, device=cuda, dtype=torch.bfloat16)
    x = torch.zeros(1000, 256, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(OctsamError):
        kernels.wgrad(dy, x, 1000, torch.empty(192, 256, device=cuda))


@pytest.mark.parametrize("M,O,I,ldy_pad,ldx_pad,db,beta", [
    (1176, 256, 256, 0, 0, True, 0.0),    # P*7 token rows (P = 168)
    (1176, 128, 256, 128, 0, True, 1.0),  # strided dY (a column slice), accumulate
    (168, 256, 256, 0, 1536, True, 0.0),  # hypernetwork MLP rows (P), X a slice of [P, T*C]
    (1176, 2048, 256, 0, 0, True, 0.0),   # MLP lin1
    (1176, 256, 2048, 0, 0, False, 0.0),  # MLP lin2
    (1, 64, 32, 0, 0, True, 0.0),
    (100, 32, 96, 8, 8, True, 1.0),       # fewer rows than waves x 32
    (5000, 96, 64, 0, 0, True, 0.0),
])
def test_wgrad_tok(cuda, M, O, I, ldy_pad, ldx_pad, db, beta):
    """octsam_wgrad_tok (token-side dW = dY^T X + bias column sums, one launch) vs torch fp32 on the same bf16
    operands; the fixed-order combine is bitwise repeatable."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(M + O + I + ldx_pad)
    ldy, ldx = O + ldy_pad, I + ldx_pad
    dy = torch.randn(M, ldy, generator=g).to(cuda, torch.bfloat16)
    x = torch.randn(M, ldx, generator=g).to(cuda, torch.bfloat16)
    out0 = torch.randn(O, I, generator=g).to(cuda)
    out = out0.clone()
    gdb = torch.full((O,), 7.0, device=cuda) if db else None
    kernels.wgrad_tok(dy, x, M, out, ldy=ldy, ldx=ldx, beta=beta, db=gdb)
    ref = dy[:, :O].float().t() @ x[:, :I].float() + beta * out0
    assert _rel(out, ref) < 1e-5
    if db:
        assert _rel(gdb, dy[:, :O].float().sum(0)) < 1e-5
    again = out0.clone()
    kernels.wgrad_tok(dy, x, M, again, ldy=ldy, ldx=ldx, beta=beta)
    assert torch.equal(again, out)


@pytest.mark.parametrize("N", [384, 640])
def test_gemm4w_broadcast_residual(cuda, N):
    """The row-remapped broadcast-addend kind (the decoder's [K | Q' | V] projection of the per-prompt keys plus the
    positional projection) on the two-workgroup 256x128 kernel (N not a multiple of 256) against torch fp32 and
    bit-identical to the persistent 8-phase kernel (fast path bit 1024)."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    L, P, K = 4096, 3, 256
    M = L * P
    g = torch.Generator().manual_seed(N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(L, N, generator=g).to(cuda, torch.bfloat16)
    outs = []
    for fast in (1, 1 | 1024):
        lib.octsam_gemm_set_fast_path(fast)
        out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=bias, residual=R, ldr=N, r_remap=(L, P))
        assert lib.octsam_gemm_last_path() == 2
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    ref = A.float() @ W.float().t() + bias + R.float().repeat(P, 1)
    assert _rel(outs[0], ref) < 5e-3
    assert torch.equal(outs[0], outs[1])


def test_gemm8_f32_broadcast_residual_under_e16(cuda):
    """Lean kind 27 (e16 C + a broadcast fp32 residual: the first two-way block's image-side out_proj, whose keys
    residual is the fp32 image embedding shared by the image's prompts) against torch fp32 and bit-identical to the
    general register epilogue it replaces (fast path 18)."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    L, B, rep, N, K = 4096, 2, 3, 256, 128
    M = L * B * rep
    g = torch.Generator().manual_seed(27)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(B * L, N, generator=g).to(cuda)
    outs = []
    for fast in (1, 18):
        lib.octsam_gemm_set_fast_path(fast)
        out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=bias, residual=R, ldr=N, r_remap=(L, rep))
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    ref = A.float() @ W.float().t() + bias + R.view(B, 1, L, N).expand(B, rep, L, N).reshape(M, N)
    assert _rel(outs[0], ref) < 5e-3
    assert torch.equal(outs[0], outs[1])


def test_gemm4w_patch_embed_kind(cuda):
    """The patch embedding's GEMM (fp32 encoder stream out, bias, the positional table as a periodic fp32 addend:
    lean kind 12) on the two-workgroup kernel against torch fp32 and bit-identical to the 8-phase kernel's general
    register epilogue (fast path bit 1024); timed for the record."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    L, B, N, K = 4096, 8, 768, 768
    M = L * B
    g = torch.Generator().manual_seed(12)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    pos = torch.randn(L, N, generator=g).to(cuda)
    outs = []
    for fast in (1, 1 | 1024):
        lib.octsam_gemm_set_fast_path(fast)
        out = torch.empty(M, N, device=cuda, dtype=torch.float32)
        kernels.gemm(A, W, M=M, N=N, K=K, out=out, bias=bias, residual=pos, r_remap=(L, B))
        assert lib.octsam_gemm_last_path() == 2
        outs.append(out)
    lib.octsam_gemm_set_fast_path(1)
    ref = A.float() @ W.float().t() + bias + pos.repeat(B, 1)
    assert _rel(outs[0], ref) < 5e-3
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("C", [256, 64])
def test_gemm4w_conv3x3(cuda, C):
    """The neck's conv3x3 (implicit GEMM over NHWC 64x64 images, zero padding through the zero row) on the
    two-workgroup kernel against torch fp32 conv2d and the generic register-staged path (fast path bit 1024)."""
    from dilabhelmholtzoct_amd import _lib, kernels
    lib = _lib.load()
    g = torch.Generator().manual_seed(C)
    B, Co = 2, 256
    x = torch.randn(B, 64, 64, C, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(Co, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(cuda, torch.bfloat16)
    Wr = W.permute(0, 2, 3, 1).reshape(Co, 9 * C).contiguous()
    outs = []
    for fast in (1, 1 | 1024):
        lib.octsam_gemm_set_fast_path(fast)
        out = torch.empty(B * 4096, Co, device=cuda)
        kernels.gemm(x, Wr, M=B * 4096, N=Co, K=9 * C, out=out, a_mode=3, conv_c=C)
        outs.append((out, lib.octsam_gemm_last_path()))
    lib.octsam_gemm_set_fast_path(1)
    assert outs[0][1] == 2 and outs[1][1] == 0
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), W.float(), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    for out, _ in outs:
        assert _rel(out, ref) < 1e-5


def test_wgrad_tok_group_matches_single_launches(cuda):
    """octsam_wgrad_tok_group (ABI 22): several token-side weight gradients in one launch -- the decoder backward's
    deferred form -- give the same bits as one octsam_wgrad_tok launch each (strided dy, with and without bias
    sums, beta 0 and 1, M on both sides of the single-launch kernel's 8-wave threshold)."""
    from dilabhelmholtzoct_amd import kernels
    g = torch.Generator().manual_seed(7)
    probs, refs = [], []
    for k, (M, O, I, ldy, db, beta) in enumerate([(1176, 256, 256, 256, True, 0.0), (1176, 128, 256, 384, True, 1.0),
                                                  (700, 256, 2048, 256, False, 0.0), (4096, 256, 128, 512, True, 0.0),
                                                  (147, 32, 64, 40, True, 0.0)]):
        dy = (torch.randn(M, ldy, generator=g) * 0.1).to(cuda, torch.bfloat16)
        x = torch.randn(M, I, generator=g).to(cuda, torch.bfloat16)
        out0 = torch.randn(O, I, generator=g).to(cuda)
        outs = [out0.clone(), out0.clone()]
        dbs = [torch.empty(O, device=cuda), torch.empty(O, device=cuda)] if db else [None, None]
        kernels.wgrad_tok(dy, x, M, outs[0], ldy=ldy, beta=beta, db=dbs[0])
        probs.append((dy, x, M, outs[1], ldy, None, beta, dbs[1]))
        refs.append((outs, dbs, dy, x, M, O, beta, out0))
    kernels.wgrad_tok_group(probs)
    torch.cuda.synchronize()
    for outs, dbs, dy, x, M, O, beta, out0 in refs:
        assert torch.equal(outs[0], outs[1])
        if dbs[0] is not None:
            assert torch.equal(dbs[0], dbs[1])
        ref = dy[:, :O].float().t() @ x.float() + beta * out0
        assert _rel(outs[1], ref) < 1e-5
