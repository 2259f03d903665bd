"""Cubical persistence: the HIP kernel must be BIT-EXACT (same pixel pairs, same order) with the
CPU restatement oracle/cubical_ph.c, which is itself pinned against a brute-force boundary-matrix
reduction in tests/test_oracle_ph.py."""
import numpy as np
import pytest
import torch

from oracle.ph_ref import ph_oracle

pytestmark = pytest.mark.gpu


def _maps(n, H, W, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = i % 5
        if k == 0:
            m = rng.random((H, W))
        elif k == 1:
            m = rng.integers(0, 4, (H, W)).astype(np.float64)
        elif k == 2:
            yy, xx = np.mgrid[0:H, 0:W]
            m = np.sin(xx / 3.0) * np.cos(yy / 4.0) + 0.05 * rng.random((H, W))
        elif k == 3:
            m = (rng.random((H, W)) > 0.6).astype(np.float64)
        else:
            m = np.zeros((H, W))
        out.append(m.astype(np.float32))
    return np.stack(out)


def _check(maps, cuda, max_pairs=2048):
    from dilabhelmholtzoct_amd import kernels
    p0, p1, ess, cnt = kernels.cubical_ph(torch.from_numpy(maps).to(cuda), max_pairs=max_pairs)
    p0, p1, ess, cnt = p0.cpu().numpy(), p1.cpu().numpy(), ess.cpu().numpy(), cnt.cpu().numpy()
    for i, m in enumerate(maps):
        ref = ph_oracle(m, max_pairs=max_pairs)
        assert cnt[i, 2] == 0
        got0 = [tuple(map(int, r)) for r in p0[i, : cnt[i, 0]]]
        got1 = [tuple(map(int, r)) for r in p1[i, : cnt[i, 1]]]
        assert got0 == ref["h0"], f"map {i} H0"
        assert got1 == ref["h1"], f"map {i} H1"
        assert tuple(map(int, ess[i])) == ref["essential"], f"map {i} essential"


@pytest.mark.parametrize("H,W", [(50, 50), (7, 9), (1, 5), (64, 63), (13, 1)])
def test_ph_bitexact(cuda, H, W):
    _check(_maps(10, H, W, H * 100 + W), cuda)


def test_ph_sigmoid_like(cuda):
    rng = np.random.default_rng(11)
    logits = rng.normal(0, 20, (16, 50, 50)).astype(np.float32)
    maps = (1 / (1 + np.exp(-logits))).astype(np.float32)  # many exact 0.0 / 1.0 ties
    _check(maps, cuda)


def test_ph_deterministic(cuda):
    from dilabhelmholtzoct_amd import kernels
    maps = torch.from_numpy(_maps(8, 50, 50, 3)).to(cuda)
    a = kernels.cubical_ph(maps)
    b = kernels.cubical_ph(maps)
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])
    cnt = a[3].cpu()
    for i in range(maps.shape[0]):
        assert torch.equal(a[0][i, : cnt[i, 0]], b[0][i, : cnt[i, 0]])
        assert torch.equal(a[1][i, : cnt[i, 1]], b[1][i, : cnt[i, 1]])


def _adversarial(H, W):
    """Maps at the pair-count bounds: a checkerboard (one H1 hole per interior high pixel: ~H*W/2 pairs),
    isolated minima on the even lattice (ceil(H/2)*ceil(W/2) H0 classes) and a sigmoid-saturated
    checkerboard with exact 0/1 plateaus."""
    yy, xx = np.mgrid[0:H, 0:W]
    cb = ((yy + xx) % 2).astype(np.float32)
    minima = np.where((yy % 2 == 0) & (xx % 2 == 0), 0.0, 1.0).astype(np.float32)
    minima += (np.random.default_rng(H * W).random((H, W)) * 1e-3).astype(np.float32) * (minima > 0)
    sat = (1 / (1 + np.exp(-np.where(cb > 0, 120.0, -120.0)))).astype(np.float32)
    return np.stack([cb, minima, sat])


@pytest.mark.parametrize("H,W", [(50, 50), (64, 63), (63, 64)])
def test_ph_max_pair_counts_no_overflow(cuda, H, W):
    """Verdict r1: a 50x50 checkerboard has ~1150 H1 pairs, more than the old fixed 1024 records; the
    default buffer (kernels.ph_max_pairs) must hold every map the kernel accepts, bit-exact."""
    from dilabhelmholtzoct_amd import kernels
    maps = _adversarial(H, W)
    p0, p1, ess, cnt = (t.cpu().numpy() for t in kernels.cubical_ph(torch.from_numpy(maps).to(cuda)))
    assert p1.shape[1] == kernels.ph_max_pairs(H, W)
    for i, m in enumerate(maps):
        ref = ph_oracle(m)
        assert cnt[i, 2] == 0
        assert [tuple(map(int, r)) for r in p0[i, : cnt[i, 0]]] == ref["h0"], f"map {i} H0"
        assert [tuple(map(int, r)) for r in p1[i, : cnt[i, 1]]] == ref["h1"], f"map {i} H1"
        assert tuple(map(int, ess[i])) == ref["essential"]
    assert cnt[0, 1] > 1024 and cnt[1, 0] == ((H + 1) // 2) * ((W + 1) // 2) - 1
