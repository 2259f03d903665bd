"""octsam_topo_w2 (device W2 + loss + gradient) against octsam_topo_host (the host C path it
replaces in the training step): bit-identical loss and d loss / d pred values on

* synthetic diagrams: empty / tiny / large pred and gt diagrams, grouped entries ("all" mode), H0 and H1
  columns, a zero-cost entry (inf * 0 -> NaN gradient on both sides), both diagrams large (deep augmenting
  paths), and the pair-buffer sizes of 50x50 maps (LDS scratch) and 64x63 maps (global-memory scratch);
* real persistence diagrams: 50x50 sigmoid maps of random logits and gt-like binary maps through the HIP
  persistence kernel, "first" and "all" modes;
* an overflowing pair count -> NaN loss and NaN gradient rows (the host raises).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(seed, Kn, sizes, I=50, maxp=1024, dup=False):
    rng = np.random.RandomState(seed)
    pairs = np.zeros((2 * Kn, maxp, 2), np.int32)
    cnt = np.zeros((2 * Kn, 3), np.int32)
    vals = rng.rand(2 * Kn, I * I).astype(np.float32)
    if dup:  # many equal values: tied costs, tied minima in the augmenting steps
        vals = (np.round(vals * 8) / 8).astype(np.float32)
    for k, n in enumerate(sizes):
        pairs[k, :n] = rng.randint(0, I * I, (n, 2))
        cnt[k, 1] = n
        cnt[k, 0] = rng.randint(0, 5)
    return pairs, cnt, vals


def _both(pairs, cnt, vals, entries, maps, feat_d=1, want_grad=True, dev="cuda"):
    from dilabhelmholtzoct_amd.losses import topo_host, topo_w2_device
    hl, hg = topo_host(pairs, cnt, vals, entries, maps, feat_d=feat_d, want_grad=want_grad)
    dl, dg = topo_w2_device(*(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (pairs, cnt, vals)),
                            entries, maps, feat_d=feat_d, want_grad=want_grad)
    return hl, hg, float(dl.cpu()[0]), (None if dg is None else dg.cpu().numpy())


def _assert_same(hl, hg, dl, dg):
    assert dl == hl or (math.isnan(dl) and math.isnan(hl)), (dl, hl)
    if hg is None:
        assert dg is None
        return
    assert hg.shape == dg.shape
    np.testing.assert_array_equal(np.isnan(dg), np.isnan(hg))
    ok = ~np.isnan(hg)
    assert np.array_equal(dg[ok].view(np.uint32), hg[ok].view(np.uint32)), np.abs(dg[ok] - hg[ok]).max()


@pytest.mark.parametrize("mode", ["first", "all"])
@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("dup", [False, True])
def test_device_w2_matches_host_synthetic(cuda, mode, seed, dup):
    Kn = 6
    sizes = [0, 3, 40, 120, 1, 17, 0, 5, 60, 0, 2, 30]  # pred maps then gt maps
    pairs, cnt, vals = _case(seed, Kn, sizes, dup=dup)
    maps = [10 * i for i in range(Kn)]
    entries = [[m] for m in maps] if mode == "first" else [maps[:2], maps[2:5], maps[5:]]
    for feat_d in (0, 1):
        _assert_same(*_both(pairs, cnt, vals, entries, maps, feat_d=feat_d))
    _assert_same(*_both(pairs, cnt, vals, entries, maps, want_grad=False))


@pytest.mark.parametrize("maxp", [1250, 2016])
def test_device_w2_large_diagrams(cuda, maxp):
    """Both diagrams of a map large (long augmenting paths over up to 2 * 700 columns); maxp 1250 = 50x50 maps
    (scratch in LDS), 2016 = 64x63 maps (scratch in a global workspace when LDS is too small)."""
    Kn = 3
    sizes = [700, 300, 9, 650, 500, 0]
    for dup in (False, True):
        pairs, cnt, vals = _case(7, Kn, sizes, maxp=maxp, dup=dup)
        maps = [0, 1, 2]
        _assert_same(*_both(pairs, cnt, vals, [[0], [1], [2]], maps))
        _assert_same(*_both(pairs, cnt, vals, [[0, 1, 2]], maps))


def test_device_w2_zero_cost_entry_nan_gradient(cuda):
    pairs, cnt, vals = _case(3, 1, [2, 2])
    vals[1] = vals[0]
    pairs[1] = pairs[0]  # identical diagrams: cost 0, d sqrt / d cost = inf
    hl, hg, dl, dg = _both(pairs, cnt, vals, [[0]], [0])
    assert hl == dl == 0.0
    assert np.isnan(dg).any()
    _assert_same(hl, hg, dl, dg)


def test_device_w2_overflow_gives_nan(cuda):
    from dilabhelmholtzoct_amd.losses import topo_w2_device
    pairs, cnt, vals = _case(4, 1, [2, 2])
    cnt[0, 2] = 1
    loss, grad = topo_w2_device(*(torch.from_numpy(a).to(cuda) for a in (pairs, cnt, vals)), [[0]], [0])
    assert math.isnan(float(loss.cpu()[0]))
    assert bool(torch.isnan(grad).all()), "an overflowed step must not hand Adam a finite topo gradient"


@pytest.mark.parametrize("mode", ["first", "all"])
def test_device_w2_real_diagrams(cuda, mode):
    """Diagrams of the persistence kernel on 50x50 resampled maps, the training step's configuration."""
    from dilabhelmholtzoct_amd.losses import topo_device_forward, topo_index
    g = torch.Generator().manual_seed(11)
    B, N, H, W = 3, 4, 96, 100
    masks = (torch.randn(B, N, H, W, generator=g) * 4).to(cuda)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    gt = torch.zeros(B, N, H, W, dtype=torch.uint8)
    for b in range(B):
        for n in range(N):
            cy, cx, r = 20 + 10 * n, 30 + 8 * b, 12 + 3 * n
            ring = ((yy - cy) ** 2 + (xx - cx) ** 2 <= r * r) & ((yy - cy) ** 2 + (xx - cx) ** 2 >= (r // 2) ** 2)
            gt[b, n] = ring.to(torch.uint8)
    gt = gt.to(cuda)
    entries, maps, midx = topo_index(B, N, mode, None, cuda)
    pairs, cnt, vals = topo_device_forward(masks, gt, midx, interp=50)
    assert int(cnt[:, 1].max()) > 10  # non-trivial diagrams
    _assert_same(*_both(pairs.cpu().numpy(), cnt.cpu().numpy(), vals.cpu().numpy(), entries, maps))
