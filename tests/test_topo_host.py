"""octsam_topo_host (one C call for the whole host half of topo_loss) against the per-entry Python
formulation it replaced (kept here as the checker: octsam_w2_host per map pair, numpy accumulation),
on random diagrams with empty, tiny and large pred / gt diagrams, grouped entries ("all" mode) and a
zero-cost entry (inf * 0 -> nan gradient, as torch's pow backward gives). Bit-identical loss and gradient."""
import math

import numpy as np
import pytest

from dilabhelmholtzoct_amd import kernels as K
from dilabhelmholtzoct_amd.losses import topo_host


def _reference(pairs_h, cnt_h, vals_h, entries, maps, lamda=0.1, feat_d=1, loss_q=2, want_grad=True):
    Kn = len(maps)
    col = 0 if feat_d == 0 else 1

    def diagram(k):
        n = cnt_h[k, col]
        pr = pairs_h[k, :n]
        v = vals_h[k]
        return np.stack([v[pr[:, 0]], v[pr[:, 1]]], 1) if n else np.zeros((0, 2), np.float32), pr

    pos = {m: i for i, m in enumerate(maps)}
    dpred = np.zeros((Kn, vals_h.shape[1]), np.float32) if want_grad else None
    total = 0.0
    for e in entries:
        costs, grads = [], []
        for m in e:
            k = pos[m]
            d1, pr1 = diagram(k)
            d2, _ = diagram(Kn + k)
            c, g = K.w2_host(d1, d2, float(loss_q))
            costs.append(c)
            grads.append((k, pr1, g))
        tot = float(np.float32(sum(costs)))
        # q = 2: sqrt for the 1/q power (correctly rounded, the same bits on the host and the device)
        total += math.sqrt(tot) if loss_q == 2 else tot ** (1.0 / loss_q)
        if want_grad:
            if tot > 0:
                dd = 0.5 / math.sqrt(tot) if loss_q == 2 else (1.0 / loss_q) * (tot ** (1.0 / loss_q - 1.0))
            else:
                dd = float("inf")
            for k, pr1, g in grads:
                if len(pr1) == 0:
                    continue
                scale = lamda / len(entries) * dd
                np.add.at(dpred[k], pr1[:, 0], (scale * g[:, 0]).astype(np.float32))
                np.add.at(dpred[k], pr1[:, 1], (scale * g[:, 1]).astype(np.float32))
    return lamda * total / len(entries), dpred


def _case(seed, Kn, sizes, I=50, maxp=1024):
    rng = np.random.RandomState(seed)
    pairs = np.zeros((2 * Kn, maxp, 2), np.int32)
    cnt = np.zeros((2 * Kn, 3), np.int32)
    vals = rng.rand(2 * Kn, I * I).astype(np.float32)
    for k, n in enumerate(sizes):
        pairs[k, :n] = rng.randint(0, I * I, (n, 2))
        cnt[k, 1] = n
        cnt[k, 0] = rng.randint(0, 5)
    return pairs, cnt, vals


@pytest.mark.parametrize("mode", ["first", "all"])
@pytest.mark.parametrize("seed", [0, 1])
def test_topo_host_matches_per_entry_path(mode, seed):
    Kn = 6
    sizes = [0, 3, 40, 120, 1, 17, 0, 5, 60, 0, 2, 30]  # pred maps then gt maps
    pairs, cnt, vals = _case(seed, Kn, sizes)
    maps = [10 * i for i in range(Kn)]
    entries = [[m] for m in maps] if mode == "first" else [maps[:2], maps[2:5], maps[5:]]
    for feat_d in (0, 1):
        want_l, want_g = _reference(pairs, cnt, vals, entries, maps, feat_d=feat_d)
        got_l, got_g = topo_host(pairs, cnt, vals, entries, maps, feat_d=feat_d)
        assert got_l == want_l
        np.testing.assert_array_equal(got_g, want_g)
    l_only, g_none = topo_host(pairs, cnt, vals, entries, maps, want_grad=False)
    assert g_none is None and l_only == _reference(pairs, cnt, vals, entries, maps)[0]


def test_topo_host_zero_cost_entry_gives_nan_gradient():
    pairs, cnt, vals = _case(3, 1, [2, 2])
    vals[1] = vals[0]
    pairs[1] = pairs[0]  # identical diagrams: cost 0
    want_l, want_g = _reference(pairs, cnt, vals, [[0]], [0])
    got_l, got_g = topo_host(pairs, cnt, vals, [[0]], [0])
    assert got_l == want_l == 0.0
    np.testing.assert_array_equal(np.isnan(got_g), np.isnan(want_g))


def test_topo_host_overflow_raises():
    pairs, cnt, vals = _case(4, 1, [2, 2])
    cnt[0, 2] = 1
    with pytest.raises(RuntimeError):
        topo_host(pairs, cnt, vals, [[0]], [0])


def test_topo_host_error_messages():
    """Argument errors of the host entry points set octsam_last_error."""
    from dilabhelmholtzoct_amd import _lib
    lib = _lib.load()
    pairs, cnt, vals = _case(5, 1, [2, 2])
    flat = np.array([3], np.int32)
    off = np.array([0, 1], np.int32)
    loss = np.zeros(1, np.float64)
    rc = lib.octsam_topo_host(pairs.ctypes.data, cnt.ctypes.data, vals.ctypes.data, 1, pairs.shape[1],
                              vals.shape[1], flat.ctypes.data, off.ctypes.data, 1, 1, 2.0, 0.1, 0,
                              loss.ctypes.data, None)
    assert rc == 1 and b"outside" in lib.octsam_last_error()
    cnt[1, 1] = pairs.shape[1] + 1
    flat[0] = 0
    rc = lib.octsam_topo_host(pairs.ctypes.data, cnt.ctypes.data, vals.ctypes.data, 1, pairs.shape[1],
                              vals.shape[1], flat.ctypes.data, off.ctypes.data, 1, 1, 2.0, 0.1, 0,
                              loss.ctypes.data, None)
    assert rc == 1 and b"overflow" in lib.octsam_last_error()
    cost = np.zeros(1, np.float64)
    assert lib.octsam_w2_host(None, 2, None, 0, 2.0, cost.ctypes.data, None) == 1
    assert b"octsam_w2_host" in lib.octsam_last_error()
