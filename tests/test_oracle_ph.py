"""Pins the PH oracle (oracle/cubical_ph.c) against an independent brute-force Z/2 boundary
matrix reduction under gudhi's total order, including heavy ties (binary and integer maps)."""
import numpy as np
import pytest

from oracle.ph_ref import ph_bruteforce, ph_oracle


@pytest.mark.parametrize("seed", range(6))
def test_oracle_vs_bruteforce(seed):
    rng = np.random.default_rng(seed)
    for t in range(60):
        H, W = int(rng.integers(1, 9)), int(rng.integers(1, 9))
        kind = t % 4
        if kind == 0:
            x = rng.random((H, W))
        elif kind == 1:
            x = rng.integers(0, 3, (H, W))
        elif kind == 2:
            x = rng.random((H, W)) > 0.5
        else:
            x = np.round(rng.normal(size=(H, W)), 1)
        x = np.asarray(x, np.float32)
        assert ph_oracle(x) == ph_bruteforce(x)


def test_known_answers():
    # a ring: one H1 class born at 0 (ring), dies at 1 (hole centre)
    x = np.zeros((5, 5), np.float32)
    x[2, 2] = 1.0
    r = ph_oracle(x)
    assert r["h1"] == [(1, 12)] or len(r["h1"]) == 1 and r["h1"][0][1] == 12
    assert r["h0"] == []
    assert r["essential"][1] == 12
    # two basins -> one finite H0 pair
    y = np.array([[0, 2, 1]], np.float32)
    r = ph_oracle(y)
    assert r["h0"] == [(2, 1)]
    assert r["h1"] == []
    assert r["essential"] == (0, 1)
    # constant map: nothing finite
    r = ph_oracle(np.ones((4, 6), np.float32))
    assert r["h0"] == [] and r["h1"] == []


def test_oracle_medium_bruteforce():
    rng = np.random.default_rng(42)
    x = (rng.random((12, 11)) * 4).round().astype(np.float32)
    assert ph_oracle(x) == ph_bruteforce(x)
