"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

Two independent CPU restatements of the cubical persistence used by the reference's topological
loss (ref:octsam/models/topological_loss.py:55-63 -> torch_topological CubicalComplex -> gudhi):

* ``ph_oracle``     — ctypes binding of oracle/cubical_ph.c (union-find / Alexander-dual union-find),
                      the bit-exact target of the HIP kernel.
* ``ph_bruteforce`` — pure-Python Z/2 boundary-matrix column reduction over the full cubical
                      complex under gudhi's total order (value, dimension, bitmap position); used
                      only on small maps to pin ``ph_oracle``.

Both return ``{"h0": [(creator, destroyer), ...], "h1": [...], "essential": (creator, argmax)}``
with pixel indices in C order, pairs sorted by decreasing persistence then by destroyer filtration
order (the order the HIP kernel and octsam_cubical_ph() use). Parity with gudhi itself is
UNPINNED: gudhi/torch_topological are absent and the reference ships no tests or fixtures.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "liboracle_ph.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        lib = ctypes.CDLL(path)
        lib.oracle_cubical_ph.restype = ctypes.c_int
        lib.oracle_cubical_ph.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def ph_oracle(x: np.ndarray, max_pairs: int | None = None) -> dict:
    x = np.ascontiguousarray(x, dtype=np.float32)
    H, W = x.shape
    if max_pairs is None:
        max_pairs = 2 * H * W + H + W + 1
    p0 = np.zeros((max_pairs, 2), np.int32)
    p1 = np.zeros((max_pairs, 2), np.int32)
    n0 = np.zeros(1, np.int32)
    n1 = np.zeros(1, np.int32)
    ess = np.zeros(2, np.int32)
    ovf = _lib().oracle_cubical_ph(x.ctypes.data, H, W, max_pairs, p0.ctypes.data, n0.ctypes.data,
                                   p1.ctypes.data, n1.ctypes.data, ess.ctypes.data)
    return {"h0": [tuple(map(int, r)) for r in p0[: n0[0]]],
            "h1": [tuple(map(int, r)) for r in p1[: n1[0]]],
            "essential": (int(ess[0]), int(ess[1])),
            "overflow": bool(ovf)}


# ----------------------------------------------------------------------------- brute force
def _cell_value(x, W2, H2, p):
    X, Y = p % W2, p // W2
    H, W = x.shape
    vals = []
    for dy in ((0,) if Y & 1 else (-1, 1)):
        for dx in ((0,) if X & 1 else (-1, 1)):
            XX, YY = X + dx, Y + dy
            if 0 <= XX < W2 and 0 <= YY < H2:
                vals.append(x[YY >> 1, XX >> 1])
    return min(vals)


def _top_coface(x, W2, H2, vals, p):
    W = x.shape[1]
    while True:
        X, Y = p % W2, p // W2
        if X & 1 and Y & 1:
            return (Y >> 1) * W + (X >> 1)
        v = vals[p]
        cands = []
        if not Y & 1:
            if Y > 0:
                cands.append(p - W2)
            if Y < H2 - 1:
                cands.append(p + W2)
        if not X & 1:
            if X > 0:
                cands.append(p - 1)
            if X < W2 - 1:
                cands.append(p + 1)
        nxt = next(c for c in cands if vals[c] == v)
        p = nxt


def ph_bruteforce(x: np.ndarray) -> dict:
    """Z/2 column reduction of the full boundary matrix (small maps only)."""
    x = np.asarray(x, dtype=np.float32)
    H, W = x.shape
    W2, H2 = 2 * W + 1, 2 * H + 1
    n = W2 * H2
    vals = [float(_cell_value(x, W2, H2, p)) for p in range(n)]
    dims = [((p % W2) & 1) + ((p // W2) & 1) for p in range(n)]
    order = sorted(range(n), key=lambda p: (vals[p], dims[p], p))
    rank = [0] * n
    for i, p in enumerate(order):
        rank[p] = i
    cols = []
    for p in order:
        X, Y = p % W2, p // W2
        bits = 0
        if X & 1:
            bits |= (1 << rank[p - 1]) | (1 << rank[p + 1])
        if Y & 1:
            bits |= (1 << rank[p - W2]) | (1 << rank[p + W2])
        cols.append(bits)
    low_owner = {}
    pairs = []
    for j in range(n):
        c = cols[j]
        while c:
            low = c.bit_length() - 1
            if low in low_owner:
                c ^= cols[low_owner[low]]
            else:
                low_owner[low] = j
                pairs.append((low, j))
                break
        cols[j] = c
    paired = set()
    out = {0: [], 1: []}
    for lo, hi in pairs:
        paired.add(lo)
        paired.add(hi)
        pb, pd = order[lo], order[hi]
        if vals[pd] > vals[pb]:
            d = dims[pb]
            out[d].append(((vals[pd] - vals[pb]), (vals[pd], dims[pd], pd),
                           _top_coface(x, W2, H2, vals, pb), _top_coface(x, W2, H2, vals, pd)))
    ess = [order[i] for i in range(n) if i not in paired]
    assert len(ess) == 1 and dims[ess[0]] == 0, "rectangle complex must have one essential H0 class"
    res = {}
    for d in (0, 1):
        lst = sorted(out[d], key=lambda r: (-r[0], r[1]))
        res[f"h{d}"] = [(c, dd) for _, _, c, dd in lst]
    res["essential"] = (_top_coface(x, W2, H2, vals, ess[0]), int(np.argmax(x.ravel())))
    res["overflow"] = False
    return res
