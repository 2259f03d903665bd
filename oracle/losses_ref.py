"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

CPU restatements (torch fp32/fp64, autograd) of the reference's loss path:
* ``dicece_ref``   — monai==1.3.0 DiceCELoss(sigmoid=True) (ref:environment.yml:224; called at
                     ref:octsam/models/training_utils.py:32,62). monai is absent: its published algorithm
                     is restated (DiceLoss smooth_nr = smooth_dr = 1e-5, include_background, batch=False,
                     mean reduction; nn.CrossEntropyLoss over dim 1 with probability targets; with one
                     channel that CE is 0 — monai 1.3.0 has no BCE branch). Pinned by closed-form cases
                     in tests/test_host_logic.py (no monai fixtures exist).
* ``topo_loss_ref`` — ref:octsam/models/topological_loss.py:11-96 with torch_topological's
                     CubicalComplex / batch_iter / WassersteinDistance restated (unpinned third-party
                     versions): persistence pairs from oracle/cubical_ph.c, the transport plan from
                     scipy.optimize.linear_sum_assignment on the diagonal-augmented square problem (same
                     optimum as POT's ot.emd2; plan ties may differ), cost and gradient through torch
                     autograd exactly as WassersteinDistance builds its matrix; loss_r adds
                     torch_topological.utils.total_persistence(diagram, p=q) = sum |death - birth|^q
                     averaged over the pred diagrams (topological_loss.py:88-94).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from scipy.optimize import linear_sum_assignment

from .ph_ref import ph_oracle


def dicece_ref(input: torch.Tensor, target: torch.Tensor, smooth_nr=1e-5, smooth_dr=1e-5) -> torch.Tensor:
    p = torch.sigmoid(input)
    red = tuple(range(2, input.dim()))
    inter = (target * p).sum(red)
    g = target.sum(red)
    pr = p.sum(red)
    dice = (1.0 - (2.0 * inter + smooth_nr) / (g + pr + smooth_dr)).mean()
    ce = F.cross_entropy(input, target)
    return dice + ce


def _wasserstein_ref(D1: torch.Tensor, D2: torch.Tensor, q: float) -> torch.Tensor:
    """torch_topological WassersteinDistance(q=q, p=inf) for one diagram pair: returns sum(G * M^q)."""
    n, m = len(D1), len(D2)

    def proj(D):
        s = D[:, 0] + D[:, 1]
        return 0.5 * torch.stack((s, s), 1)

    d11 = torch.linalg.vector_norm(D1 - proj(D1), float("inf"), dim=1)
    d22 = torch.linalg.vector_norm(D2 - proj(D2), float("inf"), dim=1)
    dist = torch.cdist(D1, D2, p=float("inf")) if n and m else torch.zeros((n, m), dtype=D1.dtype, device=D1.device)
    upper = torch.hstack((dist, d11[:, None]))
    lower = torch.cat((d22, torch.zeros(1, dtype=D1.dtype, device=D1.device)))
    M = torch.vstack((upper, lower)) ** q
    # plan of the EMD with a = (1,..,1,m), b = (1,..,1,n) via the equivalent square assignment
    Mn = M.detach().double().cpu().numpy()
    Nn = n + m
    if Nn == 0:
        return (M * 0).sum()
    C = np.zeros((Nn, Nn))
    C[:n, :m] = Mn[:n, :m]
    C[:n, m:] = Mn[:n, m:m + 1]
    C[n:, :m] = Mn[n:n + 1, :m]
    r, c = linear_sum_assignment(C)
    G = np.zeros((n + 1, m + 1))
    for i, j in zip(r, c):
        G[min(i, n), min(j, m)] += 1.0
    return (torch.from_numpy(G).to(M.device, M.dtype) * M).sum()


def _diagram(x2d: torch.Tensor, feat_d: int):
    res = ph_oracle(x2d.detach().cpu().numpy().astype(np.float32))
    if feat_d == 2:  # a 2-D cubical complex has no H2 pairs
        return torch.zeros((0, 2), dtype=x2d.dtype, device=x2d.device)
    # H0: gudhi's essential class paired with the argmax pixel (torch_topological CubicalComplex)
    pairs = list(res["h0"]) + [tuple(res["essential"])] if feat_d == 0 else res["h1"]
    if not pairs:
        return torch.zeros((0, 2), dtype=x2d.dtype, device=x2d.device)
    idx = torch.tensor(pairs, dtype=torch.long, device=x2d.device)
    flat = x2d.reshape(-1)
    return torch.stack((flat[idx[:, 0]], flat[idx[:, 1]]), 1)


def topo_entries(B: int, N: int, mode: str = "first"):
    if B == 1:
        return [[n] for n in range(N)]
    if N == 1:
        return [[b] for b in range(B)]
    if mode == "all":
        return [[b * N + n for n in range(N)] for b in range(B)]
    return [[b * N] for b in range(B)]


def topo_loss_ref(pred_obj, true_obj, lamda, interp=0, feat_d=2, loss_q=2, mode="first", loss_r=False):
    """pred_obj/true_obj [B, N, H, W]; see module docstring. interp=0: no resampling (:48-52)."""
    if lamda == 0.0:
        return 0.0
    if interp:
        size = (interp, interp)
        p = F.interpolate(pred_obj, size=size, mode="bilinear", align_corners=True)
        t = F.interpolate(true_obj, size=size, mode="bilinear", align_corners=True)
    else:
        p, t = pred_obj, true_obj
    B, N, H, W = p.shape
    pm = p.reshape(B * N, H, W)
    tm = t.reshape(B * N, H, W)
    vals, reg = [], []
    for e in topo_entries(B, N, mode):
        tot = 0.0
        for k in e:
            dp = _diagram(pm[k], feat_d)
            tot = tot + _wasserstein_ref(dp, _diagram(tm[k], feat_d), loss_q)
            reg.append((dp[:, 1] - dp[:, 0]).abs().pow(loss_q).sum())
        vals.append(tot ** (1.0 / loss_q))
    loss = torch.stack(vals).mean()
    if loss_r:
        loss = loss + torch.stack(reg).mean()
    return lamda * loss
