"""Phase timing inside the 8-phase GEMM (diagnostics): fast path 9 runs the one-tile-per-workgroup kernel with
s_memtime stamps per workgroup (entry, main loop done, epilogue stores done) and its XCC / CU ids
(octsam_gemm_debug_stamps). For the encoder shapes this prints the median main-loop and epilogue cycles per tile,
the gap between a workgroup's end and the next workgroup's start on the same CU, and how aligned the epilogues
are across the chip (share of each XCC's CUs inside an epilogue over time). Diagnostic only."""
import ctypes
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dilabhelmholtzoct_amd import _lib, kernels as K  # noqa: E402

lib = _lib.load()
SHAPES = [("qkv", 32768, 2304, 768, 0, 0), ("fc1", 32768, 3072, 768, 2, 0), ("fc2", 32768, 768, 3072, 0, 1)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


for name, M, N, Kd, act, res in SHAPES:
    A = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    out = torch.randn(M, N, device="cuda") if res else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    R = out if res else None
    run = lambda: K.gemm(A, W, M=M, N=N, K=Kd, out=out, bias=bias, act=act, residual=R)  # noqa: E731
    lib.octsam_gemm_set_fast_path(1)
    us_default = t(run)
    lib.octsam_gemm_set_fast_path(9)
    us_stamped = t(run)
    run()
    torch.cuda.synchronize()
    nwg = ((M + 255) // 256) * ((N + 255) // 256)
    buf = np.zeros(nwg * 4, dtype=np.int64)
    assert lib.octsam_gemm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), nwg) == 0
    lib.octsam_gemm_set_fast_path(1)
    st = buf.reshape(nwg, 4)
    t0, t1, t2, ids = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
    xcc = (ids >> 32) & 0xF
    hw = ids & 0xFFFFFFFF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    slot = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    ml, ep = t1 - t0, t2 - t1
    row = {"name": name, "M": M, "N": N, "K": Kd, "wg": nwg, "us_default": round(us_default, 1),
           "us_stamped": round(us_stamped, 1), "mainloop_cyc_median": int(np.median(ml)),
           "epilogue_cyc_median": int(np.median(ep)), "epilogue_cyc_p90": int(np.percentile(ep, 90)),
           "mainloop_cyc_p90": int(np.percentile(ml, 90))}
    # per CU: gaps between consecutive workgroups, and kernel span per XCC (cycles)
    gaps, spans, busy_ml, busy_ep = [], [], [], []
    for x in np.unique(xcc):
        m = xcc == x
        spans.append(int(t2[m].max() - t0[m].min()))
        for sl in np.unique(slot[m]):
            mm = m & (slot == sl)
            o = np.argsort(t0[mm])
            a0, a2 = t0[mm][o], t2[mm][o]
            gaps += list(a0[1:] - a2[:-1])
    row["xcc_span_cyc_median"] = int(np.median(spans))
    row["cu_gap_cyc_median"] = int(np.median(gaps)) if gaps else None
    row["clock_ghz_est"] = round(statistics.median(spans) / us_stamped / 1e3, 3)
    # alignment: on XCC 0, the share of its CUs inside an epilogue, sampled at 64 points across the span
    m = xcc == np.unique(xcc)[0]
    base = t0[m].min()
    span = t2[m].max() - base
    ncu = len(np.unique(slot[m]))
    prof = []
    for i in range(48):
        tt = base + span * (i + 0.5) / 48
        inside = ((t1[m] <= tt) & (t2[m] > tt)).sum()
        prof.append(round(inside / ncu, 2))
    row["xcc0_epilogue_share_profile"] = prof
    row["xcc0_cus"] = int(ncu)
    print(json.dumps(row), flush=True)
