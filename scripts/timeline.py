#!/usr/bin/env python3
"""Occupancy of the pipelined step's timeline from a rocprofv3 kernel trace (diagnostics): over the window spanned by
the last N steps' kernels, how long the GPU ran encoder kernels only, decoder kernels only, both, or nothing, and which
decoder kernels ran ALONE longest (the ones on the step's critical path while the encoder stream was idle or waiting).
Encoder kernels are recognised by name (ViT attention, the encoder GEMM kinds, patchify, encoder LayerNorms) -- a
heuristic good enough for a profile. usage: timeline.py <dir with *kernel_trace.csv> [window_ms]"""
import collections
import csv
import glob
import os
import sys

ENC = ("vit_attn", "patchify", "ln_fwd_kernel<768>", "gemm8_kernel<0, 0, 4>", "gemm8_kernel<0, 2, 1>",
       "gemm8_kernel<0, 0, 1>", "gemm4w_kernel<0, 4, false>", "gemm4w_kernel<0, 2, true>", "ln_fwd_kernel<64>",
       "gemm4w_kernel<0, 12, false>")


def main():
    root = sys.argv[1]
    win_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
    ks = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    ks.sort()
    t_end = ks[-1][1]
    t0 = t_end - int(win_ms * 1e6)
    ks = [k for k in ks if k[1] > t0]
    ev = []
    for s, e, n in ks:
        s = max(s, t0)
        enc = any(p in n for p in ENC)
        ev.append((s, 1, enc, n))
        ev.append((e, -1, enc, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    n_enc = n_dec = 0
    running = collections.Counter()
    last = t0
    acc = collections.Counter()
    alone = collections.Counter()
    for t, d, enc, n in ev:
        dt = t - last
        if dt > 0:
            key = ("both" if n_enc and n_dec else "encoder only" if n_enc else "decoder only" if n_dec else "idle")
            acc[key] += dt
            if n_dec and not n_enc:
                for name, c in running.items():
                    if c > 0 and not any(p in name for p in ENC):
                        alone[name] += dt / max(1, sum(v > 0 for v in running.values()))
        last = t
        if enc:
            n_enc += d
        else:
            n_dec += d
        running[n] += d
    tot = sum(acc.values())
    print(f"window {tot / 1e6:.2f} ms")
    for k in ("encoder only", "both", "decoder only", "idle"):
        print(f"  {k:13s} {acc[k] / 1e6:8.3f} ms  {100 * acc[k] / tot:5.1f} %")
    print("decoder kernels running without an encoder kernel beside them (ms in the window):")
    for name, v in alone.most_common(25):
        print(f"  {v / 1e6:7.3f}  {name[:110]}")


if __name__ == "__main__":
    main()
