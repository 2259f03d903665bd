"""The val-Dice oracle's fast host path (tests/valdice_protocol.fast_host_batches: components labelled once per
seed, uint8 gt, cached image processing) against the restated reference path it replaces (host_batches:
SAMDataset + custom_collate + SamProcessor, ref:octsam/models/training_utils.py:381-458): every tensor equal, over
two epochs (the prompt redraw) and a ragged last batch. CPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import valdice_protocol as P  # noqa: E402


def test_fast_host_batches_match_reference_path():
    for seed, n, epoch in ((2001, 10, 0), (2001, 10, 1), (3005, 8, 0)):
        ref = P.host_batches(seed, n, epoch)
        got = P.fast_host_batches(seed, n, epoch)
        assert len(ref) == len(got)
        for r, g in zip(ref, got):
            assert set(r) == set(g), (set(r), set(g))
            for k in r:
                a, b = r[k], g[k]
                assert torch.is_tensor(a) and torch.is_tensor(b), k
                assert a.dtype == b.dtype and a.shape == b.shape, (k, a.dtype, b.dtype, a.shape, b.shape)
                assert torch.equal(a, b), k
