"""Encoder lookahead (FusedTrainStep(graphs=True, pipeline=True)): the next batch's encoder phase replays on a
side stream during this step's decoder. The frozen encoder reads no trainable weight, so losses and updated
decoder parameters must be bit-identical to the plain graph step over the same batch sequence — alternating
batches (the prefetched embedding must belong to the right batch), a wrong next_batch hint (the step must
notice and rerun its own encoder), batches with another prompt count (same pixels shape: the lookahead still
applies, the decoder graphs differ) and a batch of another pixel shape in between."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(dev, seed, B=2, epoch=0):
    from dilabhelmholtzoct_amd import data
    sd = data.SAMDataset(data.synthetic_oct(seed=seed, n=B), {"prompt_type": "bboxes"}, epoch_seed=epoch)
    b = data.custom_collate([sd[i] for i in range(B)])
    return data.to_device_batch(data.process_batch(data.make_processor(), b, "bboxes"), dev)


def _run(cuda, seq, hints, pipeline):
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
    step = FusedTrainStep(model, topological=True, graphs=True, pipeline=pipeline)
    losses = []
    for i, b in enumerate(seq):
        losses.append(step.step(b, next_batch=hints[i] if pipeline else None).clone())
    step.flush()
    torch.cuda.synchronize()
    return losses, model.mask_decoder.flat.detach().clone(), step


def test_pipeline_matches_graph_step(cuda):
    a, b = _batch(cuda, 3), _batch(cuda, 3, epoch=1)  # same scans and shape, other prompts
    assert a["gt_u8"].shape == b["gt_u8"].shape  # one graph shape: the two sets alternate
    assert not torch.equal(a["input_boxes"], b["input_boxes"])
    seq = [a, b, a, a, b, b, a]
    hints = seq[1:] + [None]
    hints[3] = a  # wrong hint: step 4 gets b, so it must rerun its own encoder
    ref_l, ref_p, _ = _run(cuda, seq, hints, False)
    got_l, got_p, st = _run(cuda, seq, hints, True)
    for x, y in zip(ref_l, got_l):
        assert torch.equal(x, y), (x, y)
    assert torch.equal(ref_p, got_p)
    assert st._enc_stream is not None  # the lookahead actually ran


def test_pipeline_other_shape_between(cuda):
    a, c = _batch(cuda, 3), _batch(cuda, 5, B=1)
    seq = [a, a, c, a, a]
    hints = seq[1:] + [None]
    ref_l, ref_p, _ = _run(cuda, seq, hints, False)
    got_l, got_p, _ = _run(cuda, seq, hints, True)
    for x, y in zip(ref_l, got_l):
        assert torch.equal(x, y), (x, y)
    assert torch.equal(ref_p, got_p)


def test_pipeline_across_prompt_counts(cuda):
    a, d = _batch(cuda, 3), _batch(cuda, 4)
    assert a["gt_u8"].shape[1] != d["gt_u8"].shape[1] and a["pixel_values"].shape == d["pixel_values"].shape
    seq = [a, d, a, d, d, a]
    hints = seq[1:] + [None]
    ref_l, ref_p, _ = _run(cuda, seq, hints, False)
    got_l, got_p, st = _run(cuda, seq, hints, True)
    for x, y in zip(ref_l, got_l):
        assert torch.equal(x, y), (x, y)
    assert torch.equal(ref_p, got_p)
    assert len(st._esets) == 2  # one encoder graph per parity, shared by both prompt counts
