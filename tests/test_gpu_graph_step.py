"""hipGraph replay of the training step (FusedTrainStep(graphs=True)) against the eager step on the same
model, batch and seed: losses and the updated decoder parameters must be bit-identical (same kernels, same
order, fixed-order reductions), with and without the topological loss."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(dev, B=2):
    from dilabhelmholtzoct_amd import data
    sd = data.SAMDataset(data.synthetic_oct(seed=3, n=B), {"prompt_type": "bboxes"}, epoch_seed=0)
    b = data.custom_collate([sd[i] for i in range(B)])
    return data.to_device_batch(data.process_batch(data.make_processor(), b, "bboxes"), dev)


@pytest.mark.parametrize("top", [True, False])
def test_graph_step_matches_eager(cuda, top):
    from dilabhelmholtzoct_amd.model import SamModel
    from dilabhelmholtzoct_amd.train import FusedTrainStep
    batch = _batch(cuda)
    runs = []
    for graphs in (False, True):
        model = SamModel.from_pretrained("facebook/sam-vit-base", seed=0).to(cuda)
        step = FusedTrainStep(model, topological=top, graphs=graphs)
        losses = [step.step(batch).clone() for _ in range(3)]
        step.flush()
        torch.cuda.synchronize()
        runs.append((losses, model.mask_decoder.flat.detach().clone()))
    (le, fe), (lg, fg) = runs
    for a, b in zip(le, lg):
        assert torch.equal(a, b), (a, b)
    assert torch.equal(fe, fg)
    if top:
        assert float(lg[-1][2]) > 0.0
