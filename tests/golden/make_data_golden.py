#!/usr/bin/env python3
"""Generates tests/golden/data_golden.npz from the REFERENCE's own data path
(ref:octsam/models/training_utils.py:381-458, SAMDataset.get_bboxes_and_gt_masks /
get_points_and_gt_masks / custom_collate), imported from /root/reference with its third-party
imports stubbed (wandb, monai, cv2, evaluate, albumentations, topological_loss: none of them is used by
these functions). Run in the build container only; the fixture (data, not code) is
committed and travels, the reference does not.

Inputs: 3 seeded label maps from dilabhelmholtzoct_amd.data.synthetic_label (stored in the fixture, so
the test does not depend on the generator), np.random / random seeded per item before __getitem__.
"""
import importlib.util
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/octsam/models/training_utils.py"
SEEDS = (11, 12, 13)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.util.spec_from_loader(name, loader=None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def load_reference():
    import transformers  # noqa: F401  (must precede the stubs)
    for n in ("wandb", "monai", "cv2", "evaluate", "albumentations"):
        _stub(n)
    _stub("topological_loss", topo_loss=None)
    spec = importlib.util.spec_from_file_location("ref_training_utils", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def labels():
    sys.path.insert(0, ROOT)
    from dilabhelmholtzoct_amd.data import synthetic_label
    rng = np.random.RandomState(2024)
    return np.stack([synthetic_label(rng, H=160, W=192, n_disks=3) for _ in SEEDS])


def main():
    ref = load_reference()
    labs = labels()
    data = [{"image": np.repeat((lab * 18)[:, :, None], 3, 2).astype(np.uint8), "label": lab} for lab in labs]
    out = {"labels": labs, "seeds": np.asarray(SEEDS)}
    for prompt in ("bboxes", "points"):
        ds = ref.SAMDataset(data, {"pseudocolor": None, "prompt_type": prompt})
        items = []
        for i, s in enumerate(SEEDS):
            np.random.seed(s)
            random.seed(s)
            items.append(ds[i])
        images, pr, gt, mv = ref.custom_collate(items)
        out[f"{prompt}_prompt"] = pr.numpy()
        out[f"{prompt}_gt_bits"] = np.packbits(gt.numpy().astype(np.uint8), axis=-1)
        out[f"{prompt}_gt_shape"] = np.asarray(gt.shape)
        out[f"{prompt}_gt_dtype"] = np.asarray(str(gt.dtype))
        out[f"{prompt}_mask_values"] = mv.numpy()
        out[f"{prompt}_images"] = images.numpy()[:, ::8, ::8]  # spot check of the image stack
    np.savez_compressed(os.path.join(HERE, "data_golden.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
