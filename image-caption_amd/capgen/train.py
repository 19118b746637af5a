"""`train()` — the training loop of main.py:25-153 over the HBM-resident input pipeline.

Cadence restated from the reference:
- every step: `MODEL.train_step` on one shuffled per-caption batch (main.py:60-67);
- every `eval_every` (100) steps: `compute_loss` on the first train and first valid batch,
  logged under `write_log` keys (main.py:69-81, WRITE_LOG of core/config.py:65-68);
- every `sample_every` (2500) steps: one greedy caption of the batch's first image next to its
  ground truths (main.py:83-102);
- per epoch: train/valid loss averaged over the zipped train/valid batches (len = the shorter
  loader, as zip() gives), greedy captions of every valid image, the candidate list written to
  `target_dir/valid.candidate.captions.pkl`, optional `evaluate(target_dir)` scores
  (main.py:104-146), and `model_{epoch}.pt` under `output_path/model/` (main.py:151).

Differences by design: batches never leave HBM (capgen.data.DeviceFeatureStore +
ResidentBatches; `train_step_resident` gathers the images inside the pack kernel), and the
TensorBoard writer / COCO evaluation (un-vendored coco-caption) are caller hooks (`log`,
`evaluate`).  The model is duck-typed: anything with the TRANSFORMER methods main.py uses.
"""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch

from .data import DeviceFeatureStore, ResidentBatches


def _gather(store, idx):
    return store.features.index_select(0, idx.long()), store.positions.index_select(0, idx.long())


def train(model, train_split, valid_split, num_epoch, batch_size, output_path, target_dir=None,
          eval_every=100, sample_every=2500, write_log=("loss",), evaluate=None, log=print,
          device="cuda:0", feature_dtype=torch.bfloat16, seed=0):
    """train_split / valid_split: dicts as returned by capgen.data.load_split (features,
    positions, captions, image_idxs).  Returns the per-epoch score dicts."""
    model_dir = os.path.join(output_path, "model")
    os.makedirs(model_dir, exist_ok=True)
    target_dir = target_dir or os.path.join(output_path, "valid")
    os.makedirs(target_dir, exist_ok=True)

    stores, loaders = {}, {}
    for name, split, shuffle in (("train", train_split, True), ("valid", valid_split, False)):
        stores[name] = DeviceFeatureStore(split["features"], split["positions"], device=device, dtype=feature_dtype)
        loaders[name] = ResidentBatches(split["captions"], split["image_idxs"], batch_size, device=device,
                                        shuffle=shuffle, seed=seed)
    # the fixed evaluation batches: the first train (shuffled) and valid batch (main.py:45-55)
    eval_batches = {n: next(iter(loaders[n])) for n in ("train", "valid")}
    n_valid_images = stores["valid"].n_images
    train_caps = np.asarray(train_split["captions"])
    train_img = np.asarray(train_split["image_idxs"])

    def loss_of(name, idx, caps):
        f, p = _gather(stores[name], idx)
        return model.compute_loss(object_features=f, position_features=p, target_caption=caps)

    n_iter = len(loaders["train"])
    history = []
    for epoch in range(1, num_epoch + 1):
        log(f"Epoch {epoch}")
        for i, (idx, caps) in enumerate(loaders["train"]):
            model.train_step_resident(stores["train"], idx, caps)
            step = i + n_iter * (epoch - 1)
            if (i + 1) % eval_every == 0:
                tl = loss_of("train", *eval_batches["train"])
                vl = loss_of("valid", *eval_batches["valid"])
                log({"step": step, **{k: {"train": tl[k].mean().item(), "valid": vl[k].mean().item()}
                                      for k in write_log}})
            if (i + 1) % sample_every == 0:
                f, p = _gather(stores["train"], idx[:1])
                sample, _ = model.generate_caption(object_features=f, position_features=p)
                img = int(idx[0].item())
                truths = model.decode_captions(train_caps[train_img == img])
                log({"step": step, "sample": sample[0], "truths": truths})

        # evaluation (main.py:104-146)
        valid_caption = [""] * n_valid_images
        logs = {k: {"train": 0.0, "valid": 0.0} for k in write_log}
        for (t_idx, t_caps), (v_idx, v_caps) in zip(loaders["train"], loaders["valid"]):
            tl = loss_of("train", t_idx, t_caps)
            vl = loss_of("valid", v_idx, v_caps)
            for k in write_log:
                logs[k]["train"] += tl[k].mean().item()
                logs[k]["valid"] += vl[k].mean().item()
            f, p = _gather(stores["valid"], v_idx)
            captions, _ = model.generate_caption(object_features=f, position_features=p)
            for j, c in zip(v_idx.tolist(), captions):
                valid_caption[j] = c
        # the reference divides by len(valid_dataloader) (main.py:130-132)
        for k in write_log:
            logs[k]["train"] /= max(1, len(loaders["valid"]))
            logs[k]["valid"] /= max(1, len(loaders["valid"]))
        with open(os.path.join(target_dir, "valid.candidate.captions.pkl"), "wb") as fh:
            pickle.dump(valid_caption, fh)
        scores = dict(evaluate(target_dir) if evaluate is not None else {})
        scores.update(logs)
        log({"epoch": epoch, "train_loss": scores["loss"]["train"] if "loss" in scores else None,
             "valid_loss": scores["loss"]["valid"] if "loss" in scores else None})
        model.save(path=os.path.join(model_dir, f"model_{epoch}.pt"))
        history.append(scores)
    return history
