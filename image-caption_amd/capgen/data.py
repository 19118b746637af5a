"""Input pipeline for the training loop: the MI355X-first replacement
for `TrainDataset` + `DataLoader(batch_size, shuffle=True)` + the per-step `.to(DEVICE)` of
main.py:37-43 / dataset.py:8-29 / models.py:120-122.

The reference keeps the whole split in host RAM and copies every batch (18.9 MB f32 at C2)
synchronously to the GPU.  Here the split's region features and positions are uploaded ONCE
into HBM (a COCO train split is ~113k images x 37 x 2048 bf16 = ~17 GB of 288 GB), and a step
only names its images: the encoder-input pack kernel gathers image `img_idx[b]` straight from
the resident store (capgen_train_step_indexed).  Captions (int32, ~30 MB for COCO) are resident
too; shuffling is a device permutation per epoch.

On-disk format: `{split}.features.npy` [n_images, N, F], `{split}.positions.npy` [n_images, N, P],
`{split}.captions.npy` [n_captions, T] and `{split}.image.indices.npy` [n_captions], loaded with
numpy's non-pickling loader (memory-mapped, streamed to the device in chunks).  The reference
writes hickle (HDF5) + pickle files (core/utils.py:32-64); hickle/h5py are not part of this
image, so converting those files to .npy is a one-time step outside this package.
"""
from __future__ import annotations

import os

import numpy as np
import torch


class DeviceFeatureStore:
    """Region features [n_images, N, F] (bf16 or f32) and positions [n_images, N, P] (f32),
    resident on one device."""

    def __init__(self, features, positions, device="cuda:0", dtype=torch.bfloat16, chunk_images=4096):
        self.device = torch.device(device)
        n, N, F = features.shape
        if positions.shape[:2] != (n, N):
            raise ValueError("capgen.data: features and positions disagree on [n_images, N]")
        self.features = torch.empty((n, N, F), dtype=dtype, device=self.device)
        self.positions = torch.empty(tuple(positions.shape), dtype=torch.float32, device=self.device)
        for s in range(0, n, chunk_images):  # bounded host memory: memmap slices -> device
            e = min(n, s + chunk_images)
            self.features[s:e].copy_(torch.as_tensor(np.ascontiguousarray(features[s:e])).to(dtype))
            self.positions[s:e].copy_(torch.as_tensor(np.ascontiguousarray(positions[s:e]), dtype=torch.float32))

    @property
    def n_images(self):
        return self.features.shape[0]


class ResidentBatches:
    """Per-caption batches (dataset.py:12-18 semantics: caption i with its image image_idxs[i]),
    shuffled per epoch on the device; yields (img_idx int32 [B], captions int32 [B, T]), both
    device tensors.  The last partial batch is kept, as DataLoader(drop_last=False) does."""

    def __init__(self, captions, image_idxs, batch_size, device="cuda:0", shuffle=True, seed=0):
        self.device = torch.device(device)
        self.captions = torch.as_tensor(np.asarray(captions), dtype=torch.int32).to(self.device)
        self.image_idxs = torch.as_tensor(np.asarray(image_idxs), dtype=torch.int32).to(self.device)
        if self.captions.shape[0] != self.image_idxs.shape[0]:
            raise ValueError("capgen.data: one image index per caption")
        self.batch_size, self.shuffle = int(batch_size), shuffle
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)

    def __len__(self):
        return (self.captions.shape[0] + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = self.captions.shape[0]
        order = (torch.randperm(n, generator=self.gen, device=self.device) if self.shuffle
                 else torch.arange(n, device=self.device))
        for s in range(0, n, self.batch_size):
            sel = order[s:s + self.batch_size]
            yield self.image_idxs.index_select(0, sel), self.captions.index_select(0, sel)


def load_split(data_path, split, mmap=True):
    """{split}.features/.positions/.captions/.image.indices .npy -> dict of arrays (no pickle)."""
    d = os.path.join(data_path, split)
    mode = "r" if mmap else None
    out = {}
    for key, name in [("features", "features"), ("positions", "positions"), ("captions", "captions"),
                      ("image_idxs", "image.indices")]:
        out[key] = np.load(os.path.join(d, f"{split}.{name}.npy"), mmap_mode=mode, allow_pickle=False)
    return out
