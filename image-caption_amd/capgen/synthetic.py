"""Synthetic batches with the shape and padding structure of the reference data
(SURVEY.md §8(d)): region features are post-ReLU-like non-negative values, padded
regions are all-zero rows in BOTH features and positions (so the key-pad mask of
model.py:202-209 fires), positions carry a sorted box + one class confidence
(data/detect_for_preprocess.py:134-138, image row core/preprocess.py:121-123), and
captions are <START> words <END> <NULL>... (core/preprocess.py:322-338).
"""
from __future__ import annotations

import torch

START, END, PAD = 1, 2, 0


def synthetic_batch(B: int, N: int, F: int, P: int, T: int, V: int, seed: int = 0,
                    min_valid: int | None = None):
    """Returns (feats f32 [B,N,F], pos f32 [B,N,P], caps int32 [B,T]) on CPU."""
    g = torch.Generator().manual_seed(seed)
    feats = torch.randn(B, N, F, generator=g).clamp_min_(0.0)
    if min_valid is None:
        min_valid = min(12, N)
    n_valid = torch.randint(min_valid, N + 1, (B,), generator=g)
    pos = torch.zeros(B, N, P)
    box = torch.rand(B, N, 4, generator=g)
    x = torch.sort(box[..., 0:4:2], dim=-1).values
    y = torch.sort(box[..., 1:4:2], dim=-1).values
    pos[..., 0], pos[..., 2] = x[..., 0], x[..., 1]
    pos[..., 1], pos[..., 3] = y[..., 0], y[..., 1]
    if P > 4:
        cls = torch.randint(4, P, (B, N), generator=g)
        conf = 0.01 + 0.99 * torch.rand(B, N, generator=g)
        pos.scatter_(2, cls.unsqueeze(-1), conf.unsqueeze(-1))
    pos[:, 0, :] = 0.0
    pos[:, 0, 2] = 1.0
    pos[:, 0, 3] = 1.0                       # whole-image row [0, 0, 1, 1]
    valid = torch.arange(N)[None, :] < n_valid[:, None]
    feats *= valid[..., None]
    pos *= valid[..., None]
    caps = torch.zeros(B, T, dtype=torch.int32)
    caps[:, 0] = START
    lo, hi = min(5, T - 2), T - 2
    lengths = torch.randint(lo, hi + 1, (B,), generator=g)
    words = torch.randint(4, V, (B, T), generator=g, dtype=torch.int32)
    for b in range(B):
        l = int(lengths[b])
        caps[b, 1:1 + l] = words[b, :l]
        caps[b, 1 + l] = END
    return feats, pos, caps
