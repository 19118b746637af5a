"""Host-side text helpers of the boundary (core/utils.py:67-103)."""
from __future__ import annotations

import io
import json
import pickle

import numpy as np


def decode_captions(captions, index_to_word):
    """ids -> sentences: skip <START> at t=0, <END> -> '.' and stop, drop <NULL>
    (core/utils.py:67-103; its 'a'->'an' branch can never fire and is omitted)."""
    captions = np.asarray(captions)
    rows = captions[None] if captions.ndim == 1 else captions
    out = []
    for row in rows:
        words = []
        for t, idx in enumerate(row):
            w = index_to_word[int(idx)]
            if w == "<START>" and t == 0:
                continue
            if w == "<END>":
                words.append(".")
                break
            if w != "<NULL>":
                words.append(w)
        out.append(" ".join(words))
    return out


class _VocabUnpickler(pickle.Unpickler):
    """word_index.pkl holds a plain {str: int} dict; refuse anything that is not data."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"capgen: refusing to load {module}.{name} from a vocabulary file")


def load_word_to_idx(path):
    """Vocabulary file of core/models.py:22 ({word: index}); JSON or a data-only pickle."""
    with open(path, "rb") as f:
        raw = f.read()
    if path.endswith(".json"):
        return {str(k): int(v) for k, v in json.loads(raw.decode()).items()}
    d = _VocabUnpickler(io.BytesIO(raw)).load()
    if not isinstance(d, dict):
        raise ValueError("capgen: vocabulary file must hold a dict")
    return {str(k): int(v) for k, v in d.items()}
