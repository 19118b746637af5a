"""Helpers shared by the parity tests: load a golden fixture and its config."""
import os
import zlib

import numpy as np

from capgen.config import preset

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# must mirror tests/golden/gen_golden.py FIXTURES (cfg, B, N, T, seed, beam_k)
FIXTURE_CFG = {
    "c1": (lambda: preset("C1"), 0),
    "c1_encmask": (lambda: preset("C1", encode_mask=True), 1),
    "c1_focal": (lambda: preset("C1", output_name="FocalLoss_Transformer"), 2),
    "c2s": (lambda: preset("C2", num_vocab=1000), 3),
    "c1_splitpos": (lambda: preset("C1", split_position=True), 4),
    "c1_imgobj": (lambda: preset("C1", split_image_objects=True), 7),
    "c1_movefirst": (lambda: preset("C1", move_first_image_feature=True), 8),
    # POLICY_FIXTURES (PolicyNetwork decoding, log-softmax scoring)
    "c1_policy": (lambda: preset("C1"), 9),
    "c2s_policy": (lambda: preset("C2", num_vocab=1000), 10),
    # RL_FIXTURES (SCST, injected rewards)
    "c5_rl": (lambda: preset("C1"), 5),
    "c5_rl_pad": (lambda: preset("C1"), 6),
    "c5_rl_c2s": (lambda: preset("C2", num_vocab=1000), 12),
}


def load_fixture(tag):
    z = np.load(os.path.join(GOLDEN, f"{tag}.npz"), allow_pickle=False)
    make, seed = FIXTURE_CFG[tag]
    cfg = make()
    assert int(z["seed"]) == seed
    return cfg, seed, {k: z[k] for k in z.files}


def sample_index(name, numel, n=8):
    r = np.random.default_rng(zlib.crc32(name.encode()))
    return np.sort(r.choice(numel, size=min(n, numel), replace=False))
