"""SCST host pieces: the CIDEr-D / BLEU-4 restatements (capgen/scst.py, parity unpinned — the
reference's coco-caption scorers are un-vendored) and the reward assembly."""
import math

import numpy as np

from capgen.scst import Bleu, CiderD, RewardScorer


def test_bleu_identical_and_disjoint():
    b = Bleu(4)
    same = b.compute_score({0: ["a man riding a horse ."]}, {0: ["a man riding a horse ."]})[1]
    assert all(abs(s[0] - 1.0) < 1e-6 for s in same)
    disj = b.compute_score({0: ["a man riding a horse ."]}, {0: ["two cats sleep"]})[1][3][0]
    assert disj < 1e-6


def test_bleu_hand_computed():
    # hyp "the cat sat" vs ref "the cat sat on the mat": p1 = p2 = p3 = 1, p4 = tiny/small;
    # brevity penalty exp(1 - 6/3); BLEU-1 = exp(-1)
    b = Bleu(4)
    per = b.compute_score({0: ["the cat sat on the mat"]}, {0: ["the cat sat"]})[1]
    assert abs(per[0][0] - math.exp(1 - 6 / 3)) < 1e-9
    assert abs(per[2][0] - math.exp(1 - 6 / 3)) < 1e-9


def test_ciderd_properties():
    c = CiderD()
    gts = {0: ["a man riding a horse ."], 1: ["two dogs play in the park ."], 2: ["a red bus on a street ."]}
    res = {0: ["a man riding a horse ."], 1: ["a cat ."], 2: ["a red bus on a road ."]}
    mean, s = c.compute_score(gts, res)
    assert abs(s[0] - 10.0) < 1e-9            # identical caption: cosine 1 at every n, no length penalty
    assert 0.0 <= s[1] < s[2] < s[0]          # partial overlap scores between
    assert abs(mean - s.mean()) < 1e-12


def test_reward_scorer_weights_and_entropy():
    idx = {0: "<NULL>", 1: "<START>", 2: "<END>", 3: "a", 4: "man", 5: "horse", 6: "dog"}
    sc = RewardScorer(idx, cider_reward_weight=0.5, bleu_reward_weight=2.0, entropy_reward_weight=0.25)
    target = np.array([[3, 4, 2, 0], [3, 6, 2, 0]])
    sample = np.array([[3, 4, 2, 0], [3, 5, 2, 0]])
    r = sc.scores(target, sample)
    cider = CiderD().compute_score({0: ["a man ."], 1: ["a dog ."]}, {0: ["a man ."], 1: ["a horse ."]})[1]
    bleu = np.array(Bleu(4).compute_score({0: ["a man ."], 1: ["a dog ."]}, {0: ["a man ."], 1: ["a horse ."]})[1][3])
    np.testing.assert_allclose(r, 0.5 * cider + 2.0 * bleu)
    np.testing.assert_allclose(sc.total(r, [1.0, 2.0]), r + 0.25 * np.array([1.0, 2.0]))


def test_native_rewards_equal_python_restatement():
    """libcapgen's host scorer (token ids, csrc/scst_host.cpp) equals the Python CiderD/Bleu
    restatement on decoded strings: random samples with <END>/<NULL>/<START> anywhere, a small
    vocabulary (many shared n-grams), with and without a "." word in the vocabulary."""
    rng = np.random.default_rng(7)
    for with_dot in (False, True):
        words = ["<NULL>", "<START>", "<END>"] + [f"w{i}" for i in range(20)] + (["."] if with_dot else [])
        idx = dict(enumerate(words))
        for B, L in ((64, 19), (5, 3), (1, 6)):
            target = rng.integers(3, len(words), size=(B, L))
            sample = rng.integers(0, len(words), size=(B, L))
            for b in range(B):  # end the references at a random length, pad after
                e = rng.integers(1, L + 1)
                if e < L:
                    target[b, e] = 2
                    target[b, e + 1:] = 0
            py = RewardScorer(idx, cider_reward_weight=1.0, bleu_reward_weight=1.0, native=False)
            nat = RewardScorer(idx, cider_reward_weight=1.0, bleu_reward_weight=1.0)
            assert nat.native and not py.native
            np.testing.assert_allclose(nat.scores(target, sample), py.scores(target, sample), rtol=1e-9, atol=1e-12)


def test_native_rewards_packed_and_general_keys_agree():
    """The native scorer packs n-grams into 64-bit keys when every token id (the "." id
    included) is below 65534 and falls back to general keys otherwise; both give the same
    rewards: the same token streams scored with ids shifted above 65534 (general path) and
    as is (packed path), with the "." sentinel (no "." word) and with a real "." id."""
    from capgen.scst import native_rewards
    rng = np.random.default_rng(11)
    B, L = 32, 12
    target = rng.integers(3, 40, size=(B, L))
    sample = rng.integers(0, 40, size=(B, L))
    for b in range(B):
        e = rng.integers(1, L + 1)
        if e < L:
            target[b, e] = 2
            target[b, e + 1:] = 0
    shift = 70000  # ids >= 3 moved above the 16-bit slot range; <NULL>/<START>/<END> keep theirs
    t2 = np.where(target >= 3, target + shift, target)
    s2 = np.where(sample >= 3, sample + shift, sample)
    for dot in (-1, 5):
        a = native_rewards(target, sample, 1, 2, 0, dot, 1.0, 1.0)
        b = native_rewards(t2, s2, 1, 2, 0, dot + shift if dot >= 0 else -1, 1.0, 1.0)
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-14)
