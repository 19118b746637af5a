"""Host-side rewards for self-critical training (StructureCriterion.get_scores, loss.py:154-181).

The reference scores samples with coco-caption's CIDEr-D (`CiderD(df='coco-val')`), BLEU-4
(`Bleu(4)`, per-sentence) and a self-CIDEr diversity term, imported from the UN-VENDORED
`core.metrics` package (loss.py:7-9): no source, no pinned version and no `coco-val` document
frequency table exist in the reference.  These are restatements of the published algorithms
(Vedantam et al. 2015 CIDEr-D as in the coco-caption / ruotianluo `cider` scorers; Papineni et
al. 2002 BLEU with coco-caption's per-sentence smoothing and 'closest' reference length).
PARITY UNPINNED: nothing in the reference pins their values; the loss mechanics that consume
them are pinned by tests/golden/c5_rl*.npz (injected rewards).

Document frequencies: `df="corpus"` (default) computes them from the references being scored
(coco-caption's CiderD 'corpus' mode); pass `df=(document_frequency, ref_len)` to use a
precomputed table such as coco-val's.
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict

import numpy as np


def _ngrams(sentence: str, n: int = 4) -> Counter:
    words = sentence.split()
    c = Counter()
    for k in range(1, n + 1):
        for i in range(len(words) - k + 1):
            c[tuple(words[i:i + k])] += 1
    return c


class Bleu:
    """coco-caption Bleu(4).compute_score: returns (corpus scores [4], per-sentence scores [4][B])."""

    def __init__(self, n: int = 4):
        self.n = n

    def compute_score(self, gts: dict, res: dict):
        n, tiny, small = self.n, 1e-15, 1e-9
        per = [[] for _ in range(n)]
        tot_guess, tot_correct = [0] * n, [0] * n
        tot_test = tot_ref = 0
        for key in sorted(res):
            hyp = res[key]
            assert isinstance(hyp, list) and len(hyp) == 1
            refs = gts[key]
            test = hyp[0].split()
            testlen = len(test)
            counts = _ngrams(hyp[0], n)
            reflens = [len(r.split()) for r in refs]
            maxref = Counter()
            for r in refs:
                for g, c in _ngrams(r, n).items():
                    maxref[g] = max(maxref[g], c)
            reflen = min((abs(l - testlen), l) for l in reflens)[1]  # 'closest'
            guess = [max(0, testlen - k + 1) for k in range(1, n + 1)]
            correct = [0] * n
            for g, c in counts.items():
                correct[len(g) - 1] += min(maxref.get(g, 0), c)
            tot_test += testlen
            tot_ref += reflen
            for k in range(n):
                tot_guess[k] += guess[k]
                tot_correct[k] += correct[k]
            b = 1.0
            for k in range(n):
                b *= (correct[k] + tiny) / (guess[k] + small)
                per[k].append(b ** (1.0 / (k + 1)))
            ratio = (testlen + tiny) / (reflen + small)
            if ratio < 1:
                for k in range(n):
                    per[k][-1] *= math.exp(1 - 1 / ratio)
        corpus, b = [], 1.0
        for k in range(n):
            b *= (tot_correct[k] + tiny) / (tot_guess[k] + small)
            corpus.append(b ** (1.0 / (k + 1)))
        ratio = (tot_test + tiny) / (tot_ref + small)
        if ratio < 1:
            corpus = [c * math.exp(1 - 1 / ratio) for c in corpus]
        return corpus, per


class CiderD:
    """CIDEr-D (sigma 6, clipped n-gram tf-idf, Gaussian length penalty, x10), n = 1..4."""

    def __init__(self, df="corpus", n: int = 4, sigma: float = 6.0):
        self.df_mode, self.n, self.sigma = df, n, sigma

    def _vec(self, counts, df, ref_len):
        vec = [defaultdict(float) for _ in range(self.n)]
        norm = [0.0] * self.n
        length = 0
        for g, tf in counts.items():
            k = len(g) - 1
            vec[k][g] = float(tf) * (ref_len - np.log(max(1.0, df.get(g, 0.0))))
            norm[k] += vec[k][g] ** 2
            if k == 1:  # as in the coco-caption scorer: the "length" counts bigrams
                length += tf
        return vec, [np.sqrt(x) for x in norm], length

    def _sim(self, vh, vr, nh, nr, lh, lr):
        delta = float(lh - lr)
        val = np.zeros(self.n)
        for k in range(self.n):
            for g in vh[k]:
                val[k] += min(vh[k][g], vr[k][g]) * vr[k][g]
            if nh[k] != 0 and nr[k] != 0:
                val[k] /= nh[k] * nr[k]
            val[k] *= np.e ** (-(delta ** 2) / (2 * self.sigma ** 2))
        return val

    def compute_score(self, gts: dict, res: dict):
        keys = sorted(res)
        crefs = [[_ngrams(r) for r in gts[k]] for k in keys]
        ctest = []
        for k in keys:
            assert isinstance(res[k], list) and len(res[k]) == 1
            ctest.append(_ngrams(res[k][0]))
        if self.df_mode == "corpus":
            df = Counter()
            for refs in crefs:
                for g in {g for r in refs for g in r}:
                    df[g] += 1
            ref_len = np.log(float(len(crefs)))
        else:
            df, ref_len = self.df_mode
        scores = []
        for test, refs in zip(ctest, crefs):
            vh, nh, lh = self._vec(test, df, ref_len)
            acc = np.zeros(self.n)
            for r in refs:
                vr, nr, lr = self._vec(r, df, ref_len)
                acc += self._sim(vh, vr, nh, nr, lh, lr)
            scores.append(np.mean(acc) / len(refs) * 10.0)
        scores = np.array(scores)
        return float(scores.mean()) if len(scores) else 0.0, scores


def self_cider_single(res_one: list) -> float:
    """get_self_cider_scores (loss.py:183-205) for ONE caption per image: the self-CIDEr kernel is
    1x1, eigvals = [k/10], and the diversity -log(sqrt(e)/sqrt(e))/1e-8 is exactly 0 (the
    reference's inf for an all-zero kernel is not reproduced)."""
    return 0.0


def native_rewards(target, sample, start_id, end_id, null_id, dot_id, cider_w, bleu_w):
    """cider_w * CIDEr-D + bleu_w * BLEU-4 per image, computed by libcapgen's host code
    (csrc/scst_host.cpp: the arithmetic of CiderD(df='corpus') and Bleu(4) above on token ids)."""
    import ctypes as C
    from . import _lib
    lib = _lib.load()
    t = np.ascontiguousarray(target, dtype=np.int64)
    s = np.ascontiguousarray(sample, dtype=np.int64)
    assert t.ndim == 2 and t.shape == s.shape
    B, L = t.shape
    out = np.empty(B, dtype=np.float64)
    _lib.check(lib.capgen_scst_rewards(t.ctypes.data_as(C.c_void_p), L, s.ctypes.data_as(C.c_void_p), L, B, L,
                                       int(start_id), int(end_id), int(null_id), int(dot_id), float(cider_w),
                                       float(bleu_w), out.ctypes.data_as(C.c_void_p)))
    return out


class RewardScorer:
    """StructureCriterion.get_scores + the entropy / self-CIDEr terms (loss.py:115-181).

    native=True (default with corpus document frequencies): the rewards come from libcapgen's
    host code on token ids (`native_rewards`), the Python CiderD/Bleu above being the
    restatement it is tested against (tests/test_scst.py)."""

    def __init__(self, idx_to_word, cider_reward_weight=1.0, bleu_reward_weight=1.0, entropy_reward_weight=1.0,
                 self_cider_reward_weight=1.0, df="corpus", native=True):
        from .utils import decode_captions
        self._decode = lambda ids: decode_captions(ids, idx_to_word)
        self.cider_w, self.bleu_w = cider_reward_weight, bleu_reward_weight
        self.entropy_w, self.self_cider_w = entropy_reward_weight, self_cider_reward_weight
        self.ciderD = CiderD(df=df)
        self.bleu = Bleu(4)
        w2i = {w: i for i, w in (idx_to_word.items() if isinstance(idx_to_word, dict) else enumerate(idx_to_word))}
        self._ids = (w2i.get("<START>", 1), w2i.get("<END>", 2), w2i.get("<NULL>", 0), w2i.get(".", -1))
        self.native = native and isinstance(df, str) and df == "corpus"

    def scores(self, target, sample):
        """target = caption[:, 1:] [B, L], sample [B, L] (host int arrays) -> reward [B]."""
        if self.native:
            return native_rewards(target, sample, *self._ids, self.cider_w, self.bleu_w)
        res = self._decode(np.asarray(sample))
        gts = self._decode(np.asarray(target))
        res_d = {i: [res[i]] for i in range(len(res))}
        gts_d = {i: [gts[i]] for i in range(len(gts))}
        cider = self.ciderD.compute_score(gts_d, res_d)[1] if self.cider_w > 0 else 0.0
        if self.bleu_w > 0:
            try:
                bleu = np.array(self.bleu.compute_score(gts_d, res_d)[1][3])
            except Exception:  # loss.py:168-173 swallows scorer failures as 0
                bleu = 0.0
        else:
            bleu = 0.0
        return self.cider_w * np.asarray(cider, dtype=np.float64) + self.bleu_w * np.asarray(bleu, dtype=np.float64)

    def total(self, reward, entropy):
        """reward + entropy_w * masked mean entropy + self_cider_w * self-CIDEr (0 here)."""
        return np.asarray(reward, dtype=np.float64) + self.entropy_w * np.asarray(entropy, dtype=np.float64)
