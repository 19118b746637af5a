"""`TRANSFORMER` — drop-in for core/models.py:18-135 (the object `main.py` drives).

main.py uses exactly: train_step, compute_loss, generate_caption, decode_captions, save,
load (main.py:65,70,73,85,112,116,124,151).  Inputs arrive as host tensors; the wrapper
stages them into persistent device buffers so the captured train-step hipGraph replays
with fixed pointers (the reference did a synchronous pageable `.to(DEVICE)` per step,
models.py:120-122).
"""
from __future__ import annotations

import numpy as np
import torch

from .config import CapgenConfig
from .model import PolicyNetwork, Transformer
from .staging import HostBatchStager
from .utils import decode_captions, load_word_to_idx


def _on_device(t) -> bool:
    return isinstance(t, torch.Tensor) and t.is_cuda


class MODEL_init:
    def __init__(self, word_to_idx=None, word_to_idx_path=None):
        if word_to_idx is None:
            if word_to_idx_path is None:
                raise ValueError("capgen: pass word_to_idx or word_to_idx_path (models.py:22)")
            word_to_idx = load_word_to_idx(word_to_idx_path)
        self.num_vocab = len(word_to_idx)
        self.idx_to_word = {i: w for w, i in word_to_idx.items()}
        self.model = None

    def train_step(self, *a, **k):
        raise NotImplementedError

    def compute_loss(self, *a, **k):
        raise NotImplementedError

    def generate_caption(self, object_features, position_features, beam_size=None):
        """models.py:34-56: None/1 -> greedy (+attention_list); int > 1 -> beam search."""
        if beam_size in [None, 1]:
            ids, attention_list = self.model.generate_caption_vector(object_features=object_features,
                                                                     position_features=position_features)
            return self.decode_captions(ids.cpu().numpy()), attention_list
        if isinstance(beam_size, int) and beam_size > 1:
            ids = self.model.beam_search(object_features=object_features, position_features=position_features,
                                         beam_size=beam_size)
            return self.decode_captions(ids.cpu().numpy()), None
        assert isinstance(beam_size, int)
        assert beam_size > 1 or beam_size in [None, 1]

    def decode_captions(self, caption_vector):
        return decode_captions(caption_vector, self.idx_to_word)

    def save(self, path):
        torch.save(self.model.state_dict(), path)

    def load(self, path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(sd)
        self.model.eval()


class TRANSFORMER(MODEL_init):
    def __init__(self, config: CapgenConfig | None = None, word_to_idx=None, word_to_idx_path=None,
                 device="cuda:0", state_dict=None):
        super().__init__(word_to_idx, word_to_idx_path)
        cfg = (config or CapgenConfig()).replace(num_vocab=self.num_vocab)
        self.config = cfg
        self.device = torch.device(device)
        self.model = Transformer.from_config(cfg, self.device, state_dict=state_dict)
        self._stage = {}
        self._host_stager = None

    def _staged(self, name, t, dtype):
        buf = self._stage.get(name)
        if buf is None or buf.shape != t.shape or buf.dtype != dtype:
            buf = torch.empty(t.shape, dtype=dtype, device=self.device)
            self._stage[name] = buf
        buf.copy_(t, non_blocking=True)
        return buf

    def train_step(self, batch_features, batch_positions, batch_captions):
        """models.py:115-126: zero_grad + forward + backward + Adam, one engine call.

        Host (CPU / numpy) batches -- what main.py's DataLoader yields -- go through pinned,
        double-buffered staging with the copy on a side stream, overlapped with the previous
        step (capgen.staging.HostBatchStager); device tensors are staged by a D2D copy."""
        if not _on_device(batch_features):
            st = self._host_stager
            if st is None or not st.fits(batch_features, batch_positions, batch_captions):
                B, N, F = batch_features.shape
                st = self._host_stager = HostBatchStager(self.device, B, N, F, batch_positions.shape[2],
                                                         batch_captions.shape[1])
            st.run(self.model.engine, batch_features, batch_positions, batch_captions)
            return
        fdt = torch.bfloat16 if self.config.dtype == "bf16" else torch.float32
        f = self._staged("f", batch_features, fdt)
        p = self._staged("p", batch_positions, torch.float32)
        c = self._staged("c", batch_captions, torch.int32)
        self.model.engine.train_step(f, p, c)

    def train_step_resident(self, store, img_idx, captions):
        """train_step over an HBM-resident split (capgen.data.DeviceFeatureStore / ResidentBatches):
        the batch names its images; nothing is copied from the host."""
        self.model.engine.train_step_indexed(store.features, store.positions, img_idx, captions)

    def compute_loss(self, object_features, position_features, target_caption):
        """models.py:128-135 (no_grad; dropout follows train/eval state)."""
        with torch.no_grad():
            return self.model(object_features=object_features, position_features=position_features,
                              target_caption=target_caption)


class SelfCriticNetwork(MODEL_init):
    """Drop-in for core/models.py:137-211 (SCST, config C5): same network as TRANSFORMER
    (PolicyNetwork, model_RL.py:10-97 = Encoder/Decoder/classifer), trained on
    (1 - w) * CE + w * structure loss with CIDEr-D + BLEU-4 + entropy rewards (loss.py:31-220).

    One step = capgen_rl_sample (GPU) -> host scoring of the greedy-from-logits samples
    (capgen/scst.py, parity unpinned) -> capgen_rl_finish (GPU: loss, backward, Adam).

    df: CIDEr-D document frequencies.  The reference scores with CiderD(df='coco-val')
    (loss.py:112), a table computed from the COCO validation references that the reference does
    not ship; the default 'corpus' computes them from the references being scored (coco-caption's
    corpus mode) and warns.  Pass df=(document_frequency, ref_len) to use a precomputed table."""

    def __init__(self, config: CapgenConfig | None = None, word_to_idx=None, word_to_idx_path=None,
                 device="cuda:0", state_dict=None, structure_loss_weight=0.5, cider_reward_weight=1.0,
                 bleu_reward_weight=1.0, entropy_reward_weight=1.0, self_cider_reward_weight=1.0, df="corpus"):
        super().__init__(word_to_idx, word_to_idx_path)
        from .scst import RewardScorer
        cfg = (config or CapgenConfig()).replace(num_vocab=self.num_vocab)
        self.config = cfg
        self.device = torch.device(device)
        # PolicyNetwork (model_RL.py): generate_caption then decodes with LogSoftmax scoring
        self.model = PolicyNetwork.from_config(cfg, self.device, state_dict=state_dict)
        if isinstance(df, str) and df == "corpus":
            import warnings
            warnings.warn("capgen SelfCriticNetwork: CIDEr-D document frequencies from the scored references "
                          "(df='corpus'); the reference uses CiderD(df='coco-val') (loss.py:112), whose table is "
                          "not shipped with it -- pass df=(document_frequency, ref_len) for that reward",
                          stacklevel=2)
        self.structure_loss_weight = float(structure_loss_weight)  # core/config.py:81-85
        self.scorer = RewardScorer(self.idx_to_word, cider_reward_weight, bleu_reward_weight, entropy_reward_weight,
                                   self_cider_reward_weight, df=df)

    def _step(self, object_features, position_features, target_caption, train):
        eng = self.model.engine
        sample, entropy, _ = eng.rl_sample(object_features, position_features, target_caption)
        target = torch.as_tensor(target_caption)[:, 1:].cpu().numpy()
        reward = np.broadcast_to(self.scorer.scores(target, sample.cpu().numpy()), (sample.shape[0],))
        total = self.scorer.total(reward, entropy.cpu().numpy())
        out = eng.rl_finish(total, self.structure_loss_weight, train=train)
        return out, reward

    def train_step(self, batch_features, batch_positions, batch_captions):
        """models.py:179-195: forward, sample, reward, loss.backward(), Adam step."""
        self._step(batch_features, batch_positions, batch_captions, train=True)

    def compute_loss(self, object_features, position_features, target_caption):
        """models.py:198-211 -> {'loss', 'language_model_loss', 'structure_loss', 'reward'}
        (config.py:65-68 keys; reward [B, 1] as in loss.py:121)."""
        with torch.no_grad():
            out, reward = self._step(object_features, position_features, target_caption, train=False)
        return {"loss": out[0], "language_model_loss": out[1], "structure_loss": out[2],
                "reward": torch.as_tensor(np.array(reward), dtype=torch.float32).view(-1, 1)}
