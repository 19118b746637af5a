"""`Transformer` — drop-in for core/TRANSFORMER/model.py:8-209 backed by libcapgen.

Same constructor keywords, same `forward(object_features, position_features,
target_caption) -> {'loss': ...}`, `generate_caption_vector(...) -> (LongTensor [B,
max_length+1], attention_list)` and `beam_search(..., beam_size) -> LongTensor [B,
max_length]`, same state_dict keys.  `loss.backward()` runs the engine's hand-written
backward pass; `CapgenAdam` plays torch.optim.Adam (models.py:111-113).
"""
from __future__ import annotations

import numpy as np
import torch

from .config import CapgenConfig
from .engine import Engine


class _EngineLoss(torch.autograd.Function):
    """Connects the engine's loss scalar to autograd: backward() = capgen_backward."""

    @staticmethod
    def forward(ctx, anchor, loss, engine_box):
        ctx.engine = engine_box[0]
        return loss.clone().reshape(())

    @staticmethod
    def backward(ctx, grad):
        ctx.engine.backward()
        return torch.zeros(1, device=grad.device), None, None


class Transformer:
    def __init__(self, num_vocab, max_length, encode_dim_positions, encode_dim_features, device,
                 output_name="Transformer", encode_mask=False, pad_idx=0, dropout=0.2,
                 encode_input_size=512, encode_q_k_dim=512, encode_v_dim=512, encode_hidden_size=2048,
                 encode_num_blocks=6, encode_num_heads=8, dim_word_embedding=512, decode_input_size=512,
                 decode_q_k_dim=512, decode_v_dim=512, decode_hidden_size=2048, decode_num_blocks=6,
                 decode_num_heads=8, move_first_image_feature=False, split_position=False,
                 split_image_objects=False, dtype="bf16", learning_rate=5e-4, seed=1234, state_dict=None):
        self.config = CapgenConfig(
            num_vocab=num_vocab, max_length=max_length, encode_dim_positions=encode_dim_positions,
            encode_dim_features=encode_dim_features, output_name=output_name, encode_mask=encode_mask,
            pad_idx=pad_idx, dropout=dropout, encode_input_size=encode_input_size,
            encode_q_k_dim=encode_q_k_dim, encode_v_dim=encode_v_dim, encode_hidden_size=encode_hidden_size,
            encode_num_blocks=encode_num_blocks, encode_num_heads=encode_num_heads,
            dim_word_embedding=dim_word_embedding, decode_input_size=decode_input_size,
            decode_q_k_dim=decode_q_k_dim, decode_v_dim=decode_v_dim, decode_hidden_size=decode_hidden_size,
            decode_num_blocks=decode_num_blocks, decode_num_heads=decode_num_heads,
            move_first_image_feature=move_first_image_feature, split_position=split_position,
            split_image_objects=split_image_objects, dtype=dtype, learning_rate=learning_rate, seed=seed)
        self.max_length = max_length
        self.num_vocab = num_vocab
        self.pad_idx = pad_idx
        self.device = torch.device(device)
        self.engine = Engine(self.config, self.device)
        if state_dict is None:
            from .params import reference_init_state_dict
            state_dict = reference_init_state_dict(self.config, seed=seed)
            state_dict = {k: torch.from_numpy(v) for k, v in state_dict.items()}
        self.engine.load_state_dict(state_dict)
        self._anchor = torch.zeros(1, device=self.device, requires_grad=True)
        self.training = True

    @classmethod
    def from_config(cls, cfg: CapgenConfig, device, state_dict=None):
        obj = cls.__new__(cls)
        obj.config = cfg
        obj.max_length, obj.num_vocab, obj.pad_idx = cfg.max_length, cfg.num_vocab, cfg.pad_idx
        obj.device = torch.device(device)
        obj.engine = Engine(cfg, obj.device)
        if state_dict is None:
            from .params import reference_init_state_dict
            state_dict = {k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=cfg.seed).items()}
        obj.engine.load_state_dict(state_dict)
        obj._anchor = torch.zeros(1, device=obj.device, requires_grad=True)
        obj.training = True
        return obj

    # ---- nn.Module-like surface ----------------------------------------------------------
    def train(self, mode: bool = True):
        self.training = bool(mode)
        self.engine.set_training(self.training)
        return self

    def eval(self):
        return self.train(False)

    def to(self, device):
        if torch.device(device) != self.device:
            raise NotImplementedError("capgen: an engine is bound to the device it was created on")
        return self

    def parameters(self):
        return iter([self._anchor])

    def state_dict(self):
        return self.engine.state_dict()

    def load_state_dict(self, state_dict, strict=True):
        self.engine.load_state_dict(state_dict, strict=strict)

    # ---- reference API (model.py:79-209) ----------------------------------------------------
    def forward(self, object_features, position_features, target_caption):
        loss = self.engine.forward(object_features, position_features, target_caption)
        if torch.is_grad_enabled():
            loss = _EngineLoss.apply(self._anchor, loss, [self.engine])
        else:
            loss = loss.clone().reshape(())
        return {"loss": loss}

    __call__ = forward

    def generate_caption_vector(self, object_features, position_features):
        ids, attn = self.engine.greedy(object_features, position_features, want_attention=True)
        attn = attn.cpu().numpy()
        return ids, [attn[t] for t in range(attn.shape[0])]

    def beam_search(self, object_features, position_features, beam_size=1):
        return self.engine.beam(object_features, position_features, beam_size)

    def get_attention_key_pad_mask(self, k, q):
        """model.py:202-209 (host helper; the kernels derive the same mask on device)."""
        assert k.size(0) == q.size(0)
        mask = torch.count_nonzero(k, dim=2).eq(0)
        return mask.unsqueeze(1).expand(k.size(0), q.size(1), k.size(1))

    # ---- test hooks -----------------------------------------------------------------
    def logits(self, B, T):
        return self.engine.logits(B, T)

    def grads(self):
        return self.engine.grads_state_dict()


class PolicyNetwork(Transformer):
    """Drop-in for core/TRANSFORMER/model_RL.py:10-208 (the SCST model): the same encoder /
    decoder / classifer weights as Transformer, but `forward` returns the logits (model_RL.py:
    75-90), `sample` is argmax of LogSoftmax (:93-97), and decoding scores with LogSoftmax --
    greedy takes argmax of it and beam search accumulates LOG-probabilities (:72,126,157,182),
    where Transformer.beam_search adds probabilities (model.py:183)."""

    def __init__(self, num_vocab, max_length, encode_dim_positions, encode_dim_features, device, pad_idx=0,
                 dropout=0.2, encode_mask=False, encode_input_size=512, encode_q_k_dim=512, encode_v_dim=512,
                 encode_hidden_size=2048, encode_num_blocks=6, encode_num_heads=8, dim_word_embedding=512,
                 decode_input_size=512, decode_q_k_dim=512, decode_v_dim=512, decode_hidden_size=2048,
                 decode_num_blocks=6, decode_num_heads=8, move_first_image_feature=False, **kw):
        super().__init__(num_vocab, max_length, encode_dim_positions, encode_dim_features, device,
                         output_name="RL_Transformer", encode_mask=encode_mask, pad_idx=pad_idx, dropout=dropout,
                         encode_input_size=encode_input_size, encode_q_k_dim=encode_q_k_dim,
                         encode_v_dim=encode_v_dim, encode_hidden_size=encode_hidden_size,
                         encode_num_blocks=encode_num_blocks, encode_num_heads=encode_num_heads,
                         dim_word_embedding=dim_word_embedding, decode_input_size=decode_input_size,
                         decode_q_k_dim=decode_q_k_dim, decode_v_dim=decode_v_dim,
                         decode_hidden_size=decode_hidden_size, decode_num_blocks=decode_num_blocks,
                         decode_num_heads=decode_num_heads, move_first_image_feature=move_first_image_feature, **kw)
        self.engine.set_decode_log_softmax(True)

    @classmethod
    def from_config(cls, cfg: CapgenConfig, device, state_dict=None):
        obj = super().from_config(cfg, device, state_dict=state_dict)
        obj.engine.set_decode_log_softmax(True)
        return obj

    def forward(self, object_features, position_features, target_caption):
        """model_RL.py:75-90: teacher-forced logits [B, T-1, V] (f32, device)."""
        self.engine.forward(object_features, position_features, target_caption)
        B, T = target_caption.shape
        return self.engine.logits(B, T)

    __call__ = forward

    @staticmethod
    def sample(output):
        """model_RL.py:93-97: (argmax of log_softmax, log_softmax)."""
        log_probs = torch.log_softmax(output, dim=2)
        return torch.argmax(log_probs, dim=2), log_probs


class CapgenAdam:
    """optimizer.zero_grad()/step() for a capgen Transformer (torch.optim.Adam semantics,
    lr/betas/eps from the config).  zero_grad is free: backward overwrites the arena."""

    def __init__(self, model: Transformer):
        self.model = model

    def zero_grad(self, set_to_none=True):
        pass

    def step(self):
        self.model.engine.adam_step()
