"""Reference parameter names/shapes and host-side initialisers.

`reference_param_specs` lists the reference `Transformer.state_dict()` entries in
their registration order (core/TRANSFORMER/model.py:44-69, modules.py:42-62 and
100-107, model.py:232-255 and 389-417), so checkpoints interoperate with the
reference (SURVEY.md §5 "Checkpoint / resume", including the misspelled
`classifer.*`).  The engine keeps its own packed arena layout (see
include/capgen.h `capgen_param_table`); this module only knows reference names.
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import numpy as np

from .config import CapgenConfig


def _mha_specs(prefix, d):
    return [(f"{prefix}.q_linear.weight", (d, d)), (f"{prefix}.k_linear.weight", (d, d)),
            (f"{prefix}.v_linear.weight", (d, d)), (f"{prefix}.layer_norm.weight", (d,)),
            (f"{prefix}.layer_norm.bias", (d,)), (f"{prefix}.joint_linear.weight", (d, d))]


def _ffn_specs(prefix, d, f):
    return [(f"{prefix}.position_wise_1.weight", (f, d)), (f"{prefix}.position_wise_1.bias", (f,)),
            (f"{prefix}.position_wise_2.weight", (d, f)), (f"{prefix}.position_wise_2.bias", (d,)),
            (f"{prefix}.layer_norm.weight", (d,)), (f"{prefix}.layer_norm.bias", (d,))]


def reference_param_specs(cfg: CapgenConfig):
    """[(name, shape)] of trainable parameters, reference registration order."""
    d, f = cfg.encode_input_size, cfg.encode_hidden_size
    P = cfg.encode_dim_positions
    if cfg.split_position:  # model.py:231-233: object_embedding registered first
        specs = [("encoder.object_embedding.weight", (d, P - 4)), ("encoder.position_embedding.weight", (d, 4))]
    else:
        specs = [("encoder.position_embedding.weight", (d, P))]
    if cfg.split_image_objects:  # model.py:237-244: encoder.image_encoder registered next
        specs += _mha_specs("encoder.image_encoder.multihead_attention", d)
        specs += _ffn_specs("encoder.image_encoder.feed_forward", d, f)
    specs += [("encoder.feature_embedding.weight", (d, cfg.encode_dim_features)),
             ("encoder.norm.weight", (d,)), ("encoder.norm.bias", (d,))]
    for i in range(cfg.encode_num_blocks):
        specs += _mha_specs(f"encoder.encoder.{i}.multihead_attention", d)
        specs += _ffn_specs(f"encoder.encoder.{i}.feed_forward", d, f)
    dd, df = cfg.decode_input_size, cfg.decode_hidden_size
    specs += [("decoder.word_embedding.weight", (cfg.num_vocab, cfg.dim_word_embedding)),
              ("decoder.word_embedding_linear.weight", (dd, cfg.dim_word_embedding)),
              ("decoder.norm.weight", (dd,)), ("decoder.norm.bias", (dd,))]
    if cfg.move_first_image_feature:  # model.py:400-407
        specs += [("decoder.position_wise_1.weight", (df, dd)), ("decoder.position_wise_1.bias", (df,)),
                  ("decoder.position_wise_2.weight", (dd, df)), ("decoder.position_wise_2.bias", (dd,)),
                  ("decoder.layer_norm.weight", (dd,)), ("decoder.layer_norm.bias", (dd,))]
    for i in range(cfg.decode_num_blocks):
        specs += _mha_specs(f"decoder.decoder.{i}.self_attention", dd)
        specs += _mha_specs(f"decoder.decoder.{i}.encode_attention", dd)
        specs += _ffn_specs(f"decoder.decoder.{i}.feed_forward", dd, df)
    specs += [("classifer.weight", (cfg.num_vocab, dd)), ("classifer.bias", (cfg.num_vocab,))]
    return specs


PE_BUFFER = "decoder.position_embedding.pos_table"


def sinusoid_table(num_positions: int, d: int) -> np.ndarray:
    """Sinusoid position table of model.py:502-514: built in float64, cast to float32.
    angle(pos, j) = pos / 10000^(2*(j//2)/d); sin on even j, cos on odd j."""
    pos = np.arange(num_positions, dtype=np.float64)[:, None]
    j = np.arange(d)
    angle = pos / np.power(10000, 2 * (j // 2) / d)
    table = np.empty_like(angle)
    table[:, 0::2] = np.sin(angle[:, 0::2])
    table[:, 1::2] = np.cos(angle[:, 1::2])
    return table.astype(np.float32)


def num_params(cfg: CapgenConfig) -> int:
    return sum(int(np.prod(s)) for _, s in reference_param_specs(cfg))


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.default_rng([seed & 0xFFFFFFFF, zlib.crc32(name.encode())])


def fixture_state_dict(cfg: CapgenConfig, seed: int = 0, with_buffer: bool = True):
    """Deterministic closed-form weights used by the golden fixtures and the parity
    tests: every tensor is drawn from PCG64 seeded by (seed, crc32(name)),
    so the fixtures need not carry weights.  Scales keep activations O(1)."""
    sd = OrderedDict()
    for name, shape in reference_param_specs(cfg):
        r = _rng(seed, name)
        if name.endswith("layer_norm.weight") or name.endswith("norm.weight"):
            a = 1.0 + 0.1 * r.standard_normal(shape)
        elif name.endswith(".bias"):
            a = 0.05 * r.standard_normal(shape)
        elif name == "decoder.word_embedding.weight":
            a = r.standard_normal(shape)
            a[cfg.pad_idx] = 0.0          # nn.Embedding(padding_idx) zeroes the pad row
        else:
            a = r.standard_normal(shape) / math.sqrt(shape[1])
        sd[name] = a.astype(np.float32)
    if with_buffer:
        sd[PE_BUFFER] = sinusoid_table(cfg.max_length - 1, cfg.decode_input_size)[None]
    return sd


def reference_init_state_dict(cfg: CapgenConfig, seed: int = 0, with_buffer: bool = True):
    """Random init with the reference's distributions: q/k/v N(0, sqrt(2/(in+out)))
    (modules.py:45-53), xavier_normal for joint/FFN/classifier (modules.py:62,102-103,
    model.py:69), nn.Linear default U(+-1/sqrt(fan_in)) for embeddings/biases,
    nn.Embedding N(0,1) with a zero pad row, LayerNorm ones/zeros."""
    sd = OrderedDict()
    for name, shape in reference_param_specs(cfg):
        r = _rng(seed, name)
        if name.endswith("norm.weight"):
            a = np.ones(shape)
        elif name.endswith("norm.bias"):
            a = np.zeros(shape)
        elif name == "decoder.word_embedding.weight":
            a = r.standard_normal(shape)
            a[cfg.pad_idx] = 0.0
        elif any(name.endswith(s) for s in ("q_linear.weight", "k_linear.weight", "v_linear.weight",
                                             "joint_linear.weight", "position_wise_1.weight",
                                             "position_wise_2.weight")) or name == "classifer.weight":
            a = r.standard_normal(shape) * math.sqrt(2.0 / (shape[0] + shape[1]))
        elif name.endswith(".bias"):
            wshape = dict(reference_param_specs(cfg))[name[:-4] + "weight"]
            bound = 1.0 / math.sqrt(wshape[1])
            a = r.uniform(-bound, bound, shape)
        else:
            bound = 1.0 / math.sqrt(shape[1])
            a = r.uniform(-bound, bound, shape)
        sd[name] = a.astype(np.float32)
    if with_buffer:
        sd[PE_BUFFER] = sinusoid_table(cfg.max_length - 1, cfg.decode_input_size)[None]
    return sd
