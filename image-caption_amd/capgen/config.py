"""Model / solver configuration for the capgen engine.

Field names follow the keyword arguments of the reference `Transformer.__init__`
(core/TRANSFORMER/model.py:10-36) and the constants of core/config.py:5-62, so a
reference config module can be turned into a `CapgenConfig` one-to-one
(`from_reference_constants`).  The presets C1/C2 are SURVEY.md §8 configs.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass
class CapgenConfig:
    # vocabulary / lengths (model.py:10-11; models.py:86-87 passes MAX_LENGTH+2)
    num_vocab: int = 10000
    max_length: int = 20
    # encoder inputs (config.py:51-56)
    encode_dim_features: int = 2048
    encode_dim_positions: int = 84
    # encoder (model.py:19-24)
    encode_input_size: int = 512
    encode_q_k_dim: int = 512
    encode_v_dim: int = 512
    encode_hidden_size: int = 2048
    encode_num_blocks: int = 6
    encode_num_heads: int = 8
    # decoder (model.py:26-32)
    dim_word_embedding: int = 512
    decode_input_size: int = 512
    decode_q_k_dim: int = 512
    decode_v_dim: int = 512
    decode_hidden_size: int = 2048
    decode_num_blocks: int = 6
    decode_num_heads: int = 8
    # regularisation / misc (model.py:15-17, modules.py:8)
    dropout: float = 0.2
    attention_dropout: float = 0.1      # hard-coded in ScaledDotProductAttention
    pad_idx: int = 0
    encode_mask: bool = False
    output_name: str = "Transformer"    # 'FocalLoss' substring selects FocalLoss (model.py:73)
    # variants that exist in the reference but are not on the measured path
    move_first_image_feature: bool = False
    split_position: bool = False
    split_image_objects: bool = False
    # solver (config.py:59-62, models.py:111-113; torch.optim.Adam defaults)
    learning_rate: float = 5e-4
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    # engine-only knobs
    dtype: str = "bf16"                 # "fp32" (parity mode) or "bf16" (perf mode)
    max_batch: int = 256                # workspace sizing (images per call)
    max_regions: int = 37               # N upper bound (NUM_OBJECT+1)
    seed: int = 1234

    @property
    def focal_loss(self) -> bool:
        return self.output_name.find("FocalLoss") != -1

    def replace(self, **kw) -> "CapgenConfig":
        return dataclasses.replace(self, **kw)

    def check_supported(self) -> None:
        """Raise NotImplementedError for reference variants the engine does not build."""
        if self.split_position and self.split_image_objects:
            raise NotImplementedError("capgen: split_position with split_image_objects fails in the reference "
                                      "itself (model.py:258-292 feeds the full position row to Linear(4, d))")
        if self.encode_input_size != self.decode_input_size:
            raise NotImplementedError("capgen: encoder and decoder widths must match "
                                      "(cross-attention K/V are projected from the encoder output)")
        for pre in ("encode", "decode"):
            d = getattr(self, f"{pre}_input_size")
            qk = getattr(self, f"{pre}_q_k_dim")
            v = getattr(self, f"{pre}_v_dim")
            h = getattr(self, f"{pre}_num_heads")
            if qk != d or v != d:
                raise NotImplementedError("capgen: q_k_dim / v_dim must equal input_size")
            if d % h or (d // h) % 8 or d // h > 128:
                raise NotImplementedError("capgen: head size must be a multiple of 8 and <= 128")
            if d % 64:
                raise NotImplementedError("capgen: model width must be a multiple of 64")
        if self.max_length - 1 > 64 or self.max_regions > 64:
            raise NotImplementedError("capgen: sequence lengths above 64 are not supported")
        if self.num_vocab % 8:
            raise NotImplementedError("capgen: num_vocab must be a multiple of 8")
        if self.dtype not in ("fp32", "bf16"):
            raise ValueError(f"capgen: dtype must be 'fp32' or 'bf16', got {self.dtype!r}")


def preset(name: str, **overrides) -> CapgenConfig:
    """SURVEY.md §8 configs. C1: CPU plumbing shape; C2: the 1-GPU headline shape."""
    if name == "C1":
        cfg = CapgenConfig(num_vocab=1000, max_length=10, encode_dim_features=512,
                           encode_input_size=128, encode_q_k_dim=128, encode_v_dim=128,
                           encode_hidden_size=512, encode_num_blocks=2, encode_num_heads=4,
                           dim_word_embedding=128, decode_input_size=128, decode_q_k_dim=128,
                           decode_v_dim=128, decode_hidden_size=512, decode_num_blocks=2,
                           decode_num_heads=4, max_batch=64, max_regions=8)
    elif name in ("C2", "C3", "C4", "C5"):
        cfg = CapgenConfig(max_regions=36)
    else:
        raise KeyError(name)
    return cfg.replace(**overrides)


# shape of one batch for a preset: (B, N, T)
PRESET_BATCH = {"C1": (8, 8, 10), "C2": (64, 36, 20), "C3": (64, 36, 20), "C4": (256, 36, 20)}


def from_reference_constants(ns, num_vocab: int, dtype: str = "bf16") -> CapgenConfig:
    """Build a config from a namespace holding the reference core/config.py constants
    (the exact mapping of core/models.py:86-110)."""
    g = ns if isinstance(ns, dict) else vars(ns)
    return CapgenConfig(
        num_vocab=num_vocab, max_length=g["MAX_LENGTH"] + 2,
        encode_dim_positions=g["ENCODE_DIM_POSITIONS"], encode_dim_features=g["ENCODE_DIM_FEATURES"],
        encode_input_size=g["ENCODE_INPUT_SIZE"], encode_q_k_dim=g["ENCODE_Q_K_DIM"],
        encode_v_dim=g["ENCODE_V_DIM"], encode_hidden_size=g["ENCODE_HIDDEN_SIZE"],
        encode_num_blocks=g["ENCODE_NUM_BLOCKS"], encode_num_heads=g["ENCODE_NUM_HEADS"],
        dim_word_embedding=g["DIM_WORD_EMBEDDING"], decode_input_size=g["DECODE_INPUT_SIZE"],
        decode_q_k_dim=g["DECODE_Q_K_DIM"], decode_v_dim=g["DECODE_V_DIM"],
        decode_hidden_size=g["DECODE_HIDDEN_SIZE"], decode_num_blocks=g["DECODE_NUM_BLOCKS"],
        decode_num_heads=g["DECODE_NUM_HEADS"], dropout=g["DROPOUT"], pad_idx=g["PAD_IDX"],
        encode_mask=g.get("ENCODE_MASK", False), output_name=g.get("OUTPUT_NAME", "Transformer"),
        move_first_image_feature=g.get("MOVE_FIRST_IMAGE_FAETURE", False),
        split_position=g.get("SPLIT_POSITION", False),
        split_image_objects=g.get("SPLIT_IMAGE_OBJECTS", False),
        learning_rate=g.get("LEARNING_RATE", 5e-4), dtype=dtype,
        max_batch=max(256, g.get("BATCH_SIZE", 32)), max_regions=g.get("NUM_OBJECT", 36) + 1)
