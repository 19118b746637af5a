"""ctypes binding of libcapgen.so (the C ABI declared in include/capgen.h).

The library is loaded AFTER `import torch`, so its NEEDED libamdhip64.so.7 resolves to
the HIP runtime torch already mapped: device pointers, streams and events are shared
with PyTorch.  There is no fallback: if the library is missing, importing the engine
raises, loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CAPGEN_LIB_PATH") or os.path.join(_HERE, "libcapgen.so")  # (diagnostic builds)
ABI_VERSION = 11

F32, BF16 = 0, 1


class capgen_config(C.Structure):
    _fields_ = [
        ("num_vocab", C.c_int32), ("max_length", C.c_int32),
        ("dim_features", C.c_int32), ("dim_positions", C.c_int32),
        ("enc_d", C.c_int32), ("enc_ff", C.c_int32), ("enc_blocks", C.c_int32), ("enc_heads", C.c_int32),
        ("dim_word_embedding", C.c_int32),
        ("dec_d", C.c_int32), ("dec_ff", C.c_int32), ("dec_blocks", C.c_int32), ("dec_heads", C.c_int32),
        ("dropout", C.c_float), ("attention_dropout", C.c_float),
        ("pad_idx", C.c_int32), ("encode_mask", C.c_int32), ("focal_loss", C.c_int32),
        ("split_position", C.c_int32), ("split_image_objects", C.c_int32),
        ("move_first_image_feature", C.c_int32),
        ("dtype", C.c_int32), ("max_batch", C.c_int32), ("max_regions", C.c_int32),
        ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
        ("seed", C.c_uint64),
    ]


class capgen_param_info(C.Structure):
    _fields_ = [("name", C.c_char * 96), ("ndim", C.c_int32), ("rows", C.c_int64), ("cols", C.c_int64),
                ("offset", C.c_int64), ("row_stride", C.c_int64)]


_P = C.c_void_p
_SIGS = {
    "capgen_last_error": (C.c_char_p, []),
    "capgen_abi_version": (C.c_int, []),
    "capgen_set_knob": (C.c_int, [C.c_char_p, C.c_int, _P]),
    "capgen_debug_build": (C.c_int, []),
    "capgen_param_table": (C.c_int, [C.POINTER(capgen_config), C.POINTER(capgen_param_info), C.c_int,
                                     C.POINTER(C.c_int), C.POINTER(C.c_int64)]),
    "capgen_create": (C.c_int, [C.POINTER(capgen_config), C.c_int, C.POINTER(_P)]),
    "capgen_destroy": (C.c_int, [_P]),
    "capgen_get_params": (C.c_int, [_P, _P, C.c_int64]),
    "capgen_set_params": (C.c_int, [_P, _P, C.c_int64]),
    "capgen_get_grads": (C.c_int, [_P, _P, C.c_int64]),
    "capgen_set_grads": (C.c_int, [_P, _P, C.c_int64]),
    "capgen_get_adam_state": (C.c_int, [_P, C.POINTER(C.c_int64), _P, _P, C.c_int64]),
    "capgen_set_adam_state": (C.c_int, [_P, C.c_int64, _P, _P, C.c_int64]),
    "capgen_arenas": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_int64)]),
    "capgen_set_training": (C.c_int, [_P, C.c_int]),
    "capgen_set_graph": (C.c_int, [_P, C.c_int]),
    "capgen_set_decode_log_softmax": (C.c_int, [_P, C.c_int]),
    "capgen_forward": (C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "capgen_backward": (C.c_int, [_P, _P]),
    "capgen_adam_step": (C.c_int, [_P, _P]),
    "capgen_train_step": (C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "capgen_compute_loss": (C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "capgen_copy_logits": (C.c_int, [_P, _P, C.c_int64, _P]),
    "capgen_greedy": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, C.c_int, _P, _P, _P]),
    "capgen_beam": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "capgen_set_rng_seed": (C.c_int, [_P, C.c_uint64]),
    "capgen_debug_gemm": (C.c_int, [C.c_int, C.c_int, C.c_int, _P, C.c_int64, C.c_int, _P, C.c_int64, C.c_int,
                                    _P, C.c_int64, C.c_int, C.c_int, _P, C.c_float, C.c_int, C.c_int, _P]),
    "capgen_debug_gemm_tiled": (C.c_int, [C.c_int, C.c_int, C.c_int, _P, C.c_int64, _P, C.c_int64, C.c_int, _P, _P,
                                          C.c_int64, C.c_int, _P, C.c_int, C.c_int, _P, C.c_int64, _P]),
    "capgen_debug_gemm_tiled_ln": (C.c_int, [C.c_int, C.c_int, _P, _P, _P, _P, _P, C.c_int, _P, C.c_int, C.c_int, _P, _P,
                                             _P, _P, C.c_int64, C.c_int, _P]),
    "capgen_debug_gemm_variant": (C.c_int, [C.c_int]),
    "capgen_debug_splitk_protocol": (C.c_int, [C.c_int]),
    "capgen_debug_splitk_diag": (C.c_int, [_P, C.c_int]),
    "capgen_debug_gemm_timing_buf": (C.c_int, [_P]),
    "capgen_debug_copy_buffer": (C.c_int, [_P, C.c_int, _P, C.c_int64]),
    "capgen_train_step_indexed": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P,
                                            _P]),
    "capgen_rl_sample": (C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P]),
    "capgen_rl_finish": (C.c_int, [_P, _P, C.c_float, _P, C.c_int, _P]),
    "capgen_debug_attention": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P,
                                         C.c_int, C.c_float, _P, _P, _P, _P, _P, _P, _P]),
    "capgen_debug_attention_bwd_wo": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int, _P, _P,
                                                _P, _P, _P, _P]),
    "capgen_debug_qkv_attention": (C.c_int, [C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, C.c_int, C.c_int, _P]),
    "capgen_debug_cross_attention": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, _P]),
    "capgen_dp_unique_id": (C.c_int, [C.c_char_p]),
    "capgen_dp_init": (C.c_int, [_P, C.c_char_p, C.c_int, C.c_int]),
    "capgen_dp_set_global_count": (C.c_int, [_P, C.c_float]),
    "capgen_dp_sync_adam_state": (C.c_int, [_P]),
    "capgen_dp_comm_info": (C.c_int, [_P, _P, _P]),
    "capgen_dp_check": (C.c_int, [_P, _P, _P]),
    "capgen_params_checksum": (C.c_int, [_P, _P]),
    "capgen_dp_buckets": (C.c_int, [_P, _P, _P, C.c_int, _P]),
    "capgen_dp_debug_shard": (C.c_int, [_P, C.c_int, C.c_int]),
    "capgen_tune_load": (C.c_int, [C.c_char_p]),
    "capgen_tune_save": (C.c_int, [C.c_char_p]),
    "capgen_tune_live_count": (C.c_int, []),
    "capgen_debug_hazard": (C.c_int, [C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int)]),
    "capgen_debug_side_delay": (C.c_int, [C.c_double]),
    "capgen_debug_collectives": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_int]),
    "capgen_debug_stamps": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_char_p, C.c_int]),
    "capgen_scst_rewards": (C.c_int, [_P, C.c_int64, _P, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int64, C.c_double, C.c_double, _P]),
}
EXPORTED = tuple(_SIGS)

_lib = None


def load():
    """dlopen libcapgen.so once; raises if it was not built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"capgen: {LIB_PATH} is missing — build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (make -C image-caption_amd/csrc)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.capgen_abi_version() != ABI_VERSION:
        raise ImportError("capgen: libcapgen.so ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError("capgen: " + load().capgen_last_error().decode(errors="replace"))


def to_c_config(cfg) -> capgen_config:
    cfg.check_supported()
    c = capgen_config()
    c.num_vocab, c.max_length = cfg.num_vocab, cfg.max_length
    c.dim_features, c.dim_positions = cfg.encode_dim_features, cfg.encode_dim_positions
    c.enc_d, c.enc_ff = cfg.encode_input_size, cfg.encode_hidden_size
    c.enc_blocks, c.enc_heads = cfg.encode_num_blocks, cfg.encode_num_heads
    c.dim_word_embedding = cfg.dim_word_embedding
    c.dec_d, c.dec_ff = cfg.decode_input_size, cfg.decode_hidden_size
    c.dec_blocks, c.dec_heads = cfg.decode_num_blocks, cfg.decode_num_heads
    c.dropout, c.attention_dropout = cfg.dropout, cfg.attention_dropout
    c.pad_idx, c.encode_mask, c.focal_loss = cfg.pad_idx, int(cfg.encode_mask), int(cfg.focal_loss)
    c.split_position = int(cfg.split_position)
    c.split_image_objects = int(cfg.split_image_objects)
    c.move_first_image_feature = int(cfg.move_first_image_feature)
    c.dtype = F32 if cfg.dtype == "fp32" else BF16
    c.max_batch, c.max_regions = cfg.max_batch, cfg.max_regions
    c.lr, c.beta1, c.beta2, c.eps = cfg.learning_rate, cfg.beta1, cfg.beta2, cfg.eps
    c.seed = cfg.seed & 0xFFFFFFFFFFFFFFFF
    return c


def param_table(cfg):
    """[(name, ndim, rows, cols, offset, row_stride)], arena_elems — host-only, no GPU needed."""
    lib = load()
    c = to_c_config(cfg)
    n = C.c_int(0)
    total = C.c_int64(0)
    check(lib.capgen_param_table(C.byref(c), None, 0, C.byref(n), C.byref(total)))
    arr = (capgen_param_info * n.value)()
    check(lib.capgen_param_table(C.byref(c), arr, n.value, C.byref(n), C.byref(total)))
    out = [(p.name.decode(), p.ndim, p.rows, p.cols, p.offset, p.row_stride) for p in arr]
    return out, total.value


TUNE_TABLE = os.path.join(_HERE, "tune_gfx950.txt")


def tune_save(path: str = TUNE_TABLE) -> int:
    """Write every GEMM autotune choice this process knows (tuned or loaded) to `path`."""
    n = load().capgen_tune_save(path.encode())
    if n < 0:
        check(1)
    return n


def tune_load(path: str) -> int:
    """Merge a persisted autotune table (-1: no such file)."""
    return load().capgen_tune_load(path.encode())


def tune_live_count() -> int:
    """GEMM shapes this process tuned live (0 when the persisted table covered every shape)."""
    return load().capgen_tune_live_count()


def hazard_start() -> None:
    """Start logging every launch / event / host sync of the engines (clears the log)."""
    check(load().capgen_debug_hazard(1, None, 0, None))


def hazard_stop() -> None:
    check(load().capgen_debug_hazard(0, None, 0, None))


def hazard_check(cap: int = 8192):
    """(number of unordered conflicting launch pairs since hazard_start, report text)."""
    buf = C.create_string_buffer(cap)
    n = C.c_int(0)
    check(load().capgen_debug_hazard(2, buf, cap, C.byref(n)))
    return n.value, buf.value.decode(errors="replace")


def side_delay(us: float) -> None:
    """Spin `us` microseconds in front of every launch off the critical stream (0 = off)."""
    check(load().capgen_debug_side_delay(float(us)))


def set_knob(name: str, value: int) -> int:
    """Set a run-time switch (capgen_set_knob; name without the CAPGEN_ prefix); returns the old value."""
    old = C.c_int(0)
    check(load().capgen_set_knob(name.encode(), int(value), C.byref(old)))
    return old.value


def debug_build() -> bool:
    """True in the debug library (libcapgen_debug.so, CAPGEN_LIB_PATH)."""
    return bool(load().capgen_debug_build())
