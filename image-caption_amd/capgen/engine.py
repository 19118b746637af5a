"""Python handle over one libcapgen engine (one process, one device).

Thin: argument checking, dtype/layout normalisation of torch tensors, the
state_dict <-> packed-arena mapping, and current-stream plumbing.  All compute is in
libcapgen.so.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .config import CapgenConfig
from .params import PE_BUFFER, sinusoid_table


def _ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Engine:
    def __init__(self, cfg: CapgenConfig, device="cuda:0"):
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("capgen: the engine runs on a HIP device (cuda:N under ROCm)")
        self.lib = _lib.load()
        self._c = _lib.to_c_config(cfg)
        self.table, self.arena_elems = _lib.param_table(cfg)
        h = C.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        _lib.check(self.lib.capgen_create(C.byref(self._c), idx, C.byref(h)))
        self.h = h
        self.training = True
        self._loss = torch.zeros(1, dtype=torch.float32, device=self.device)

    def close(self):
        if getattr(self, "h", None):
            self.lib.capgen_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- module state -------------------------------------------------------------------
    def set_training(self, training: bool):
        self.training = bool(training)
        _lib.check(self.lib.capgen_set_training(self.h, int(self.training)))

    def set_decode_log_softmax(self, enable: bool):
        """PolicyNetwork decoding (model_RL.py:72,126,182): greedy / beam score with LogSoftmax and
        beams accumulate log-probabilities; False (default) = Transformer (Softmax, probabilities)."""
        _lib.check(self.lib.capgen_set_decode_log_softmax(self.h, int(enable)))

    def set_graph(self, enable: bool):
        _lib.check(self.lib.capgen_set_graph(self.h, int(enable)))

    def _arena_to_host(self, fn) -> np.ndarray:
        buf = np.empty(self.arena_elems, dtype=np.float32)
        _lib.check(fn(self.h, buf.ctypes.data_as(C.c_void_p), self.arena_elems))
        return buf

    def _unpack(self, arena: np.ndarray) -> "OrderedDict[str, torch.Tensor]":
        sd = OrderedDict()
        for name, ndim, rows, cols, off, stride in self.table:
            view = np.lib.stride_tricks.as_strided(arena[off:], shape=(rows, cols), strides=(stride * 4, 4))
            a = np.array(view, dtype=np.float32)
            sd[name] = torch.from_numpy(a if ndim == 2 else a.reshape(cols))
        return sd

    def state_dict(self, with_buffer: bool = True):
        """Reference-named f32 CPU tensors (checkpoint-compatible with model.py's keys)."""
        torch.cuda.current_stream(self.device).synchronize()
        sd = self._unpack(self._arena_to_host(self.lib.capgen_get_params))
        if with_buffer:
            sd[PE_BUFFER] = torch.from_numpy(sinusoid_table(self.cfg.max_length - 1, self.cfg.decode_input_size)[None])
        return sd

    def grads_state_dict(self):
        torch.cuda.current_stream(self.device).synchronize()
        return self._unpack(self._arena_to_host(self.lib.capgen_get_grads))

    def set_grads_arena(self, arena: np.ndarray):
        """Overwrite the whole f32 gradient arena (layout: capgen_param_table) from host memory."""
        a = np.ascontiguousarray(arena, dtype=np.float32)
        assert a.size == self.arena_elems
        torch.cuda.current_stream(self.device).synchronize()
        _lib.check(self.lib.capgen_set_grads(self.h, a.ctypes.data_as(C.c_void_p), self.arena_elems))

    def params_arena(self) -> np.ndarray:
        """The whole f32 parameter arena as a host copy."""
        torch.cuda.current_stream(self.device).synchronize()
        return self._arena_to_host(self.lib.capgen_get_params)

    def set_params_arena(self, arena: np.ndarray):
        """Overwrite the whole f32 parameter arena (and the bf16 shadow) from host memory."""
        a = np.ascontiguousarray(arena, dtype=np.float32)
        assert a.size == self.arena_elems
        torch.cuda.current_stream(self.device).synchronize()
        _lib.check(self.lib.capgen_set_params(self.h, a.ctypes.data_as(C.c_void_p), self.arena_elems))

    def grads_arena(self) -> np.ndarray:
        """The whole f32 gradient arena as a host copy."""
        torch.cuda.current_stream(self.device).synchronize()
        return self._arena_to_host(self.lib.capgen_get_grads)

    def load_state_dict(self, sd, strict: bool = True):
        arena = np.zeros(self.arena_elems, dtype=np.float32)
        seen = set()
        for name, ndim, rows, cols, off, stride in self.table:
            if name not in sd:
                if strict:
                    raise KeyError(f"capgen: missing key {name!r} in state_dict")
                continue
            v = sd[name]
            v = v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, np.float32)
            want = (rows, cols) if ndim == 2 else (cols,)
            if tuple(v.shape) != want:
                raise ValueError(f"capgen: {name}: shape {tuple(v.shape)} != {want}")
            view = np.lib.stride_tricks.as_strided(arena[off:], shape=(rows, cols), strides=(stride * 4, 4))
            view[...] = v.reshape(rows, cols)
            seen.add(name)
        if strict:
            extra = set(sd) - seen - {PE_BUFFER}
            if extra:
                raise KeyError(f"capgen: unexpected keys in state_dict: {sorted(extra)[:5]}")
        torch.cuda.current_stream(self.device).synchronize()
        _lib.check(self.lib.capgen_set_params(self.h, arena.ctypes.data_as(C.c_void_p), self.arena_elems))

    def adam_state(self):
        step = C.c_int64(0)
        m = np.empty(self.arena_elems, np.float32)
        v = np.empty(self.arena_elems, np.float32)
        _lib.check(self.lib.capgen_get_adam_state(self.h, C.byref(step), m.ctypes.data_as(C.c_void_p),
                                                  v.ctypes.data_as(C.c_void_p), self.arena_elems))
        return step.value, self._unpack(m), self._unpack(v)

    # ---- inputs ----------------------------------------------------------------------
    def _inputs(self, feats, pos, caps=None):
        dev = self.device
        if feats.dtype not in (torch.float32, torch.bfloat16):
            feats = feats.float()
        feats = feats.to(dev, non_blocking=True).contiguous()
        pos = pos.to(dev, dtype=torch.float32, non_blocking=True).contiguous()
        if feats.dim() != 3 or pos.dim() != 3 or feats.shape[:2] != pos.shape[:2]:
            raise ValueError("capgen: object_features [B,N,F] and position_features [B,N,P] must agree")
        if feats.shape[2] != self.cfg.encode_dim_features or pos.shape[2] != self.cfg.encode_dim_positions:
            raise ValueError("capgen: feature widths do not match the config")
        ft = _lib.BF16 if feats.dtype == torch.bfloat16 else _lib.F32
        if caps is not None:
            caps = caps.to(dev, dtype=torch.int32, non_blocking=True).contiguous()
            if caps.dim() != 2 or caps.shape[0] != feats.shape[0]:  # model.py:203
                raise ValueError("capgen: target_caption must be [B, T] with the batch of the features")
        return feats, ft, pos, caps

    # ---- hot path --------------------------------------------------------------------
    def forward(self, feats, pos, caps, loss_out=None):
        f, ft, p, c = self._inputs(feats, pos, caps)
        B, N, _ = f.shape
        out = self._loss if loss_out is None else loss_out
        _lib.check(self.lib.capgen_forward(self.h, _ptr(f), ft, _ptr(p), _ptr(c), B, N, c.shape[1], _ptr(out),
                                           _stream(self.device)))
        return out

    def backward(self):
        _lib.check(self.lib.capgen_backward(self.h, _stream(self.device)))

    def adam_step(self):
        _lib.check(self.lib.capgen_adam_step(self.h, _stream(self.device)))

    def train_step(self, feats, pos, caps, loss_out=None):
        f, ft, p, c = self._inputs(feats, pos, caps)
        B, N, _ = f.shape
        out = self._loss if loss_out is None else loss_out
        _lib.check(self.lib.capgen_train_step(self.h, _ptr(f), ft, _ptr(p), _ptr(c), B, N, c.shape[1], _ptr(out),
                                              _stream(self.device)))
        return out

    def train_step_raw(self, f, ft, p, c, B, N, T, out):
        """Pre-normalised device tensors (bench loop): no checks, no copies."""
        _lib.check(self.lib.capgen_train_step(self.h, _ptr(f), ft, _ptr(p), _ptr(c), B, N, T, _ptr(out),
                                              _stream(self.device)))

    def train_step_indexed(self, feat_store, pos_store, img_idx, caps, out=None):
        """Training step reading features of images img_idx[b] from device-resident stores
        (capgen.data.DeviceFeatureStore): no per-step host->device copy of features."""
        assert feat_store.is_cuda and pos_store.is_cuda and img_idx.is_cuda and caps.is_cuda
        assert feat_store.dim() == 3 and pos_store.shape[:2] == feat_store.shape[:2]
        ft = _lib.BF16 if feat_store.dtype == torch.bfloat16 else _lib.F32
        idx = img_idx.to(torch.int32).contiguous()
        c = caps.to(torch.int32).contiguous()
        B, T = c.shape
        out = self._loss if out is None else out
        _lib.check(self.lib.capgen_train_step_indexed(self.h, _ptr(feat_store), ft, _ptr(pos_store),
                                                      feat_store.shape[0], _ptr(idx), _ptr(c), B,
                                                      feat_store.shape[1], T, _ptr(out), _stream(self.device)))
        return out

    def compute_loss(self, feats, pos, caps):
        out = torch.zeros(1, dtype=torch.float32, device=self.device)
        f, ft, p, c = self._inputs(feats, pos, caps)
        B, N, _ = f.shape
        _lib.check(self.lib.capgen_compute_loss(self.h, _ptr(f), ft, _ptr(p), _ptr(c), B, N, c.shape[1], _ptr(out),
                                                _stream(self.device)))
        return out

    def logits(self, B, T):
        out = torch.empty(B * (T - 1), self.cfg.num_vocab, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.capgen_copy_logits(self.h, _ptr(out), out.numel(), _stream(self.device)))
        return out.view(B, T - 1, -1)

    def greedy(self, feats, pos, want_attention=True):
        f, ft, p, _ = self._inputs(feats, pos)
        B, N, _ = f.shape
        T = self.cfg.max_length
        ids = torch.empty(B, T + 1, dtype=torch.int64, device=self.device)
        attn = torch.empty(T - 1, B, N, dtype=torch.float32, device=self.device) if want_attention else None
        _lib.check(self.lib.capgen_greedy(self.h, _ptr(f), ft, _ptr(p), B, N, _ptr(ids), _ptr(attn),
                                          _stream(self.device)))
        return ids, attn

    def beam(self, feats, pos, beam_size):
        f, ft, p, _ = self._inputs(feats, pos)
        B, N, _ = f.shape
        ids = torch.empty(B, self.cfg.max_length, dtype=torch.int64, device=self.device)
        _lib.check(self.lib.capgen_beam(self.h, _ptr(f), ft, _ptr(p), B, N, int(beam_size), _ptr(ids),
                                        _stream(self.device)))
        return ids

    # ---- SCST (SelfCriticNetwork) -------------------------------------------------------
    def rl_sample(self, feats, pos, caps):
        """Teacher-forced forward + PolicyNetwork.sample (model_RL.py:75-97): returns
        (sample int64 [B, T-1], per-image masked mean entropy f32 [B], LM CE loss f32 [1])."""
        f, ft, p, c = self._inputs(feats, pos, caps)
        B, N, _ = f.shape
        T = c.shape[1]
        seq = torch.empty(B, T - 1, dtype=torch.int64, device=self.device)
        ent = torch.empty(B, dtype=torch.float32, device=self.device)
        lm = torch.empty(1, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.capgen_rl_sample(self.h, _ptr(f), ft, _ptr(p), _ptr(c), B, N, T, _ptr(seq), _ptr(ent),
                                             _ptr(lm), _stream(self.device)))
        return seq, ent, lm

    def rl_finish(self, scores, structure_loss_weight: float, train: bool = True):
        """ReinforcementLearningLoss (loss.py:53-76) on the last rl_sample, with per-image total
        scores [B]; train=True also runs backward + Adam.  Returns {loss, lm, struct} [3]."""
        sc = torch.as_tensor(scores, dtype=torch.float32).to(self.device).contiguous()
        out = torch.empty(3, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.capgen_rl_finish(self.h, _ptr(sc), float(structure_loss_weight), _ptr(out), int(train),
                                             _stream(self.device)))
        return out

    def set_rng_seed(self, seed: int):
        _lib.check(self.lib.capgen_set_rng_seed(self.h, seed & 0xFFFFFFFFFFFFFFFF))

    # ---- data parallel -----------------------------------------------------------------
    @staticmethod
    def dp_unique_id() -> bytes:
        lib = _lib.load()
        buf = C.create_string_buffer(128)
        _lib.check(lib.capgen_dp_unique_id(buf))
        return buf.raw

    def dp_init(self, uid: bytes, rank: int, world: int):
        assert len(uid) == 128
        _lib.check(self.lib.capgen_dp_init(self.h, uid, rank, world))

    def dp_comm_info(self):
        """(communicator size, this rank) of the engine's RCCL communicator; (0, 0) before dp_init."""
        n, r = C.c_int(0), C.c_int(0)
        _lib.check(self.lib.capgen_dp_comm_info(self.h, C.byref(n), C.byref(r)))
        return n.value, r.value

    def dp_check(self, loss: torch.Tensor | None = None):
        """Run the data-parallel consistency check now (collective over the engine communicator, any
        world size): every rank's global non-pad count and loss must agree (max == min); raises
        RuntimeError otherwise.  `loss`: the [1] f32 device tensor the last step wrote (None = the
        engine's internal loss).  The step runs the same check once by itself at world > 1."""
        _lib.check(self.lib.capgen_dp_check(self.h, _ptr(loss), _stream(self.device)))

    def params_checksum(self) -> int:
        """Exact, order-independent checksum of the f32 parameters (equal on every rank of a DP run)."""
        v = C.c_uint64(0)
        _lib.check(self.lib.capgen_params_checksum(self.h, C.byref(v)))
        return v.value

    def dp_set_global_count(self, count: float):
        _lib.check(self.lib.capgen_dp_set_global_count(self.h, float(count)))

    def dp_sync_adam_state(self):
        """Collective (every rank): all-gather the sharded Adam moments (see capgen.h)."""
        _lib.check(self.lib.capgen_dp_sync_adam_state(self.h))

    def dp_buckets(self):
        """The last train step's gradient buckets as [(offset, count)] over the parameter arena."""
        cap = 256
        offs = np.zeros(cap, np.int64)
        cnts = np.zeros(cap, np.int64)
        n = C.c_int(0)
        _lib.check(self.lib.capgen_dp_buckets(self.h, offs.ctypes.data_as(C.c_void_p),
                                              cnts.ctypes.data_as(C.c_void_p), cap, C.byref(n)))
        return [(int(offs[i]), int(cnts[i])) for i in range(n.value)]

    def collectives_log(self, op: int, cap: int = 1 << 16) -> str:
        """Test hook: 1 = start recording the engine's RCCL calls, 0 = stop, 2 = the recorded calls."""
        buf = C.create_string_buffer(cap)
        _lib.check(self.lib.capgen_debug_collectives(self.h, int(op), buf, cap))
        return buf.value.decode()

    def stamps(self, op: int):
        """Diagnostic un-profiled timeline (capgen_debug_stamps): op 1 on, 0 off, 3 arm; op 2 returns
        [(name, start_us, end_us)] of the last step's stamped launches (unlaunched slots: 0, 0)."""
        cap = 8192
        out = np.zeros(2 * cap, np.float64)
        names = C.create_string_buffer(1 << 20)
        n = self.lib.capgen_debug_stamps(self.h, int(op), out.ctypes.data_as(C.c_void_p), 2 * cap, names, 1 << 20)
        if n < 0:
            _lib.check(1)
        if op != 2:
            return None
        lines = names.value.decode().split("\n")
        return [(lines[i], out[2 * i], out[2 * i + 1]) for i in range(n)]

    def dp_debug_shard(self, rank: int, world: int):
        """Test hook: update as rank `rank` of `world` would under the sharded update, no collectives."""
        _lib.check(self.lib.capgen_dp_debug_shard(self.h, int(rank), int(world)))
