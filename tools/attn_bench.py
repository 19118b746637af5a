"""Attention kernel timings through capgen_debug_attention (event-timed, bf16)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402

lib = _lib.load()
for (B, H, Lq, Lk, causal) in [(64, 8, 36, 36, 0), (64, 8, 19, 19, 1), (64, 8, 19, 36, 0)]:
    dk = 64
    q, k, v, do = (torch.randn(B, L, H * dk, device="cuda", dtype=torch.bfloat16) for L in (Lq, Lk, Lk, Lq))
    valid = torch.ones(B, Lk, dtype=torch.uint8, device="cuda")
    o = torch.empty_like(q)
    dq, dkk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    P = lambda t: C.c_void_p(t.data_ptr())
    s = torch.cuda.current_stream()
    for mode in ("fwd", "fwd+bwd"):
        def call():
            _lib.check(lib.capgen_debug_attention(1, B, H, Lq, Lk, dk, P(q), P(k), P(v), P(valid), causal, 8.0, P(o),
                                                  None, P(do) if mode != "fwd" else None, P(dq), P(dkk), P(dv),
                                                  C.c_void_p(s.cuda_stream)))
        for _ in range(10):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            call()
        e1.record()
        e1.synchronize()
        print(f"B={B} H={H} Lq={Lq} Lk={Lk} {mode}: {e0.elapsed_time(e1) * 10:.2f} us", flush=True)
