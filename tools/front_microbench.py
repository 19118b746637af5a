"""Isolated cost of the fused attention front (qkv_attn.hip) against the pair it replaces, at the C2
step's shapes: encoder self-attention (64 images x 36 rows, key-valid + causal off), decoder
self-attention (64 x 19, key ids + causal), decoder cross front (64 x 19 queries over 36 keys).

  fused : capgen_debug_qkv_attention / capgen_debug_cross_attention (one launch)
  pair  : capgen_debug_gemm (the projection) + capgen_debug_attention (the MFMA attention)

Each timed with HIP events over 200 back-to-back launches after a warm-up (L2-warm: a lower bound of
the in-step cost).  Prints one JSON line per shape."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    H, d = 8, 512
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, B, L, Lk, cross in (("enc self 64x36", 64, 36, 36, False), ("dec self 64x19", 64, 19, 19, False),
                                  ("dec cross 64x19x36", 64, 19, 36, True)):
        X = (torch.randn(B * L, d, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        W = (torch.randn(3 * d, d, generator=g) / d ** 0.5).to(torch.bfloat16).to(dev)
        qkv = torch.empty(B * L, 3 * d, device=dev, dtype=torch.bfloat16)
        o = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
        if cross:
            KV = (torch.randn(B * Lk, 2 * d, generator=g)).to(torch.bfloat16).to(dev)
            q = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
            valid = torch.ones(B, Lk, dtype=torch.uint8, device=dev)
            Wq = W[:d].contiguous()
            fused = lambda: lib.capgen_debug_cross_attention(B, L, Lk, H, p(X), p(Wq), p(KV), p(q), p(o), p(valid), None)
            k = torch.randn(B * Lk, d, generator=g).to(torch.bfloat16).to(dev)  # (packed copies: the hook
            v = torch.randn(B * Lk, d, generator=g).to(torch.bfloat16).to(dev)  # takes row stride H * 64)

            def pair():
                lib.capgen_debug_gemm(B * L, d, d, p(X), d, 0, p(Wq), d, 0, p(q), d, 1, 1, None, 1.0, 0, 0, None)
                lib.capgen_debug_attention(1, B, H, L, Lk, 64, p(q), p(k), p(v), p(valid), 0, 8.0, p(o), None, None,
                                           None, None, None, None)
        else:
            ids = torch.randint(3, 100, (B, L), generator=g, dtype=torch.int32).to(dev)
            fused = lambda: lib.capgen_debug_qkv_attention(B, L, H, p(X), p(W), p(qkv), p(o), None, p(ids), 0, 1, None)
            # (the attention hook takes packed [B, L, H * 64] tensors: separate buffers of the same size)
            qv, kv_, vv = (torch.randn(B * L, d, generator=g).to(torch.bfloat16).to(dev) for _ in range(3))

            def pair():
                lib.capgen_debug_gemm(B * L, 3 * d, d, p(X), d, 0, p(W), d, 0, p(qkv), 3 * d, 1, 1, None, 1.0, 0, 0,
                                      None)
                lib.capgen_debug_attention(1, B, H, L, L, 64, p(qv), p(kv_), p(vv), None, 1, 8.0, p(o), None, None,
                                           None, None, None, None)
        tf, tp = timed(fused), timed(pair)
        print(json.dumps({"shape": name, "fused_us": round(tf, 2), "pair_us": round(tp, 2)}), flush=True)


if __name__ == "__main__":
    main()
