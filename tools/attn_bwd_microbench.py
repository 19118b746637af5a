"""Isolated kernel durations of the fused attention-backward output side (qkv_attn_bwd) against the
pair it replaces (the dX GEMM dO = dA . Wo, then the MFMA attention backward), at the C2 step's
shapes: encoder self 64 x 36, decoder self 64 x 19 (causal), decoder cross 64 x 19 over 36 keys.
Each hook runs 100 times back to back; run under `rocprofv3 --kernel-trace --stats` and read the
per-kernel averages (the fused hook also re-tiles Wo per call: a separate small kernel)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    H, d = 8, 512
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    g = torch.Generator(device="cpu").manual_seed(0)
    rnd = lambda *s: (torch.randn(*s, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    reps = int(os.environ.get("REPS", "100"))
    for B, Lq, Lk, causal in ((64, 36, 36, 0), (64, 19, 19, 1), (64, 19, 36, 0)):
        q, dA, dq, dO = rnd(B * Lq, d), rnd(B * Lq, d), rnd(B * Lq, d), rnd(B * Lq, d)
        k, v, dk, dv = rnd(B * Lk, d), rnd(B * Lk, d), rnd(B * Lk, d), rnd(B * Lk, d)
        o = rnd(B * Lq, d)
        Wo = (torch.randn(d, d, generator=g) / d ** 0.5).to(torch.bfloat16).to(dev)
        valid = torch.ones(B, Lk, dtype=torch.uint8, device=dev)
        for _ in range(reps):
            lib.capgen_debug_attention_bwd_wo(B, Lq, Lk, H, p(q), p(k), p(v), p(valid), causal, p(dA), p(Wo), p(dq),
                                              p(dk), p(dv), None)
        for _ in range(reps):
            # dO = dA . Wo  (NN: B operand transposed)
            lib.capgen_debug_gemm(B * Lq, d, d, p(dA), d, 0, p(Wo), d, 1, p(dO), d, 1, 1, None, 1.0, 0, 0, None)
            lib.capgen_debug_attention(1, B, H, Lq, Lk, 64, p(q), p(k), p(v), p(valid), causal, 8.0, p(o), None,
                                       p(dO), p(dq), p(dk), p(dv), None)
        torch.cuda.synchronize()
        print(f"done B={B} Lq={Lq} Lk={Lk}", flush=True)


if __name__ == "__main__":
    main()
