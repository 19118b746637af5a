"""Library reference: torch.matmul (hipBLASLt) time for the train step's GEMM shapes, beside
capgen's tuned kernel (capgen_debug_gemm, autotuned).  Diagnostic only."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402

SHAPES = [  # M, N, K, ta, tb, f32out  (capgen convention: NT fwd, NN dX (tb), TN dW (ta, tb))
    (2304, 1536, 512, 0, 0, 0), (2304, 512, 512, 0, 0, 0), (2304, 2048, 512, 0, 0, 0), (2304, 512, 2048, 0, 0, 0),
    (2304, 512, 2176, 0, 0, 0), (2304, 6144, 512, 0, 0, 0), (1216, 10000, 512, 0, 0, 1),
    (2304, 512, 1536, 0, 1, 0), (2304, 2048, 512, 0, 1, 0), (2304, 512, 2048, 0, 1, 0), (2304, 512, 6144, 0, 1, 0),
    (1216, 512, 10000, 0, 1, 0),
    (1536, 512, 2304, 1, 1, 1), (512, 512, 2304, 1, 1, 1), (2048, 512, 2304, 1, 1, 1), (512, 2048, 2304, 1, 1, 1),
    (6144, 512, 2304, 1, 1, 1), (10000, 512, 1216, 1, 1, 1),
]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


lib = _lib.load()
for (M, N, K, ta, tb, f32) in SHAPES:
    A = torch.randn((K, M) if ta else (M, K), device="cuda", dtype=torch.bfloat16)
    B = torch.randn((K, N) if tb else (N, K), device="cuda", dtype=torch.bfloat16)
    opA = A.t() if ta else A
    opB = B if tb else B.t()
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
    if f32:
        t_lib = timeit(lambda: torch.matmul(opA.float(), opB.float(), out=out)) if False else \
            timeit(lambda: out.copy_(torch.matmul(opA, opB)))
    else:
        t_lib = timeit(lambda: torch.matmul(opA, opB, out=out))
    s = torch.cuda.current_stream()
    Cc = torch.empty(M, N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
    t_cg = timeit(lambda: _lib.check(lib.capgen_debug_gemm(
        M, N, K, C.c_void_p(A.data_ptr()), M if ta else K, ta, C.c_void_p(B.data_ptr()), N if tb else K, tb,
        C.c_void_p(Cc.data_ptr()), N, 1, 0 if f32 else 1, None, 1.0, 0, 0, C.c_void_p(s.cuda_stream))))
    fl = 2 * M * N * K
    print(f"M={M:5d} N={N:5d} K={K:5d} ta={ta} tb={tb} f32={f32}: hipBLASLt {t_lib:7.2f} us "
          f"({fl / t_lib / 1e6:6.1f} TF/s)   capgen {t_cg:7.2f} us ({fl / t_cg / 1e6:6.1f} TF/s)", flush=True)
