"""GEMM microbenchmark via the capgen_debug_gemm test hook (run under rocprofv3 for
exact per-dispatch durations, or standalone for event timing)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402

lib = _lib.load()


def run(M, N, K, ta=0, tb=0, out_f32=False, reps=20, bias=False, relu=False):
    A = torch.randn((K, M) if ta else (M, K), device="cuda", dtype=torch.bfloat16)
    B = torch.randn((K, N) if tb else (N, K), device="cuda", dtype=torch.bfloat16)
    Cc = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    b = torch.zeros(N, device="cuda")
    def args():
        s = torch.cuda.current_stream()
        return (M, N, K, C.c_void_p(A.data_ptr()), M if ta else K, ta, C.c_void_p(B.data_ptr()), N if tb else K, tb,
                C.c_void_p(Cc.data_ptr()), N, 1, 0 if out_f32 else 1, C.c_void_p(b.data_ptr()) if bias else None,
                1.0, 0, int(relu), C.c_void_p(s.cuda_stream))
    g = torch.cuda.CUDAGraph()
    global _CS
    if "_CS" not in globals():
        _CS = torch.cuda.Stream()
    with torch.cuda.stream(_CS):  # warm-up on the capture stream: sizes its split-K workspace
        _lib.check(lib.capgen_debug_gemm(*args()))
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=_CS):
        for _ in range(reps):
            _lib.check(lib.capgen_debug_gemm(*args()))
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    tf = 2 * M * N * K / (us * 1e-6) / 1e12
    print(f"M={M:6d} N={N:6d} K={K:6d} ta={ta} tb={tb} f32={int(out_f32)}  {us:8.2f} us  {tf:7.1f} TF/s", flush=True)
    return us


def sweep():
    shapes = [(2304, 2048, 512, 0, 0, 0), (4096, 4096, 4096, 0, 0, 0), (2304, 6144, 512, 0, 0, 0),
              (2048, 512, 2304, 1, 1, 1), (2304, 512, 2048, 0, 1, 0), (1216, 512, 512, 0, 1, 0)]
    for v in range(0, 10):
        _lib.check(lib.capgen_debug_gemm_variant(v))
        print(f"--- variant {v}")
        for sh in shapes:
            try:
                run(*sh)
            except RuntimeError as e:
                print("  skip", e)
    _lib.check(lib.capgen_debug_gemm_variant(0))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "lat":
    for (M, N, K, v) in [(64, 64, 64, 6), (64, 64, 4096, 6), (64, 64, 4096, 7), (128, 128, 4096, 3),
                         (128, 128, 4096, 1), (256, 128, 4096, 9), (16384, 64, 4096, 6), (16384, 64, 4096, 7),
                         (16384, 128, 4096, 3), (16384, 128, 4096, 1), (32768, 128, 4096, 9)]:
        _lib.check(lib.capgen_debug_gemm_variant(v))
        print(f"v{v}", end=" ")
        run(M, N, K, 0, 0, 0)
elif __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "one":
    M, N, K, ta, tb, f32, v = map(int, sys.argv[2:9])
    _lib.check(lib.capgen_debug_gemm_variant(v))
    run(M, N, K, ta, tb, f32)
elif __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "kscan":
    # per-tile cost model: exactly 256 tiles (one per CU), time vs K -> slope (per 64-deep
    # K step) and intercept (fixed per-tile overhead)
    for (v, M, N) in [(6, 1024, 1024), (12, 1024, 1024), (3, 2048, 2048), (1, 2048, 2048), (16, 2048, 2048)]:
        _lib.check(lib.capgen_debug_gemm_variant(v + 100))
        for K in (64, 128, 256, 512, 1024, 2048, 4096):
            us = run(M, N, K, 0, 0, 0, reps=20)
        print(f"--- variant {v}", flush=True)
    _lib.check(lib.capgen_debug_gemm_variant(0))
elif __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sk":
    # split-K study: eager launches (the split-K workspace is per stream), event timing
    shapes = [(512, 512, 2304, 1, 1, 1), (2048, 512, 2304, 1, 1, 1), (2304, 512, 2048, 0, 0, 0),
              (2304, 512, 2048, 0, 1, 0), (1216, 512, 10000, 0, 1, 0)]
    variants = (6, 12, 13, 14, 8)
    for (M, N, K, ta, tb, f32) in shapes:
        A = torch.randn((K, M) if ta else (M, K), device="cuda", dtype=torch.bfloat16)
        B = torch.randn((K, N) if tb else (N, K), device="cuda", dtype=torch.bfloat16)
        Cc = torch.empty(M, N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
        ref = None
        for v in variants:
            for sk in (1, 2, 3, 4, 6):
                _lib.check(lib.capgen_debug_gemm_variant(v + 100 * sk))
                s = torch.cuda.current_stream()
                call = lambda: _lib.check(lib.capgen_debug_gemm(
                    M, N, K, C.c_void_p(A.data_ptr()), M if ta else K, ta, C.c_void_p(B.data_ptr()), N if tb else K,
                    tb, C.c_void_p(Cc.data_ptr()), N, 1, 0 if f32 else 1, None, 1.0, 0, 0, C.c_void_p(s.cuda_stream)))
                for _ in range(5):
                    call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    call()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 50
                out = Cc.float()
                if ref is None:
                    ref = out.clone()
                err = (out - ref).abs().max().item() / ref.abs().max().item()
                print(f"M={M} N={N} K={K} ta={ta} tb={tb} v={v} sk={sk}: {us:7.2f} us "
                      f"{2 * M * N * K / us / 1e6:6.1f} TF/s  rel.diff {err:.1e}", flush=True)
    _lib.check(lib.capgen_debug_gemm_variant(0))
elif __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "nnnt":
    # forward (NT) vs input-gradient (NN) layout on the step's shapes, autotuned variant, alone
    for (M, N, K) in [(2304, 2048, 512), (2304, 512, 2048), (2304, 1536, 512), (2304, 512, 1536), (2304, 512, 512),
                      (1216, 2048, 512), (1216, 512, 2048), (1216, 1536, 512), (1216, 512, 1536), (1216, 512, 512),
                      (1216, 512, 10000)]:
        for tb in (0, 1):
            run(M, N, K, 0, tb, 0)
elif __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sweep":
    sweep()
elif __name__ == "__main__" and len(sys.argv) == 1:
    shapes = [(2304, 2048, 512, 0, 0, 0), (2304, 2048, 2048, 0, 0, 0), (2304, 2048, 8192, 0, 0, 0),
              (4096, 4096, 4096, 0, 0, 0), (2304, 6144, 512, 0, 0, 0), (1216, 10000, 512, 0, 0, 1),
              (1216, 512, 512, 0, 1, 0), (2304, 512, 2048, 0, 1, 0), (2048, 512, 2304, 1, 1, 1),
              (512, 512, 2304, 1, 1, 1), (1216, 512, 10000, 0, 1, 0), (512, 2176, 2304, 1, 1, 1)]
    for sh in shapes:
        run(*sh)


def matrix(shapes, sks=(1, 2, 4, 8), variants=range(1, 23)):
    """Every (variant, split-K) on each shape, graph-replayed (device time per launch)."""
    for sh in shapes:
        res = []
        for v in variants:
            for sk in sks:
                _lib.check(lib.capgen_debug_gemm_variant(v + 100 * sk))
                try:
                    us = run(*sh, reps=20)
                    res.append((us, v, sk))
                except RuntimeError as e:
                    print("  skip", v, sk, e)
        res.sort()
        print(f"best for {sh}: " + ", ".join(f"v{v}x{sk} {us:.2f}" for us, v, sk in res[:6]), flush=True)
    _lib.check(lib.capgen_debug_gemm_variant(0))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "matrix2":
    matrix([(1216, 512, 10000, 0, 1, 0), (2304, 512, 6144, 0, 1, 0), (1216, 10000, 512, 0, 0, 1)],
           variants=(1, 3, 4, 5, 6, 8, 10, 17, 20))
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "matrix":
    matrix([(2304, 512, 2048, 0, 1, 0), (2304, 2048, 512, 0, 0, 0), (2304, 512, 512, 0, 0, 0),
            (1216, 512, 2048, 0, 1, 0), (2304, 1536, 512, 0, 0, 0)])
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "matrix3":
    # decoder-side shapes (M = 64 x 19 = 1216 rows)
    matrix([(1216, 512, 2048, 0, 0, 0), (1216, 512, 2048, 0, 1, 0), (1216, 2048, 512, 0, 1, 0),
            (1216, 512, 512, 0, 0, 0), (1216, 512, 512, 0, 1, 0)], sks=(1, 2, 3, 4))


def cold(shapes, choices):
    """Event-timed eager launches, each after a 64 MB scrub write (the autotuner's cold-L2 clock)."""
    scrub = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    for (M, N, K, ta, tb, f32) in shapes:
        A = torch.randn((K, M) if ta else (M, K), device="cuda", dtype=torch.bfloat16)
        Bm = torch.randn((K, N) if tb else (N, K), device="cuda", dtype=torch.bfloat16)
        Cc = torch.empty(M, N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
        res = []
        for ch in choices:
            _lib.check(lib.capgen_debug_gemm_variant(ch))
            s = torch.cuda.current_stream()
            call = lambda: _lib.check(lib.capgen_debug_gemm(
                M, N, K, C.c_void_p(A.data_ptr()), M if ta else K, ta, C.c_void_p(Bm.data_ptr()), N if tb else K,
                tb, C.c_void_p(Cc.data_ptr()), N, 1, 0 if f32 else 1, None, 1.0, 0, 0, C.c_void_p(s.cuda_stream)))
            call()
            tot = 0.0
            for r in range(10):
                scrub.fill_(r)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                call()
                e1.record()
                e1.synchronize()
                tot += e0.elapsed_time(e1) * 1e3
            res.append((tot / 10, ch))
        _lib.check(lib.capgen_debug_gemm_variant(0))
        print(f"M={M} N={N} K={K} ta={ta} tb={tb}: " + ", ".join(f"v{c % 100}x{max(1, c // 100)} {us:.2f}"
                                                           for us, c in sorted(res)), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "cold":
    # the LN-producing shapes (N = d = 512) under the tuner's cold-L2 clock
    # (profiles/r02_fullrow_probe.txt also ranked a since-removed 32x512 full-row variant here)
    cold([(2304, 512, 512, 0, 0, 0), (1216, 512, 512, 0, 0, 0), (2304, 512, 2048, 0, 0, 0),
          (1216, 512, 2048, 0, 0, 0), (2304, 512, 2048, 0, 1, 0), (1216, 512, 512, 0, 1, 0)],
         [7, 21, 6, 12, 17, 207, 221, 307])
