"""Split-K combine stress test (diagnostic for the in-launch hand-off, gemm_bf16.hip gemm_tile).

Two DIFFERENT split-K GEMMs alternate on one stream, so they share the stream's slab workspace
and ticket array but leave different bytes in it; each output is compared bit for bit with the
first output of the same GEMM (the combine sums slices in a fixed order, so a correct hand-off
is bit-reproducible).  A second stream keeps the chip busy (uneven load), and the alternation
leaves the previous GEMM's slab lines warm in the combining CUs' caches (the guide's L1-warm
consumer condition, cdna_hip_programming.md Guideline 16 pitfall 3).

Usage: python tools/splitk_stress.py [pairs] [protocols...]   (protocol bits: include/capgen.h,
capgen_debug_splitk_protocol).  Prints one line per (protocol, variant): mismatching launches and
the average launch time of the pair.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402

lib = _lib.load()
DEV = "cuda:0"


def ptr(t):
    return C.c_void_p(t.data_ptr())


class G:
    """C[M,N] = A . op(B) through the engine's bf16 GEMM (NN layout: A [M][K], B [K][N])."""

    def __init__(self, M, N, K, seed):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.M, self.N, self.K = M, N, K
        self.A = torch.randn(M, K, generator=g).bfloat16().to(DEV)
        self.B = torch.randn(K, N, generator=g).bfloat16().to(DEV)
        self.C = torch.empty(M, N, dtype=torch.float32, device=DEV)
        self.ref = None

    def run(self, s):
        _lib.check(lib.capgen_debug_gemm(self.M, self.N, self.K, ptr(self.A), self.K, 0, ptr(self.B), self.N, 1,
                                         ptr(self.C), self.N, 1, 0, None, 1.0, 0, 0, C.c_void_p(s.cuda_stream)))


def timing(protos, variants):
    """Device time per GEMM of the three GEMMs per (protocol, variant): 20 launches of each
    captured into one graph and replayed (no host launch cost), two interleaved rounds."""
    cs = torch.cuda.Stream()
    gms = [G(2304, 512, 2048, 1), G(1216, 512, 2048, 2), G(2304, 512, 1536, 3)]
    for rnd in range(2):
        for v in variants:
            _lib.check(lib.capgen_debug_gemm_variant(v))
            row = []
            for proto in protos:
                _lib.check(lib.capgen_debug_splitk_protocol(proto))
                with torch.cuda.stream(cs):
                    for gm in gms:  # sizes this stream's split-K workspace outside the capture
                        gm.run(cs)
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=cs):
                    for _ in range(20):
                        for gm in gms:
                            gm.run(cs)
                graph.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    graph.replay()
                e1.record()
                torch.cuda.synchronize()
                row.append(f"p{proto}={e0.elapsed_time(e1) * 1e3 / 300:.2f}")
                del graph
            print(f"round {rnd} variant {v:4d} us/GEMM: " + " ".join(row), flush=True)
    _lib.check(lib.capgen_debug_gemm_variant(0))
    _lib.check(lib.capgen_debug_splitk_protocol(0))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "time":
        return timing([int(x) for x in sys.argv[2:]] or [22, 0, 8, 1], [17 + 800, 6 + 800, 3 + 800, 17 + 400,
                                                                          6 + 200, 17 + 200])
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    protos = [int(x) for x in sys.argv[2:]] or [22, 0]
    torch.cuda.init()
    s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    X = G(2304, 512, 2048, 1)   # encoder FFN dX shape
    Y = G(1216, 512, 2048, 2)   # decoder FFN dX shape
    Z = G(2304, 512, 1536, 3)   # encoder QKV dX shape
    big = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
    variants = [17 + 800, 6 + 800, 3 + 800, 17 + 400, 1 + 400]   # tile variant + 100 * split-K
    for proto in protos:
        _lib.check(lib.capgen_debug_splitk_protocol(proto))
        for v in variants:
            _lib.check(lib.capgen_debug_gemm_variant(v))
            for gm in (X, Y, Z):
                gm.run(s)
                torch.cuda.synchronize()
                gm.ref = gm.C.clone()
            bad = torch.zeros(3, dtype=torch.int64, device=DEV)
            # load on the side stream for the whole loop
            with torch.cuda.stream(side):
                for _ in range(pairs // 2):
                    big = (big @ big).clamp_(-1, 1)
            for it in range(pairs):
                for i, gm in enumerate((X, Y, Z)):
                    gm.C.fill_(float("nan"))  # a tile the combine skips cannot keep an old result
                    gm.run(s)
                    bad[i] += (gm.C != gm.ref).any().long()
            torch.cuda.synchronize()
            # launch time of the three GEMMs back to back, no load
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(50):
                for gm in (X, Y, Z):
                    gm.run(s)
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 150
            b = bad.tolist()
            print(f"proto {proto:2d} variant {v:4d}: mismatching launches X {b[0]}/{pairs} Y {b[1]}/{pairs} "
                  f"Z {b[2]}/{pairs}; {us:.2f} us per GEMM", flush=True)
    _lib.check(lib.capgen_debug_gemm_variant(0))
    _lib.check(lib.capgen_debug_splitk_protocol(0))


if __name__ == "__main__":
    main()
