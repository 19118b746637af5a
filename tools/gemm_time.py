"""Isolated time of the library's bf16 GEMM (capgen_debug_gemm, the tuned variant of each shape)
for the input-gradient (NN: dX[M,N] = dY[M,K] . W[K,N]) shapes of the C2 step; companion of
tools/breg_probe.hip (same shapes, same launch count).

  python tools/gemm_time.py [--reps 200]
"""
import argparse
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
from capgen import _lib  # noqa: E402

SHAPES = [(2304, 512, 2048), (1216, 512, 2048), (2304, 512, 1536), (1216, 512, 1536), (2304, 2048, 512),
          (1216, 2048, 512), (2304, 512, 512), (1216, 512, 512)]
# the C4 decode step's forward (NT) GEMMs: beam 5 x 256 images = 1280 rows, greedy 256 rows
DECODE = [(1280, 512, 512), (1280, 1536, 512), (1280, 2048, 512), (1280, 512, 2048), (256, 512, 512),
          (256, 1536, 512), (256, 2048, 512), (256, 512, 2048)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--decode", action="store_true", help="the decode step's NT shapes (Y = X . W^T)")
    a = ap.parse_args()
    lib = _lib.load()
    dev = "cuda:0"
    for M, N, K in (DECODE if a.decode else SHAPES):
        A = torch.randn(M, K, device=dev).bfloat16()
        W = torch.randn(N, K, device=dev).bfloat16() if a.decode else torch.randn(K, N, device=dev).bfloat16()
        Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        tb, ldb = (0, K) if a.decode else (1, N)

        def go():
            _lib.check(lib.capgen_debug_gemm(M, N, K, C.c_void_p(A.data_ptr()), K, 0, C.c_void_p(W.data_ptr()), ldb, tb,
                                             C.c_void_p(Cm.data_ptr()), N, 1, 1, None, 1.0, 0, 0, None))

        go()
        torch.cuda.synchronize()
        ref = A.float() @ (W.float().t() if a.decode else W.float())
        err = ((Cm.float() - ref).abs().max() / ref.abs().max()).item()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            go()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(f"library            M={M:5d} N={N:5d} K={K:5d}  {us:7.2f} us  {2.0 * M * N * K / us * 1e-6:6.1f} TF/s  "
              f"max|err|/max|ref| {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
