"""Per-k-step cost of the bf16 GEMM tile loop: fixed variants, M x 512 outputs, K swept, normal vs
'neither' (no MFMA, no operand DMA: barrier + fragment reads + epilogue only).  Ablation build.

  CAPGEN_LIB_PATH=image-caption_amd/capgen/libcapgen_ablate.so python tools/gemm_kstep_sweep.py
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
os.environ.setdefault("CAPGEN_LIB_PATH", os.path.join(REPO, "image-caption_amd", "capgen", "libcapgen_ablate.so"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402

VARIANTS = {6: "64x64w4s2", 7: "64x64w4s3", 3: "128x128w4s2", 1: "128x128w4s3", 8: "128x64w8s2",
            10: "128x128w16s2", 21: "32x64w4s3", 12: "64x64w4s4"}


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    N = 512
    for M in (2048, 2304, 4096):
        for K in (64, 512, 2048):
            A = torch.randn(M * K, device=dev).to(torch.bfloat16)
            B = torch.randn(K * N, device=dev).to(torch.bfloat16)
            Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            row = {"M": M, "N": N, "K": K}
            for v, name in VARIANTS.items():
                _lib.check(lib.capgen_debug_gemm_variant(v))
                for mode, bits in (("n", 0), ("x", 3072), ("nd", 2048), ("nm", 1024)):
                    _lib.check(lib.capgen_debug_splitk_protocol(bits))

                    def launch():
                        _lib.check(lib.capgen_debug_gemm(M, N, K, C.c_void_p(A.data_ptr()), K, 0,
                                                         C.c_void_p(B.data_ptr()), K, 0, C.c_void_p(Cm.data_ptr()),
                                                         N, 1, 1, None, 1.0, 0, 0, C.c_void_p(s.cuda_stream)))
                    for _ in range(3):
                        launch()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(40):
                        launch()
                    e1.record(s)
                    e1.synchronize()
                    row[f"{name}:{mode}"] = round(e0.elapsed_time(e1) / 40 * 1e3, 2)
            _lib.check(lib.capgen_debug_splitk_protocol(0))
            _lib.check(lib.capgen_debug_gemm_variant(0))
            print(json.dumps(row), flush=True)
    # launch floor: an empty-ish kernel chain (the 1-block GEMM)
    A = torch.randn(64 * 64, device=dev).to(torch.bfloat16)
    Cm = torch.empty(64, 64, device=dev, dtype=torch.bfloat16)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(100):
        _lib.check(lib.capgen_debug_gemm(64, 64, 64, C.c_void_p(A.data_ptr()), 64, 0, C.c_void_p(A.data_ptr()), 64, 0,
                                         C.c_void_p(Cm.data_ptr()), 64, 1, 1, None, 1.0, 0, 0, C.c_void_p(s.cuda_stream)))
    e1.record(s)
    e1.synchronize()
    print(json.dumps({"one_tile_64x64x64_us": round(e0.elapsed_time(e1) / 100 * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
