"""Cycle breakdown of one bf16 GEMM workgroup (wave 0 of block 0): kernel start, prologue DMA issue,
then for each of the first 8 k-steps: DMA wait -> barrier -> next-stage DMA issue -> fragment reads +
MFMAs, then the loop end and the epilogue.  s_memtime deltas (shader clock) and the in-kernel clock
(s_memtime / s_memrealtime).  Ablation build, protocol bit 4096 (gemm_bf16.hip ABL_T).

  make -C image-caption_amd/csrc ablate && python tools/gemm_phase_timing.py
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

CASES = [  # (variant, name, M, N, K, tb)
    (7, "64x64w4s3 NT", 2304, 512, 2048, 0), (7, "64x64w4s3 NN", 2304, 512, 2048, 1),
    (21, "32x64w4s3 NT", 2304, 512, 2048, 0), (8, "128x64w8s2 NT", 2304, 512, 2048, 0),
    (1, "128x128w4s3 NT", 2304, 512, 2048, 0), (7, "64x64w4s3 NT K512", 2304, 512, 512, 0),
]


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    buf = torch.zeros(128, dtype=torch.int64, device=dev)
    _lib.check(lib.capgen_debug_gemm_timing_buf(C.c_void_p(buf.data_ptr())))
    for v, name, M, N, K, tb in CASES:
        A = torch.randn(M * K, device=dev).to(torch.bfloat16)
        B = torch.randn(K * N, device=dev).to(torch.bfloat16)
        Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        _lib.check(lib.capgen_debug_gemm_variant(v))
        for mode, bits in (("normal", 0), ("no_dma", 2048), ("no_mfma", 1024), ("neither", 3072)):
            def launch(extra):
                _lib.check(lib.capgen_debug_splitk_protocol(bits | extra))
                _lib.check(lib.capgen_debug_gemm(M, N, K, C.c_void_p(A.data_ptr()), K, 0, C.c_void_p(B.data_ptr()),
                                                 N if tb else K, tb, C.c_void_p(Cm.data_ptr()), N, 1, 1, None, 1.0, 0, 0,
                                                 C.c_void_p(s.cuda_stream)))
            for _ in range(5):
                launch(0)
            buf.zero_()
            launch(4096)
            torch.cuda.synchronize()
            t = buf.cpu().tolist()
            mt = [t[16 + 2 * i] for i in range(36)]
            rt = [t[17 + 2 * i] for i in range(36)]
            clk = (mt[35] - mt[0]) / max(1, rt[35] - rt[0]) * 0.1  # GHz (100 MHz real-time counter)
            steps = []
            for k in range(8):
                b = 2 + 4 * k
                if mt[b + 3] == 0:
                    break
                prev = mt[b - 1] if k else mt[1]
                steps.append([mt[b] - prev, mt[b + 1] - mt[b], mt[b + 2] - mt[b + 1], mt[b + 3] - mt[b + 2]])
            out = {"case": name, "mode": mode, "clock_ghz": round(clk, 3), "total_us": round((rt[35] - rt[0]) * 0.01, 2),
                   "setup+prologue_cyc": mt[1] - mt[0], "loop_cyc": mt[34] - mt[1], "epilogue_cyc": mt[35] - mt[34],
                   "kstep_cyc[wait,barrier,issue,mfma]": steps[1:6]}
            print(json.dumps(out), flush=True)
    _lib.check(lib.capgen_debug_splitk_protocol(0))
    _lib.check(lib.capgen_debug_gemm_variant(0))
    _lib.check(lib.capgen_debug_gemm_timing_buf(None))


if __name__ == "__main__":
    main()
