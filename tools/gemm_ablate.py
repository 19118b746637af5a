"""Where a bf16 GEMM of the C2 step spends its time: each step shape with its tuned variant, timed
normal / without the MFMAs / without the operand DMA / with neither (the launch + setup + epilogue
intercept), warm (back to back) and cold (a 64 MB scrub before each launch, the tuner's clock).

Needs the ablation build:  make -C image-caption_amd/csrc ablate
  CAPGEN_LIB_PATH=image-caption_amd/capgen/libcapgen_ablate.so python tools/gemm_ablate.py
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

SHAPES = [  # (name, M, N, K, ta, tb)
    ("fwd enc QKV", 2304, 1536, 512, 0, 0), ("fwd enc Wo", 2304, 512, 512, 0, 0),
    ("fwd enc W1", 2304, 2048, 512, 0, 0), ("fwd enc W2", 2304, 512, 2048, 0, 0),
    ("fwd enc emb", 2304, 512, 2176, 0, 0), ("fwd Wkv_all", 2304, 6144, 512, 0, 0),
    ("fwd dec QKV", 1216, 1536, 512, 0, 0), ("fwd dec Wo", 1216, 512, 512, 0, 0),
    ("fwd dec W1", 1216, 2048, 512, 0, 0), ("fwd dec W2", 1216, 512, 2048, 0, 0),
    ("dX enc QKV", 2304, 512, 1536, 0, 1), ("dX enc Wo", 2304, 512, 512, 0, 1),
    ("dX enc W2", 2304, 2048, 512, 0, 1), ("dX enc W1", 2304, 512, 2048, 0, 1),
    ("dX Wkv_all", 2304, 512, 6144, 0, 1), ("dX dec QKV", 1216, 512, 1536, 0, 1),
    ("dX dec Wo", 1216, 512, 512, 0, 1), ("dX dec W2", 1216, 2048, 512, 0, 1),
    ("dX dec W1", 1216, 512, 2048, 0, 1), ("dX classifier", 1216, 512, 10000, 0, 1),
]
MODES = {"normal": 0, "no_mfma": 1024, "no_dma": 2048, "neither": 3072}


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    scrub = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    out = []
    for name, M, N, K, ta, tb in SHAPES:
        A = torch.randn(M * K, device=dev).to(torch.bfloat16)
        B = torch.randn(K * N, device=dev).to(torch.bfloat16)
        Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        lda = M if ta else K
        ldb = N if tb else K

        def launch():
            _lib.check(lib.capgen_debug_gemm(M, N, K, C.c_void_p(A.data_ptr()), lda, ta, C.c_void_p(B.data_ptr()), ldb,
                                             tb, C.c_void_p(Cm.data_ptr()), N, 1, 1, None, 1.0, 0, 0,
                                             C.c_void_p(s.cuda_stream)))
        row = {"shape": name, "M": M, "N": N, "K": K, "gflop": 2e-9 * M * N * K}
        for mode, bits in MODES.items():
            _lib.check(lib.capgen_debug_splitk_protocol(bits))
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(30):
                launch()
            e1.record(s)
            e1.synchronize()
            row[mode + "_warm_us"] = round(e0.elapsed_time(e1) / 30 * 1e3, 2)
            tot = 0.0
            for r in range(10):
                scrub.fill_(r)
                e0.record(s)
                launch()
                e1.record(s)
                e1.synchronize()
                tot += e0.elapsed_time(e1)
            row[mode + "_cold_us"] = round(tot / 10 * 1e3, 2)
        _lib.check(lib.capgen_debug_splitk_protocol(0))
        row["normal_warm_tflops"] = round(row["gflop"] / row["normal_warm_us"] * 1e3, 1)
        print(json.dumps(row), flush=True)
        out.append(row)
    with open(os.path.join(REPO, "gpurun_out", "gemm_ablate.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
