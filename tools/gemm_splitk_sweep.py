"""GPU-only timing (hipGraph replay, no host launch cost) of the step's GEMM shapes over tile variant x
split-K, against the tuned choice (capgen/tune_gfx950.txt).  The per-workgroup k-loop is latency-bound
(tools/gemm_kstep_sweep.py: time independent of M), so split-K is the lever for K-deep shapes.

  python tools/gemm_splitk_sweep.py [--variants 1,7 --splits 1 --out x.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402

SHAPES = [  # (name, M, N, K, ta, tb)
    ("fwd enc W2", 2304, 512, 2048, 0, 0), ("fwd enc QKV", 2304, 1536, 512, 0, 0),
    ("fwd enc W1", 2304, 2048, 512, 0, 0), ("fwd enc Wo", 2304, 512, 512, 0, 0),
    ("fwd enc emb", 2304, 512, 2176, 0, 0), ("fwd Wkv_all", 2304, 6144, 512, 0, 0),
    ("fwd dec W2", 1216, 512, 2048, 0, 0), ("fwd dec QKV", 1216, 1536, 512, 0, 0),
    ("fwd dec W1", 1216, 2048, 512, 0, 0), ("fwd dec Wo", 1216, 512, 512, 0, 0),
    ("dX enc W1", 2304, 512, 2048, 0, 1), ("dX enc QKV", 2304, 512, 1536, 0, 1),
    ("dX enc W2", 2304, 2048, 512, 0, 1), ("dX enc Wo", 2304, 512, 512, 0, 1),
    ("dX Wkv_all", 2304, 512, 6144, 0, 1), ("dX dec W1", 1216, 512, 2048, 0, 1),
    ("dX dec QKV", 1216, 512, 1536, 0, 1), ("dX dec W2", 1216, 2048, 512, 0, 1),
    ("dX dec Wo", 1216, 512, 512, 0, 1), ("dX classifier", 1216, 512, 10000, 0, 1),
]
VARIANTS = [1, 3, 4, 5, 6, 7, 8, 10, 12, 17, 20, 21, 23, 24, 25, 26, 27, 28, 29, 30]
SPLITS = [1, 2, 3, 4, 6, 8]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default=",".join(map(str, VARIANTS)))
    ap.add_argument("--splits", default=",".join(map(str, SPLITS)))
    ap.add_argument("--out", default="gemm_splitk_sweep.json")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",") if v]
    splits = [int(v) for v in args.splits.split(",") if v]
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    out = []
    for name, M, N, K, ta, tb in SHAPES:
        A = torch.randn(M * K, device=dev).to(torch.bfloat16)
        B = torch.randn(K * N, device=dev).to(torch.bfloat16)
        Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        lda, ldb = (M if ta else K), (N if tb else K)
        s = torch.cuda.Stream(dev)

        def launch():
            _lib.check(lib.capgen_debug_gemm(M, N, K, C.c_void_p(A.data_ptr()), lda, ta, C.c_void_p(B.data_ptr()), ldb,
                                             tb, C.c_void_p(Cm.data_ptr()), N, 1, 1, None, 1.0, 0, 0,
                                             C.c_void_p(s.cuda_stream)))

        def graph_time():
            with torch.cuda.stream(s):
                launch()  # outside the capture: workspaces, tuning
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(args.reps):
                        launch()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(3):
                    g.replay()
                e1.record(s)
                e1.synchronize()
                return e0.elapsed_time(e1) / (3 * args.reps) * 1e3
        row = {"shape": name, "M": M, "N": N, "K": K, "gflop": round(2e-9 * M * N * K, 3)}
        _lib.check(lib.capgen_debug_gemm_variant(0))
        row["tuned_us"] = round(graph_time(), 2)
        best = (1e9, None)
        for v in variants:
            for sk in splits:
                if sk > 1 and ((K + 63) // 64 < 2 * sk or v >= 23):  # (k-group variants: no grid split-K)
                    continue
                _lib.check(lib.capgen_debug_gemm_variant(v + 100 * sk))
                try:
                    t = graph_time()
                except RuntimeError:
                    continue
                row[f"v{v}s{sk}"] = round(t, 2)
                if t < best[0]:
                    best = (t, f"v{v}s{sk}")
        _lib.check(lib.capgen_debug_gemm_variant(0))
        row["best"] = best[1]
        row["best_us"] = round(best[0], 2)
        print(json.dumps({k: row[k] for k in ("shape", "gflop", "tuned_us", "best", "best_us")} if len(row) > 8 else row),
              flush=True)
        out.append(row)
    with open(os.path.join(REPO, "gpurun_out", args.out), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
