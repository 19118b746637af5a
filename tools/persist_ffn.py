"""Fault isolation of the persistent FFN pair (csrc/persist.hip, debug library only).

Runs capgen_dbg_ffn_persist in each `mode` (bit 1: W2 tasks only, H from the plain W1 launch; bit 2:
the W2 tile on a private copy of its GemmArgs; bit 4: no consumer acquire) at several grid sizes, on
one 64-row block and on the C2 encoder FFN shape, and compares H and Y bit for bit with the two plain
launches of the same tile variant (7: 64x64, 4 waves, 3 stages).  Prints one JSON line per run and
writes gpurun_out/persist_ffn.json.

  CAPGEN_LIB_PATH=image-caption_amd/capgen/libcapgen_debug.so python tools/persist_ffn.py
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
os.environ.setdefault("CAPGEN_LIB_PATH", os.path.join(REPO, "image-caption_amd", "capgen", "libcapgen_debug.so"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402


def ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def main():
    lib = _lib.load()
    assert _lib.debug_build(), "needs libcapgen_debug.so"
    fn = lib.capgen_dbg_ffn_persist
    fn.restype = C.c_int
    fn.argtypes = [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 6 + [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = []
    s = torch.cuda.Stream(dev)
    for name, M, d, fe in (("one row block", 64, 512, 2048), ("enc FFN", 2304, 512, 2048)):
        X = (torch.randn(M, d, device=dev) * 0.5).to(torch.bfloat16)
        W1 = (torch.randn(fe, d, device=dev) / d ** 0.5).to(torch.bfloat16)
        b1 = torch.randn(fe, device=dev) * 0.1
        W2 = (torch.randn(d, fe, device=dev) / fe ** 0.5).to(torch.bfloat16)
        Hr = torch.empty(M, fe, device=dev, dtype=torch.bfloat16)
        Yr = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
        _lib.check(lib.capgen_debug_gemm_variant(7))
        with torch.cuda.stream(s):
            _lib.check(lib.capgen_debug_gemm(M, fe, d, ptr(X), d, 0, ptr(W1), d, 0, ptr(Hr), fe, 1, 1, ptr(b1), 1.0, 0, 1,
                                             C.c_void_p(s.cuda_stream)))
            _lib.check(lib.capgen_debug_gemm(M, d, fe, ptr(Hr), fe, 0, ptr(W2), fe, 0, ptr(Yr), d, 1, 1, None, 1.0, 0, 0,
                                             C.c_void_p(s.cuda_stream)))
        _lib.check(lib.capgen_debug_gemm_variant(0))
        torch.cuda.synchronize()
        ref = (Hr.float() @ W2.float().t())
        scale = ref.abs().max().item()
        for mode in (0, 1, 64, 128, 256, 257):
            for grid in ((1, 8, 256) if M == 64 else (256, 512, 768)):
                H = torch.full_like(Hr, float("nan")) if not (mode & (1 | 16 | 32 | 64)) else Hr.clone()
                Y = torch.full_like(Yr, float("nan"))
                gv = C.c_int(-1)
                rc = fn(M, d, fe, ptr(X), ptr(W1), ptr(b1), ptr(W2), ptr(H), ptr(Y), grid, mode, C.byref(gv),
                        C.c_void_p(s.cuda_stream))
                torch.cuda.synchronize()
                diff = (Y.float() - Yr.float()).abs()
                tiles = [bool(torch.equal(Y[:, j * 64:(j + 1) * 64], Yr[:, j * 64:(j + 1) * 64])) for j in range(d // 64)]
                row = {"shape": name, "mode": mode, "grid": grid, "rc": rc, "giveups": gv.value,
                       "H_equal": bool(torch.equal(H, Hr)), "Y_equal": bool(torch.equal(Y, Yr)),
                       "Y_nan": bool(torch.isnan(Y).any()), "Y_maxdiff_rel": diff.nan_to_num(1e30).max().item() / scale,
                       "Y_tiles_equal": sum(tiles), "Y_tiles": len(tiles)}
                if not row["Y_equal"] and M == 64:
                    # which source would explain Y: H rows / columns shifted, or the W2 operand
                    bad = (Y.float() - Yr.float()).abs().nan_to_num(1e30) > 1e-2 * scale
                    row["bad_frac"] = bad.float().mean().item()
                    yo = Y.float()
                    for tag, cand in (("H.W2t", Hr.float() @ W2.float().t()),
                                      ("X-as-A", None if fe != d else None)):
                        if cand is not None:
                            row["rel_err_vs_" + tag] = (yo - cand).abs().nan_to_num(1e30).max().item() / scale
                    # per-k-block contribution test: Y vs H[:, :K'] . W2[:, :K']^T for prefixes
                    best = None
                    for kk in range(64, fe + 1, 64):
                        part = Hr.float()[:, :kk] @ W2.float()[:, :kk].t()
                        e = (yo - part).abs().nan_to_num(1e30).max().item() / scale
                        if best is None or e < best[1]:
                            best = (kk, e)
                    row["best_k_prefix"] = best
                print(json.dumps(row), flush=True)
                rows.append(row)
        if M == 64:
            continue

        def pair(Ho, Yo):
            _lib.check(lib.capgen_debug_gemm(M, fe, d, ptr(X), d, 0, ptr(W1), d, 0, ptr(Ho), fe, 1, 1, ptr(b1), 1.0, 0, 1,
                                             C.c_void_p(s.cuda_stream)))
            _lib.check(lib.capgen_debug_gemm(M, d, fe, ptr(Ho), fe, 0, ptr(W2), fe, 0, ptr(Yo), d, 1, 1, None, 1.0, 0, 0,
                                             C.c_void_p(s.cuda_stream)))

        def gtime(f, reps=20):
            with torch.cuda.stream(s):
                f()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(reps):
                        f()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(3):
                    g.replay()
                e1.record(s)
                e1.synchronize()
                return round(e0.elapsed_time(e1) / (3 * reps) * 1e3, 2)

        H = torch.empty_like(Hr)
        Y = torch.empty_like(Yr)
        gv = C.c_int(-1)
        tm = {"shape": name, "timing_us": {}}
        _lib.check(lib.capgen_debug_gemm_variant(7))
        tm["timing_us"]["pair_v7"] = gtime(lambda: pair(H, Y))
        _lib.check(lib.capgen_debug_gemm_variant(0))
        tm["timing_us"]["pair_tuned"] = gtime(lambda: pair(H, Y))
        for grid in (256, 512, 768, 1024):
            tm["timing_us"][f"persist_one_site_g{grid}"] = gtime(
                lambda: fn(M, d, fe, ptr(X), ptr(W1), ptr(b1), ptr(W2), ptr(H), ptr(Y), grid, 128, None,
                           C.c_void_p(s.cuda_stream)))
        tm["persist_one_site_equal_after_timing"] = bool(torch.equal(Y, Yr))
        print(json.dumps(tm), flush=True)
        rows.append(tm)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "persist_ffn.json"), "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
