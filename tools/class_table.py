"""Per-kernel-class table of one C2 train step: launches, kernel time, algorithmic FLOP and bytes
(C2 shapes), PMC bytes (FETCH_SIZE x2 + WRITE_SIZE, as tools/pmcsum.py) and MFMA
busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the class's kernel cycles, as tools/pmc_mfma.py).

usage: python tools/class_table.py <round dir of tools/round_profile.sh>   (e.g. gpurun_out/r02)
"""
import collections
import csv
import glob
import os
import sys

B, N, T, d, f, V = 64, 36, 20, 512, 2048, 10000
Me, Md = B * N, B * (T - 1)
ENC = [(Me, 3 * d, d), (Me, d, d), (Me, f, d), (Me, d, f)] * 6
DEC = [(Md, 3 * d, d), (Md, d, d), (Md, d, d), (Md, d, d), (Md, f, d), (Md, d, f)] * 6
OTHER = [(Me, d, 2176), (Md, d, d), (Me, 12 * d, d), (Md, V, d)]
# forward projections inside the fused attention fronts (qkv_attn_kernel, round 4): every self-attention
# Q/K/V projection, and the cross-attention query projection of decoder blocks 1..5 (block 0's runs as a
# GEMM on the side stream with the decoder front)
FRONT = [(Me, 3 * d, d)] * 6 + [(Md, 3 * d, d)] * 6 + [(Md, d, d)] * 5
FWD = [(Me, d, d), (Me, f, d), (Me, d, f)] * 6 + [(Md, d, d), (Md, d, d), (Md, f, d), (Md, d, f)] * 6 + \
    [(Md, d, d)] + OTHER
# input gradients: the 18 output projections' (Wo, Wo_s, Wo_c) run inside the fused attention
# backward (qkv_attn_bwd, round 4)
WO_DX = [(Me, d, d)] * 6 + [(Md, d, d)] * 12
DX = [(Me, 3 * d, d), (Me, f, d), (Me, d, f)] * 6 + [(Md, 3 * d, d), (Md, d, d), (Md, f, d), (Md, d, f)] * 6 + \
    OTHER[1:]
FWD_ALL = ENC + DEC + OTHER
LN_ROWS = [Me] * 13 + [Md] * 19
ALG = {  # class -> (GFLOP, algorithmic GB) per step
    "GEMM fwd (NT)": (sum(2 * m * n * k for m, n, k in FWD) / 1e9,
                      sum((m * k + n * k) * 2 + m * n * 2 for m, n, k in FWD) / 1e9),
    "GEMM dX (NN)": (sum(2 * m * n * k for m, n, k in DX) / 1e9,
                     sum((m * n + n * k) * 2 + m * k * 2 for m, n, k in DX) / 1e9),
    "GEMM dW (TN)": (sum(2 * m * n * k for m, n, k in FWD_ALL) / 1e9,
                     sum((m * n + m * k) * 2 + n * k * 4 for m, n, k in FWD_ALL) / 1e9),
    # fused front: read X, W, (cross: K/V); write the projection (kept for the backward) and o
    "attention front (proj+attn)": (
        sum(2 * m * n * k for m, n, k in FRONT) / 1e9,
        (6 * (Me * d + 3 * d * d + Me * 3 * d + Me * d) + 6 * (Md * d + 3 * d * d + Md * 3 * d + Md * d)
         + 5 * (Md * d + d * d + Md * d + 2 * Me * d + Md * d)) * 2 / 1e9),
    # y = LN(a + res): read a, res; write y, v (bf16)
    "LayerNorm fwd": (0, sum(4 * r * d * 2 for r in LN_ROWS) / 1e9),
    # read dy, v; write d_res, d_a
    "LayerNorm bwd": (0, sum(4 * r * d * 2 for r in LN_ROWS) / 1e9),
    # read q, k, v; write o  (self: rows x d each; cross: q/o over Md rows, k/v over Me rows)
    # (the one separate launch: decoder block 0's cross attention)
    "attention fwd": (0, (2 * Md + 2 * Me) * d * 2 / 1e9),
    # fused: read dA, the Wo^T slice, q, k, v; write dq, dk, dv (dO never leaves the launch)
    "attention bwd + Wo dX (fused)": (sum(2 * m * n * k for m, n, k in WO_DX) / 1e9,
                                      (6 * 7 * Me * d * 2 + 6 * 7 * Md * d * 2 + 6 * (3 * Md + 4 * Me) * d * 2
                                       + sum(n * k * 2 for m, n, k in WO_DX)) / 1e9),
    "Adam": (0, 30 * 55_707_408 / 1e9),
    "cross entropy": (0, (2 * Md * V * 2 + Md * ((V + 15) // 16) * 8) / 1e9),
}


def floors():
    """class -> per-XCD panel floor GB (tools/gemm_floor.py: every XCD's L2 fetches each operand panel
    its tiles read once, for the kernel's tile-to-XCD map and the autotuned tiles)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gemm_floor as gf
    t = gf.tune_table()
    return {"GEMM dX (NN)": gf.class_floor(gf.DX, t)[1] / 1e9, "GEMM fwd (NT)": gf.class_floor(gf.FWD, t)[1] / 1e9}


def klass(name):
    if "grouped" in name:
        return "GEMM dW (TN)"
    if "gemm_bf16_kernel" in name:
        if "gemm_bf16_kernelI" in name:  # mangled: ...kernelI<TO>Lb<TA>ELb<TB>E...
            lay = name.split("gemm_bf16_kernelI")[1][:24]
            ta, tb = "Lb1ELb" in lay, "ELb1E" in lay
        else:  # demangled: gemm_bf16_kernel<TO, TA, TB, ...>
            a = name.split("gemm_bf16_kernel<")[1].split(",")
            ta, tb = a[1].strip() == "true", a[2].strip() == "true"
        return "GEMM dW (TN)" if ta else "GEMM dX (NN)" if tb else "GEMM fwd (NT)"
    for key, k in (("qkv_attn_bwd", "attention bwd + Wo dX (fused)"), ("qkv_attn", "attention front (proj+attn)"),
                   ("ln_fwd", "LayerNorm fwd"), ("ln_bwd", "LayerNorm bwd"), ("attn_fwd", "attention fwd"),
                   ("attn_bwd", "attention bwd"), ("adam_kernel", "Adam"), ("ce_finish", "cross entropy"),
                   ("ce_reg", "cross entropy")):
        if key in name:
            return k
    return "other"


def steps(rows, key_s, nmax=5):
    marks = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r["Kernel_Name"]]
    n = min(nmax, len(marks) - 1)
    return rows[marks[-n - 1]:marks[-1]], n


def load(d, pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    rd = sys.argv[1]
    tr = sorted(load(os.path.join(rd, "trace"), "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    sl, n = steps(tr, "Start_Timestamp")
    t = collections.defaultdict(lambda: [0, 0.0])
    for r in sl:
        k = klass(r["Kernel_Name"])
        t[k][0] += 1 / n
        t[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / n
    by = collections.defaultdict(lambda: [0.0, 0.0])
    for col, ctr, mul in ((0, "FETCH_SIZE", 2.0), (1, "WRITE_SIZE", 1.0)):
        rows = [r for r in load(os.path.join(rd, "pmc_" + ctr), "*counter_collection.csv") if r["Counter_Name"] == ctr]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        s2, n2 = steps(rows, "Dispatch_Id")
        for r in s2:
            by[klass(r["Kernel_Name"])][col] += mul * float(r["Counter_Value"]) * 1024 / n2
    mf = collections.defaultdict(lambda: [0.0, 0.0])
    rows = load(os.path.join(rd, "pmc_mfma"), "*counter_collection.csv")
    rows.sort(key=lambda r: (int(r["Dispatch_Id"]), r["Counter_Name"]))
    s3, n3 = steps(rows, "Dispatch_Id")
    for r in s3:
        k = klass(r["Kernel_Name"])
        if r["Counter_Name"].startswith("SQ_VALU_MFMA_BUSY_CYCLES"):
            mf[k][0] += float(r["Counter_Value"])
        elif r["Counter_Name"].startswith("GRBM_GUI_ACTIVE"):
            mf[k][1] += float(r["Counter_Value"])
    fl = floors()
    print(f"{'class':16s} {'n/step':>6s} {'us/step':>8s} {'GFLOP':>7s} {'TF/s':>6s} {'alg GB':>7s} "
          f"{'PMC GB':>7s} {'PMC/alg':>7s} {'floor GB':>8s} {'PMC/floor':>9s} {'MFMA busy':>9s}")
    for k in sorted(t, key=lambda k: -t[k][1]):
        gf, ab = ALG.get(k, (0, 0))
        pb = (by[k][0] + by[k][1]) / 1e9
        busy = mf[k][0] / (mf[k][1] * 256 / 8 * 4) if mf[k][1] else 0.0  # per-XCD GRBM cycles x 32 CUs x 4 SIMDs
        tfs = gf / t[k][1] * 1e3 if gf else 0.0  # GFLOP / us = PFLOP/s
        f = fl.get(k)
        fcol = f"{f:8.3f} {pb / f:9.2f}" if f else f"{'-':>8s} {'-':>9s}"
        print(f"{k:16s} {t[k][0]:6.1f} {t[k][1]:8.1f} {gf:7.1f} {tfs:6.0f} {ab:7.3f} {pb:7.3f} "
              f"{(pb / ab if ab else 0):7.2f} {fcol} {busy:9.4f}")


if __name__ == "__main__":
    main()
