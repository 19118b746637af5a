"""HBM-side byte floor of the step's bf16 GEMM launches for the tile-to-XCD map the kernel uses
(VERDICT r5 item 5): what PMC FETCH/WRITE bytes a GEMM launch cannot go below when every XCD's L2
fetches, once, each operand panel that XCD's tiles read.

gemm_bf16_kernel (gemm_bf16.hip) deals its grid round-robin over the 8 XCDs (block b on XCD b % 8,
MI355X_MICROARCH.md § dispatch), remaps block b to slot xcd_slot(b, nblk) so each XCD owns one
contiguous slot range, splits slot -> (tile, split-K slice) and orders tiles in column-major groups of
group_m tile rows (group_m = round(sqrt(tiles / 8))).  Per XCD the floor counts the distinct A row
panels x k-range and B column panels x k-range of its tiles (bf16), every launch's C once (bf16, f32 for
f32 outputs), the ReLU-mask operand where the launch reads one, and -- with split-K -- the f32 slice
slabs written once and read once by the combining workgroup.  Summed over the XCDs this is the
'floor' column of tools/class_table.py; alg (each operand once) <= floor <= PMC.

    python tools/gemm_floor.py            # the C2 step's dX and forward GEMMs, per launch
"""
import math
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNE = os.path.join(REPO, "image-caption_amd", "capgen", "tune_gfx950.txt")


def tune_table(path=TUNE):
    """(M, N, K, ta, tb, out_bytes) -> (BM, BN, splitk) from the persisted autotune table."""
    t = {}
    for line in open(path):
        if not line.startswith("g "):
            continue
        head, _, comment = line.partition("#")
        f = head.split()
        m = re.match(r"\s*(\d+)x(\d+)", comment)
        if len(f) < 9 or not m:
            continue
        key = tuple(int(x) for x in f[1:7])
        t[key] = (int(m.group(1)), int(m.group(2)), int(f[8]))
    return t


def xcd_of_slots(nblk):
    """slot -> XCD for gemm_tile.h xcd_slot (block b on XCD b % 8)."""
    q8, r8 = nblk >> 3, nblk & 7
    owner = [0] * nblk
    for b in range(nblk):
        x = b & 7
        slot = (x * (q8 + 1) if x < r8 else r8 * (q8 + 1) + (x - r8) * q8) + (b >> 3)
        owner[slot] = x
    return owner


def floor_bytes(M, N, K, BM, BN, splitk=1, out_bytes=2, aux=False):
    """Per-XCD-panel floor of one launch C[M x N] = A[M x K] . B (both bf16)."""
    tn, tm = math.ceil(N / BN), math.ceil(M / BM)
    nblk = tn * tm * splitk
    owner = xcd_of_slots(nblk)
    per = max(1, min(tm, round(math.sqrt(tn * tm / 8.0))))
    kslice = math.ceil(K / splitk)
    a_seen = [set() for _ in range(8)]
    b_seen = [set() for _ in range(8)]
    for slot in range(nblk):
        tile, split = divmod(slot, splitk)
        mt, nt = divmod(tile, tn)
        if per > 1:
            grp = per * tn
            first = (tile // grp) * per
            gsz = min(tm - first, per)
            r = tile % grp
            mt, nt = first + r % gsz, r // gsz
        x = owner[slot]
        a_seen[x].add((mt, split))
        b_seen[x].add((nt, split))
    byts = 0
    for x in range(8):
        for mt, split in a_seen[x]:
            rows = min(BM, M - mt * BM)
            byts += rows * min(kslice, K - split * kslice) * 2
        for nt, split in b_seen[x]:
            cols = min(BN, N - nt * BN)
            byts += cols * min(kslice, K - split * kslice) * 2
    byts += M * N * out_bytes
    if aux:
        byts += M * N * 2
    if splitk > 1:
        byts += 2 * M * N * 4 * splitk
    return byts


def alg_bytes(M, N, K, out_bytes=2, aux=False):
    return (M * K + K * N) * 2 + M * N * out_bytes + (M * N * 2 if aux else 0)


B, Nr, T, d, f, V = 64, 36, 20, 512, 2048, 10000
Me, Md = B * Nr, B * (T - 1)
# (M, N, K, ta, tb, aux): the launches of one C2 train step's critical-path GEMM classes (the fused
# attention kernels carry the Q/K/V projections and the output projections' input gradients)
DX = ([(Me, d, 3 * d, 0, 1, False), (Me, f, d, 0, 1, True), (Me, d, f, 0, 1, False)] * 6
      + [(Md, d, 3 * d, 0, 1, False), (Md, d, d, 0, 1, False), (Md, f, d, 0, 1, True), (Md, d, f, 0, 1, False)] * 6
      + [(Md, d, d, 0, 1, False), (Me, d, 12 * d, 0, 1, False), (Md, d, V, 0, 1, False)])
FWD = ([(Me, d, d, 0, 0, False), (Me, f, d, 0, 0, False), (Me, d, f, 0, 0, False)] * 6
       + [(Md, d, d, 0, 0, False), (Md, d, d, 0, 0, False), (Md, f, d, 0, 0, False), (Md, d, f, 0, 0, False)] * 6
       + [(Md, d, d, 0, 0, False), (Me, d, 2176, 0, 0, False), (Md, d, d, 0, 0, False), (Me, 12 * d, d, 0, 0, False)])


def class_floor(launches, table=None):
    """(alg bytes, floor bytes, [(shape, BM, BN, splitk, alg, floor)]) for a list of launches."""
    table = table or tune_table()
    tot_a = tot_f = 0
    rows = []
    for M, N, K, ta, tb, aux in launches:
        BM, BN, sk = table.get((M, N, K, ta, tb, 2), (64, 64, 1))
        a = alg_bytes(M, N, K, aux=aux)
        fl = floor_bytes(M, N, K, BM, BN, sk, aux=aux)
        tot_a += a
        tot_f += fl
        rows.append(((M, N, K), BM, BN, sk, a, fl))
    return tot_a, tot_f, rows


def main():
    t = tune_table()
    for name, launches in (("GEMM dX (NN)", DX), ("GEMM fwd (NT)", FWD)):
        a, fl, rows = class_floor(launches, t)
        print(f"{name}: {len(launches)} launches, alg {a / 1e9:.3f} GB, per-XCD panel floor {fl / 1e9:.3f} GB "
              f"({fl / a:.2f}x alg)")
        seen = {}
        for shp, BM, BN, sk, aa, ff in rows:
            seen.setdefault((shp, BM, BN, sk), [0, aa, ff])[0] += 1
        for (shp, BM, BN, sk), (n, aa, ff) in seen.items():
            print(f"  {n:2d} x {shp[0]}x{shp[1]}x{shp[2]:<5d} tile {BM}x{BN} splitK {sk}: alg {aa / 1e6:6.2f} MB, "
                  f"floor {ff / 1e6:6.2f} MB ({ff / aa:.2f}x)")


if __name__ == "__main__":
    main()
