"""Un-profiled per-kernel timeline of the C2 bf16 train step (bench.py's workload).

Every GEMM / LayerNorm / attention launch records the 100 MHz real-time counter at its first block's
start and its last block's end (capgen_debug_stamps; StampScope in capgen_common.h) -- no profiler,
no extra launches.  Two steps run back to back and the second one is read, so the step boundary
(next forward behind the previous step's bucket Adam) is in the picture.

Reports: the critical stream's busy fraction (union of its stamped kernels / its span), the step's
span, the largest idle gaps on the critical stream with the kernels either side, and per-class
time.  Unstamped launches (pack, ce_finish, loss_finalize, Adam, column sums, folds, memsets) show up
inside gaps.  Also times 20 steps with stamps off and on (the stamps' own cost).

  python tools/stamp_timeline.py --out gpurun_out/stamps
"""
import argparse
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import torch  # noqa: E402

from capgen import preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402


def union_len(iv):
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def timed(eng, args, n=20):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        eng.train_step_raw(*args)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def analyse(rows):
    rows = [(n, s, e) for n, s, e in rows if s > 0 and e > 0 and e >= s]
    t0 = min(s for _, s, _ in rows)
    rows = [(n, s - t0, e - t0) for n, s, e in rows]
    crit = sorted([r for r in rows if r[0].startswith("crit")], key=lambda r: r[1])
    span_c = crit[-1][2] - crit[0][1]
    busy = union_len([(s, e) for _, s, e in crit])
    gaps = []
    for a, b in zip(crit, crit[1:]):
        g = b[1] - a[2]
        gaps.append((g, a[0], b[0], a[2]))
    gaps.sort(reverse=True)
    cls = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        k = " ".join(n.split()[:3]) if "gemm" in n else " ".join(n.split()[:2])
        cls[k][0] += 1
        cls[k][1] += e - s
    return {
        "step_span_us": max(e for _, _, e in rows),
        "crit_span_us": span_c, "crit_busy_us": busy, "crit_busy_frac": busy / span_c,
        "crit_kernels": len(crit), "crit_gap_sum_us": span_c - busy,
        "gaps_over_2us": sum(1 for g in gaps if g[0] > 2.0),
        "largest_gaps": [{"gap_us": round(g, 2), "after": a, "before": b, "at_us": round(t, 1)} for g, a, b, t in gaps[:25]],
        "classes": {k: {"n": v[0], "us": round(v[1], 1)} for k, v in sorted(cls.items(), key=lambda kv: -kv[1][1])},
    }, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/stamps")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    dev = torch.device("cuda", 0)
    cfg = preset("C2", dtype="bf16", dropout=0.3)
    eng = Engine(cfg, dev)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
    f, p, c = synthetic_batch(64, 36, cfg.encode_dim_features, cfg.encode_dim_positions, 20, cfg.num_vocab, seed=1000)
    f, p, c = f.to(dev, torch.bfloat16).contiguous(), p.to(dev).contiguous(), c.to(dev).contiguous()
    loss = torch.zeros(1, device=dev)
    from capgen import _lib
    a = (f, _lib.BF16, p, c, 64, 36, 20, loss)
    for _ in range(5):
        eng.train_step_raw(*a)
    torch.cuda.synchronize()
    off_ms = timed(eng, a)
    eng.stamps(1)
    for _ in range(3):
        eng.train_step_raw(*a)
    torch.cuda.synchronize()
    on_ms = timed(eng, a)
    reports = []
    for r in range(args.reps):
        eng.stamps(3)
        eng.train_step_raw(*a)
        eng.train_step_raw(*a)
        torch.cuda.synchronize()
        rep, rows = analyse(eng.stamps(2))
        reports.append(rep)
        with open(os.path.join(args.out, f"timeline_{r}.txt"), "w") as fh:
            for n, s, e in sorted(rows, key=lambda x: x[1]):
                fh.write(f"{s:9.2f} {e:9.2f} {e - s:7.2f}  {n}\n")
        print(json.dumps({k: rep[k] for k in ("step_span_us", "crit_span_us", "crit_busy_us", "crit_busy_frac",
                                              "crit_kernels", "gaps_over_2us")}), flush=True)
    eng.stamps(0)
    summary = {"ms_per_step_stamps_off": round(off_ms, 4), "ms_per_step_stamps_on": round(on_ms, 4),
               "reps": reports}
    with open(os.path.join(args.out, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps({"off_ms": off_ms, "on_ms": on_ms}), flush=True)


if __name__ == "__main__":
    main()
