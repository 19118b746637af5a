"""C4 (BASELINE.json configs[3]): generate() on 1 GPU — beam 5 and greedy over a batch of 256
images (36 x 2048 region features, max_length 20), bf16, synthetic inputs, random-init C2
weights.  KV-cached decode (model.py:101-200 restated).  Prints one JSON line per mode.

Algorithmic work (KV-cached count): beam-5 1776.7 GFLOP, greedy 699.4 GFLOP per
256-image batch.  The reference CPU path (no KV cache) took 25.0 s (beam) / 5.87 s (greedy) per
batch on the survey container's 8 cores."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import torch  # noqa: E402

from capgen import preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402

GFLOP = {"beam5": 1776.7, "greedy": 699.4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1, help="untimed calls first (CAPGEN_GEN_GRAPH=1 captures on the 2nd)")
    ap.add_argument("--modes", default="beam5,greedy")
    args = ap.parse_args()
    cfg = preset("C2", dtype="bf16")
    dev = torch.device("cuda", 0)
    eng = Engine(cfg, dev)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
    eng.set_training(False)
    B, N = args.batch, 36
    f, p, _ = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, cfg.max_length,
                              cfg.num_vocab, seed=7)
    f = f.to(dev, torch.bfloat16).contiguous()
    p = p.to(dev).contiguous()
    runs = {"beam5": lambda: eng.beam(f, p, 5), "greedy": lambda: eng.greedy(f, p, want_attention=False)}
    for name, fn in runs.items():
        if name not in args.modes.split(","):
            continue
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        print(json.dumps({"metric": f"generate {name} images/sec (C4: B={B}, max_length={cfg.max_length})",
                          "value": round(B / dt, 1), "unit": "images/s", "ms_per_batch": round(dt * 1e3, 3),
                          "achieved_tflops": round(GFLOP[name] * (B / 256) / dt / 1e3, 2), "dtype": "bf16",
                          "data": "synthetic"}), flush=True)


if __name__ == "__main__":
    main()
