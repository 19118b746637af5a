"""C4 decode concurrency probe: is the 256-image decode bound by its dependent chain of small
kernels (then two half-batch chains on two streams overlap) or by the device's throughput?

Times, per mode (beam-5 / greedy): one engine decoding all 256 images; one engine decoding 128;
two engines (same weights) decoding 128 each, issued on two torch streams so their chains run
side by side.  Prints one JSON line per measurement.  Synthetic inputs, random-init C2 weights."""
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


def main():
    cfg = preset("C2", dtype="bf16")
    dev = torch.device("cuda", 0)
    sd = {k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()}
    engs = []
    for _ in range(2):
        e = Engine(cfg, dev)
        e.load_state_dict(sd)
        e.set_training(False)
        engs.append(e)
    B, N = 256, 36
    f, p, _ = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, cfg.max_length, cfg.num_vocab,
                              seed=7)
    f = f.to(dev, torch.bfloat16).contiguous()
    p = p.to(dev).contiguous()
    halves = [(f[:B // 2].contiguous(), p[:B // 2].contiguous()), (f[B // 2:].contiguous(), p[B // 2:].contiguous())]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    reps = 5
    for mode in ("beam5", "greedy"):
        run = (lambda e, ff, pp: e.beam(ff, pp, 5)) if mode == "beam5" else \
              (lambda e, ff, pp: e.greedy(ff, pp, want_attention=False))

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        def two():
            for i in range(2):
                with torch.cuda.stream(streams[i]):
                    run(engs[i], *halves[i])

        full = timed(lambda: run(engs[0], f, p))
        half = timed(lambda: run(engs[0], *halves[0]))
        both = timed(two)
        # the two halves' ids equal the full run's (row results do not depend on the batch)
        with torch.cuda.stream(streams[0]):
            a = run(engs[0], *halves[0])
        with torch.cuda.stream(streams[1]):
            b = run(engs[1], *halves[1])
        torch.cuda.synchronize()
        ref = run(engs[0], f, p)
        torch.cuda.synchronize()
        ga = a[0] if isinstance(a, tuple) else a
        gb = b[0] if isinstance(b, tuple) else b
        gr = ref[0] if isinstance(ref, tuple) else ref
        same = bool(torch.equal(torch.cat([ga, gb]), gr))
        print(json.dumps({"mode": mode, "ms_full_256": round(full, 3), "ms_one_128": round(half, 3),
                          "ms_two_128_on_two_streams": round(both, 3), "halves_equal_full": same}), flush=True)


if __name__ == "__main__":
    main()
