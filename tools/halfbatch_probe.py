"""Does splitting the C2 batch into two concurrent half-batch chains pay on MI355X?

GPU-side time only: every stream first waits behind a sleep kernel while the host enqueues
all the work, so host launch cost is excluded.  Compares R forwards of one B=64 engine with
R forwards of two B=32 engines on two streams (and one B=32 engine alone).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "image-caption_amd"))
import torch  # noqa: E402

from capgen import preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402

N, T, R = 36, 20, 4
cfg = preset("C2", dtype="bf16", dropout=0.3)
dev = torch.device("cuda", 0)
sd = {k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()}


def make(B):
    e = Engine(cfg, dev)
    e.load_state_dict(sd)
    f, p, c = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab, seed=B)
    return e, (f.to(dev, torch.bfloat16), p.to(dev), c.to(dev))


def run(pairs, what):
    streams = [torch.cuda.Stream(dev) for _ in pairs]
    for (e, x), s in zip(pairs, streams):  # warm-up / autotune
        with torch.cuda.stream(s):
            for _ in range(2):
                e.forward(*x) if what == "fwd" else e.train_step(*x)
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(streams[0]):
        torch.cuda._sleep(500_000_000)  # ~0.2 s of GPU sleep: the host enqueues everything meanwhile
        start.record()
    for s in streams[1:]:
        s.wait_event(start)
    for r in range(R):
        for (e, x), s in zip(pairs, streams):
            with torch.cuda.stream(s):
                e.forward(*x) if what == "fwd" else e.train_step(*x)
    for s in streams[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        streams[0].wait_event(ev)
    with torch.cuda.stream(streams[0]):
        end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / R


for what in (() if os.environ.get("SIMPLE") else ("fwd", "step")):
    one64 = run([make(64)], what)
    one32 = run([make(32)], what)
    two32 = run([make(32), make(32)], what)
    print(f"{what}: one B=64 {one64:.3f} ms | one B=32 {one32:.3f} ms | two concurrent B=32 {two32:.3f} ms", flush=True)

if os.environ.get("SIMPLE"):
    import time
    for B in (64, 32):
        e, x = make(B)
        for _ in range(3):
            e.forward(*x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            e.forward(*x)
        torch.cuda.synchronize()
        print(f"simple fwd B={B}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms", flush=True)
