"""Is the step host-launch-bound?  Host time to enqueue K graph replays vs the GPU time."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "image-caption_amd"))
import torch  # noqa: E402

from capgen import _lib, preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402

B, N, T = 64, 36, 20
cfg = preset("C2", dtype="bf16", dropout=0.3)
dev = torch.device("cuda", 0)
eng = Engine(cfg, dev)
eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
eng.set_graph(len(sys.argv) > 1 and sys.argv[1] == "graph")
f, p, c = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab, seed=1000)
f, p, c = f.to(dev, torch.bfloat16).contiguous(), p.to(dev).contiguous(), c.to(dev).contiguous()
loss = torch.zeros(1, device=dev)
for _ in range(10):
    eng.train_step_raw(f, _lib.BF16, p, c, B, N, T, loss)
torch.cuda.synchronize()
K = 50
t0 = time.perf_counter()
for _ in range(K):
    eng.train_step_raw(f, _lib.BF16, p, c, B, N, T, loss)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e3 * (t1 - t0) / K:.3f} ms/step, total {1e3 * (t2 - t0) / K:.3f} ms/step")
