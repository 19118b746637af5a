"""Diagnostic: per-tensor relative gradient error of the bf16 path vs the fp32 parity path in
train mode (same dropout masks), on the c2s fixture configuration."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402
from golden_util import load_fixture  # noqa: E402

cfg, seed, z = load_fixture("c2s")
f, p, c = [torch.from_numpy(z[k]).to("cuda:0") for k in ("feats", "pos", "caps")]
res = {}
for dt in ("fp32", "bf16"):
    e = Engine(cfg.replace(dtype=dt, dropout=0.3, attention_dropout=0.3), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_training(True)
    e.set_rng_seed(1234)
    loss = e.forward(f, p, c).item()
    e.backward()
    res[dt] = (loss, {k: v.double() for k, v in e.grads_state_dict().items()})
print("loss fp32 %.6f bf16 %.6f" % (res["fp32"][0], res["bf16"][0]))
errs = []
for n, a in res["fp32"][1].items():
    b = res["bf16"][1][n]
    errs.append((((a - b).norm() / (a.norm() + 1e-12)).item(), n))
for e, n in sorted(errs, reverse=True)[:12]:
    print(f"{e:.4f} {n}")
