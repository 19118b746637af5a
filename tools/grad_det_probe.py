"""Repeat the bf16 c2s forward + backward (train-mode dropout, fixed seed) in fresh engines and
report every run whose gradients are not bit-identical to the first run's, naming the tensors
(grouped / single weight-gradient launches alternate: CAPGEN_GROUP_DW).  Usage: grad_det_probe.py ITERS"""
import os
import sys

sys.path.insert(0, "image-caption_amd")
sys.path.insert(0, "tests")
import torch  # noqa: E402

from golden_util import load_fixture  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402

cfg, seed, z = load_fixture("c2s")
f, p, c = [torch.from_numpy(z[k]).to("cuda") for k in ("feats", "pos", "caps")]


def grads(group):
    os.environ["CAPGEN_GROUP_DW"] = "1" if group else "0"
    e = Engine(cfg.replace(dtype="bf16", dropout=0.3, attention_dropout=0.3), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_training(True)
    e.set_rng_seed(5)
    e.forward(f, p, c)
    e.backward()
    g = e.grads_state_dict()
    e.close()
    return g


ref = {True: grads(True), False: grads(False)}
bad = 0
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for it in range(iters):
    for group in (True, False):
        g = grads(group)
        r = ref[group]
        d = [(k, ((g[k].double() - r[k].double()).norm() / (r[k].double().norm() + 1e-30)).item())
             for k in g if not torch.equal(g[k], r[k])]
        big = [x for x in d if x[1] > 1e-4]
        if big:
            bad += 1
            big.sort(key=lambda x: -x[1])
            print(f"iter {it} group={group}: {len(big)} tensors differ > 1e-4 (of {len(d)} not bit-equal): "
                  + ", ".join(f"{k} {v:.1e}" for k, v in big[:6]), flush=True)
g1, g0 = ref[True], ref[False]
cross = sorted((((g1[k].double() - g0[k].double()).norm() / (g1[k].double().norm() + 1e-30)).item(), k) for k in g1)[-3:]
print(f"probe: {bad} of {2 * iters} runs differ from their first run; grouped vs single worst: "
      + ", ".join(f"{k} {v:.1e}" for v, k in cross), flush=True)
