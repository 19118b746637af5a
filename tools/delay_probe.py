"""Side-stream delay injection diagnostic (tests/test_gpu_hazard.py::test_side_stream_delay_...):
runs the c2s bf16 step with a 40 us spin before every off-critical-stream launch and without, in
this process, and prints which tensors differ -- gradients of a plain forward/backward, gradients
and weights after the first bucketed train_step, and after a second one.  Knobs come from the
environment (one process per setting).

  CAPGEN_OVERLAP_DEC0=0 python tools/delay_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from capgen import _lib  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402
from golden_util import load_fixture  # noqa: E402

DEV = "cuda:0"


def run(delay, order):
    cfg, seed, z = load_fixture("c2s")
    cfg = cfg.replace(dropout=0.3, attention_dropout=0.3)
    f, p, c = [torch.from_numpy(z[k]).to(DEV) for k in ("feats", "pos", "caps")]
    e = Engine(cfg.replace(dtype="bf16"), DEV)
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_rng_seed(11)
    _lib.side_delay(delay)
    out = {}
    try:
        if "fb" in order:
            e.forward(f, p, c)
            e.backward()
            out["g_fb"] = e.grads_state_dict()
            e.set_rng_seed(11)
        e.train_step(f, p, c)
        torch.cuda.synchronize()
        out["g_s1"] = e.grads_state_dict()
        out["w_s1"] = e.state_dict(False)
        e.train_step(f, p, c)
        torch.cuda.synchronize()
        out["w_s2"] = e.state_dict(False)
    finally:
        _lib.side_delay(0.0)
    return out


def diff(a, b):
    bad = {}
    for k in a:
        if a[k].dim() == 2 and k != "decoder.word_embedding.weight" and not torch.equal(a[k], b[k]):
            bad[k] = float((a[k] - b[k]).abs().max())
    return bad


def main():
    env = {k: v for k, v in os.environ.items() if k.startswith("CAPGEN_")}
    for order in ("fb", "step"):
        ra, rb = run(40.0, order), run(0.0, order)
        rep = {"env": env, "order": order, "live_tuned": _lib.load().capgen_tune_live_count()}
        for k in ra:
            d = diff(ra[k], rb[k])
            rep[k] = {"n": len(d), "first": sorted(d.items(), key=lambda kv: -kv[1])[:6]}
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
