"""Uninitialised-read probe: the same c2s bf16 calls (forward + backward, then two bucketed
train_steps) on engines whose fresh activation workspace is filled with a byte pattern
(CAPGEN_POISON, read when the workspace is allocated) -- any read of a never-written element
changes the results deterministically.  Prints which tensors differ from the unpoisoned engine."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402
from golden_util import load_fixture  # noqa: E402


def run(poison, tag="c2s"):
    if poison is None:
        os.environ.pop("CAPGEN_POISON", None)
    else:
        os.environ["CAPGEN_POISON"] = poison
    cfg, seed, z = load_fixture(tag)
    cfg = cfg.replace(dropout=0.3, attention_dropout=0.3)
    f, p, c = [torch.from_numpy(z[k]).to("cuda:0") for k in ("feats", "pos", "caps")]
    e = Engine(cfg.replace(dtype="bf16"), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_rng_seed(11)
    out = {}
    out["loss_fb"] = e.forward(f, p, c).clone()
    e.backward()
    out["g_fb"] = e.grads_state_dict()
    e.set_rng_seed(11)
    out["loss_s1"] = e.train_step(f, p, c).clone()
    torch.cuda.synchronize()
    out["g_s1"] = e.grads_state_dict()
    out["w_s1"] = e.state_dict(False)
    out["loss_s2"] = e.train_step(f, p, c).clone()
    torch.cuda.synchronize()
    out["w_s2"] = e.state_dict(False)
    os.environ.pop("CAPGEN_POISON", None)
    return out


def cmp(a, b):
    rep = {}
    for k in a:
        if isinstance(a[k], dict):
            bad = {n: float((a[k][n].double() - b[k][n].double()).abs().max()) for n in a[k]
                   if not torch.equal(a[k][n], b[k][n])}
            nan = [n for n in a[k] if not torch.isfinite(b[k][n]).all()]
            rep[k] = {"n": len(bad), "nan": len(nan), "first": sorted(bad.items(), key=lambda kv: -kv[1])[:3]}
        else:
            rep[k] = [a[k].item(), b[k].item()]
    return rep


base = run(None)
for pz in ("0xff", "0x3f", "0x00"):
    print(json.dumps({"poison": pz, **cmp(base, run(pz))}), flush=True)
