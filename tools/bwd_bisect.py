"""Run-to-run bisection of the bf16 backward pass: two engines run the identical c2s forward +
backward (stopped early by CAPGEN_DEBUG_BWD_STOP), then intermediate gradient buffers are copied
out (capgen_debug_copy_buffer) and compared bit for bit; prints where they differ."""
import ctypes as C
import os
import sys

sys.path.insert(0, "image-caption_amd")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from capgen import _lib  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402
from golden_util import load_fixture  # noqa: E402

cfg, seed, z = load_fixture("c2s")
f, p, c = [torch.from_numpy(z[k]).to("cuda") for k in ("feats", "pos", "caps")]
B, N, _ = f.shape
Me, d = B * N, cfg.encode_input_size
lib = _lib.load()
BUFS = {0: ("tmp", Me * d), 1: ("gOut", Me * d), 2: ("gRes", Me * d), 4: ("enc5.gH", Me * cfg.encode_hidden_size),
        5: ("enc5.gAf", Me * d), 6: ("enc5.gA1", Me * d), 7: ("enc5.gQKV", Me * 3 * d)}
if os.environ.get("CAPGEN_DEBUG_BWD_STOP") == "4":  # snapshots taken around the block's MHA LayerNorm backward
    BUFS.update({8: ("snap.ln1_dy", Me * d), 9: ("snap.ln1_da", Me * d), 10: ("snap.ln1_v", Me * d),
                 11: ("snap.ln1_mean", Me * 2), 12: ("snap.ln1_rstd", Me * 2)})


def run(e):
    loss = e.forward(f, p, c).clone()
    e.backward()
    out = {"loss": loss.cpu().numpy().view(np.uint32)}
    for w, (name, n) in BUFS.items():
        buf = np.empty(n, np.uint16)
        _lib.check(lib.capgen_debug_copy_buffer(e.h, w, buf.ctypes.data_as(C.c_void_p), n * 2))
        out[name] = buf
    return out


def mk():
    e = Engine(cfg.replace(dtype="bf16"), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_training(False)
    return e


ndiff = 0
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for it in range(iters):
    a, b = mk(), mk()
    ra, rb = run(a), run(b)
    bad = []
    for name, (va) in ra.items():
        vb = rb[name]
        idx = np.nonzero(va != vb)[0]
        if len(idx) and name == "loss":
            bad.append("loss")
        elif len(idx):
            width = len(va) // Me
            rows, cols = idx // width, idx % width
            bad.append(f"{name}: {len(idx)} elems, rows {sorted(set(rows.tolist()))[:12]} cols {cols.min()}-{cols.max()}")
    if bad:
        ndiff += 1
        print(f"iter {it}: " + " | ".join(bad), flush=True)
    del a, b
print(f"SUMMARY stop={os.environ.get('CAPGEN_DEBUG_BWD_STOP')} diverging {ndiff}/{iters}", flush=True)
