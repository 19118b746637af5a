"""Where two engines' bucketed c2s bf16 steps part (the intermittent encoder-side divergence):
every engine runs forward/backward then two train_steps with CAPGEN_DEBUG_ENC_SNAP=1; after each
train_step the encoder chain's gradient after the Wkv_all input gradient and after every encoder
block is copied out.  Engine 0 is compared with engines 1..n-1: first differing slot per step."""
import ctypes as C
import json
import os
import sys

SNAP = os.environ.get("SNAP", "0") == "1"  # 1: also copy the chain gradient during the run (perturbs timing)
if SNAP:
    os.environ["CAPGEN_DEBUG_ENC_SNAP"] = "1"
CHAIN = os.environ.get("CHAIN", "0") == "1"  # 1: every block's gR / input gradient in its own buffer
if CHAIN:
    os.environ["CAPGEN_DEBUG_ENC_CHAIN"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from capgen import _lib  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402
from golden_util import load_fixture  # noqa: E402

lib = _lib.load()
cfg, seed, z = load_fixture("c2s")
cfg = cfg.replace(dropout=0.3, attention_dropout=0.3)
f, p, c = [torch.from_numpy(z[k]).to("cuda:0") for k in ("feats", "pos", "caps")]
Le = cfg.encode_num_blocks
Me = f.shape[0] * f.shape[1]
nel = Me * cfg.encode_input_size


FE = cfg.encode_hidden_size
NAMES = []


def snaps(e):
    """In chain order: eO, then per block l = Le-1 .. 0: gAf, gH, (gR), gA1, gATT1, gQKV, block output."""
    out = []
    names = []

    def grab(which, n, name):
        buf = np.empty(n, dtype=np.uint16)
        _lib.check(lib.capgen_debug_copy_buffer(e.h, which, buf.ctypes.data_as(C.c_void_p), n * 2))
        out.append(buf)
        names.append(name)
    for l in range(Le + 1):
        grab(80 + l, nel, f"forward X[{l}]")
    if CHAIN:  # the saved forward tensors the backward reads (f32 statistics as 2 x u16 per row)
        for l in range(Le):
            for j, nm in enumerate(("att", "v1", "m1", "r1", "Y", "v2", "m2", "r2")):
                grab(128 + 8 * l + j, 2 * Me if nm[0] in "mr" else nel, f"forward block {l} {nm}")
    if SNAP:
        grab(16 + Le, nel, "eO")
    if CHAIN:
        grab(13, nel, "eO")
    for l in range(Le - 1, -1, -1):
        for j, (nm, n) in enumerate((("gAf", nel), ("gH", Me * FE), ("gA1", nel), ("gATT1", nel), ("gQKV", 3 * nel))):
            grab(32 + 8 * l + j, n, f"block {l} {nm}")
            if SNAP and nm == "gH":
                grab(16 + Le + 1 + l, nel, f"block {l} gR")
            if CHAIN and nm == "gH":
                grab(96 + l, nel, f"block {l} gR")
        if CHAIN:
            grab(112 + l, nel, f"block {l} input grad")
        if SNAP:
            grab(16 + l, nel, f"after block {l}")
    NAMES[:] = names
    return out


def run():
    e = Engine(cfg.replace(dtype="bf16"), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_rng_seed(11)
    e.forward(f, p, c)
    e.backward()
    fb = snaps(e)
    e.set_rng_seed(11)
    if os.environ.get("ALT") == "1":  # a different batch for step 1 (the two images swapped): a read of a
        # line left from the previous call would now differ grossly, not by an ulp
        e.train_step(f.flip(0).contiguous(), p.flip(0).contiguous(), c.flip(0).contiguous())
    else:
        e.train_step(f, p, c)
    s1 = snaps(e)
    e.train_step(f, p, c)
    s2 = snaps(e)
    g = e.grads_state_dict()
    del e
    return fb, s1, s2, g


def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if not np.array_equal(x, y):
            xf = (x.astype(np.uint32) << 16).view(np.float32)
            yf = (y.astype(np.uint32) << 16).view(np.float32)
            rows = np.nonzero((x != y).reshape(Me, -1).any(1))[0]
            cols = np.nonzero((x != y).reshape(Me, -1).any(0))[0]
            later = [f"{NAMES[j]}:{int((u != v).sum())}" for j, (u, v) in enumerate(zip(a, b))
                     if j > i and not np.array_equal(u, v)][:6]
            return {"slot": NAMES[i], "n_elems": int((x != y).sum()), "cols": cols[:12].tolist(), "later": later,
                    "rows": rows[:12].tolist(), "n_rows": int(len(rows)),
                    "max_abs": float(np.nanmax(np.abs(xf - yf))),
                    "row_absmax": float(np.nanmax(np.abs(xf.reshape(Me, -1)[rows]))),
                    "zero_flips": int(((xf == 0) != (yf == 0)).sum()),
                    "ulps": int(np.abs(x.astype(np.int32) - y.astype(np.int32)).max())}
    return None


runs = [run() for _ in range(int(os.environ.get("N_ENGINES", "4")))]
for k in range(1, len(runs)):
    rep = {"engine": k}
    for j, name in enumerate(("fb", "step1", "step2")):
        rep[name] = first_diff(runs[0][j], runs[k][j])
    print(json.dumps(rep), flush=True)
