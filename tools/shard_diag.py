"""Where the emulated ZeRO-1 ranks' assembled parameters differ from the full bucketed Adam
(tests/test_gpu_parity.py _sharded_update_check, fp32): per parameter tensor, the count and the
largest difference, per step; for a differing bucket, whether the gradients agree, where in the
rank's chunk the differences sit and the ratio of the two updates.  DIAG_PAD=n creates n engines
first (shifts which hardware queues the engines' streams share).
python tools/shard_diag.py [world] [steps]   (round 6: the split-tail experiment, DESIGN Appendix A)"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import test_gpu_parity as T  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg, seed, z = T.load_fixture("c2s")
f, p, c = T._inputs(z)
pad = [T._engine(cfg, seed) for _ in range(int(os.environ.get("DIAG_PAD", "0")))]  # shifts stream creation order
ref = T._engine(cfg, seed)
ranks = [T._engine(cfg, seed) for _ in range(world)]
# DIAG_REF0="NAME=VALUE": a second full engine built with that switch (capgen_set_knob), to tell which
# side is wrong when the switch under test changes the step's stream schedule
ref0 = None
if os.environ.get("DIAG_REF0"):
    from capgen import _lib  # noqa: E402
    kname, kval = os.environ["DIAG_REF0"].split("=")
    old = _lib.set_knob(kname, int(kval))
    ref0 = T._engine(cfg, seed)
    _lib.set_knob(kname, old)
    ref0.set_training(False)
before = ref.params_arena()
for r, e in enumerate(ranks):
    e.set_training(False)
    e.dp_debug_shard(r, world)
ref.set_training(False)
for step in range(steps):
    ref.train_step(f, p, c)
    for e in ranks:
        e.train_step(f, p, c)
    want = ref.params_arena()
    if ref0 is not None:
        ref0.train_step(f, p, c)
        w0 = ref0.params_arena()
        t0 = 1e-6 * np.abs(w0).max()
        print(f"step {step}: ref vs ref0: {int((np.abs(want - w0) > t0).sum())} over", flush=True)
    got = np.full_like(want, np.nan)
    for r, e in enumerate(ranks):
        pr = e.params_arena()
        for off, n in ref.dp_buckets():
            ch = n // world
            got[off + r * ch: off + (r + 1) * ch] = pr[off + r * ch: off + (r + 1) * ch]
    tol = 1e-6 * np.abs(want).max()
    if ref0 is not None:
        print(f"step {step}: ranks vs ref0: {int((np.abs(got - w0) > t0).sum())} over", flush=True)
    bad = np.abs(got - want) > tol
    print(f"step {step}: {int(bad.sum())} elements over {tol:.3g}", flush=True)
    for name, ndim, rows, cols, off, ld in ref.table:
        n = (rows - 1) * ld + cols if ndim == 2 else rows
        b = bad[off: off + n]
        if b.any():
            print(f"   {name}: {int(b.sum())} of {n}, max {np.abs(got - want)[off: off + n].max():.3g}")
    if bad.any():
        # the gradients the updates used: equal between ref and the owning rank?
        gref = ref.grads_arena()
        idx = np.flatnonzero(bad)
        for off, n in ref.dp_buckets():
            sel = idx[(idx >= off) & (idx < off + n)]
            if sel.size == 0:
                continue
            ch = n // world
            owner = (sel - off) // ch
            for r in np.unique(owner)[:3]:
                gr = ranks[r].grads_arena()
                s_ = sel[owner == r]
                print(f"   bucket ({off}, {n}) rank {r}: {s_.size} bad, grads equal on them: "
                      f"{np.array_equal(gr[s_], gref[s_])}, max |dg| {np.abs(gr[s_] - gref[s_]).max():.3g}, "
                      f"grads equal on the whole chunk: {np.array_equal(gr[off + r * ch: off + (r + 1) * ch], gref[off + r * ch: off + (r + 1) * ch])}; "
                      f"first bad: got {got[s_[0]]:.6g} want {want[s_[0]]:.6g} g {gref[s_[0]]:.3g}")
                rel = s_ - (off + r * ch)
                blocks = np.unique(rel // 4096)
                du, dw = got[s_] - before[s_], want[s_] - before[s_]
                print(f"      chunk-relative {rel.min()}..{rel.max()}, 4096-blocks {blocks[:12].tolist()} ({blocks.size}), "
                      f"bad in block: {[int(((rel // 4096) == b).sum()) for b in blocks[:6]]}; "
                      f"update ratio got/want median {np.median(du / dw):.4g} [{np.percentile(du / dw, 5):.3g}, {np.percentile(du / dw, 95):.3g}]")
    for e in ranks + [ref] + ([ref0] if ref0 is not None else []):
        e.set_params_arena(got)
    before = got
