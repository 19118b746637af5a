"""Ordering of the multi-stream step (VERDICT r2 "Next round" item 1, item 6).

The engine runs a step on three HIP streams (critical path, weight gradients, gradient buckets)
ordered only by events.  These tests check that ordering mechanically and under perturbation:

* the hazard checker (csrc/hazard.h) logs every launch's stream and device byte ranges, every
  event edge and host sync, and reports launches on different streams that touch the same bytes
  (one of them writing) without an ordering edge -- for every scheduling mode of the step;
* a deliberately dropped edge (CAPGEN_DEBUG_DROP_JOIN) must be reported (the checker works);
* deterministic delay injection (a spin kernel in front of every side-stream launch) must leave
  the bf16 weight gradients and the first step's weights bit-identical to an undelayed engine;
* data parallel: ranks with DIFFERENT batches must issue the identical RCCL call sequence;
* the persisted GEMM autotune table covers the benchmarked step (no live tuning)."""
import pytest
import torch

from capgen import _lib
from capgen.params import fixture_state_dict
from golden_util import load_fixture

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _engine(cfg, seed, dtype="bf16", dropout=0.3):
    from capgen.engine import Engine
    cfg = cfg.replace(dropout=dropout, attention_dropout=dropout)
    e = Engine(cfg.replace(dtype=dtype), DEV)
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    return e


def _inputs(z):
    return [torch.from_numpy(z[k]).to(DEV) for k in ("feats", "pos", "caps")]


MODES = {
    "default": {},
    "serial_dec0": {"CAPGEN_OVERLAP_DEC0": "0"},
    "front_after_encoder": {"CAPGEN_OVERLAP_FRONT": "0"},
    "single_dw_launches": {"CAPGEN_GROUP_DW": "0"},
    "colsum_in_epilogue": {"CAPGEN_COLSUM_SIDE": "0"},
    "two_blocks_per_bucket": {"CAPGEN_BUCKET_BLOCKS": "2"},
    "stripe_memset": {"CAPGEN_STRIPE_CLEAR": "0"},
    "dp_world1_sharded": {"CAPGEN_ZERO": "2"},
}


def _logged_run(e, f, p, c):
    """Tune + warm outside the log, then log: forward/backward (gradients only) and two bucketed
    train steps back to back (the step boundary: next forward vs the previous step's buckets)."""
    e.train_step(f, p, c)
    e.forward(f, p, c)
    e.backward()
    torch.cuda.synchronize()
    _lib.hazard_start()
    try:
        e.forward(f, p, c)
        e.backward()
        e.train_step(f, p, c)
        e.train_step(f, p, c)
        torch.cuda.synchronize()
        return _lib.hazard_check()
    finally:
        _lib.hazard_stop()


@pytest.mark.parametrize("mode", list(MODES))
def test_step_has_no_unordered_conflicts(mode, set_knob):
    for k, v in MODES[mode].items():
        set_knob(k.removeprefix("CAPGEN_"), v)
    cfg, seed, z = load_fixture("c2s")
    e = _engine(cfg, seed)
    if mode.startswith("dp_"):
        from capgen.engine import Engine
        e.dp_init(Engine.dp_unique_id(), 0, 1)
    n, report = _logged_run(e, *_inputs(z))
    assert n == 0, f"{n} unordered conflicting launch pairs:\n{report}"


@pytest.mark.parametrize("tag", ["c1_imgobj", "c1_movefirst", "c1_focal"])
def test_variant_steps_have_no_unordered_conflicts(tag):
    cfg, seed, z = load_fixture(tag)
    e = _engine(cfg, seed)
    n, report = _logged_run(e, *_inputs(z))
    assert n == 0, f"{n} unordered conflicting launch pairs:\n{report}"


_DROPPED_EDGE = r"""
import sys
sys.path[:0] = [REPO, REPO + "/image-caption_amd", REPO + "/tests"]
from capgen import _lib
assert _lib.debug_build(), "expected libcapgen_debug.so"
_lib.set_knob("DEBUG_DROP_JOIN", 1)
import test_gpu_hazard as T
from golden_util import load_fixture
cfg, seed, z = load_fixture("c2s")
e = T._engine(cfg, seed)
n, report = T._logged_run(e, *T._inputs(z))
print("UNORDERED", n, "stream" in report)
"""


def test_checker_reports_a_dropped_edge():
    """Self-test: without the side-stream join at the end of backward the checker must flag the
    next launches that touch what the side stream wrote (weight gradients, the decoder folds).  The
    dropped edge is a debug-build switch (libcapgen_debug.so, make debug): one child process loads it."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dbg = os.path.join(repo, "image-caption_amd", "capgen", "libcapgen_debug.so")
    assert os.path.exists(dbg), "build the debug library: make -C image-caption_amd/csrc debug"
    env = dict(os.environ, CAPGEN_LIB_PATH=dbg)
    out = subprocess.run([sys.executable, "-c", f"REPO = {repo!r}\n" + _DROPPED_EDGE], env=env, capture_output=True,
                         text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("UNORDERED")][-1].split()
    assert int(line[1]) > 0, "the checker missed a deliberately dropped event edge"
    assert line[2] == "True"


def test_side_stream_delay_leaves_bf16_results_bit_identical():
    """Deterministic delay injection: a 40 us spin in front of every launch off the critical
    stream (weight-gradient groups, bias sums, decoder-embedding branch, bucket Adam).  Linear
    weight gradients (deterministic GEMMs) and the weights after one bucketed step must equal an
    undelayed engine's bit for bit -- any missing edge would let a consumer read early."""
    cfg, seed, z = load_fixture("c2s")
    f, p, c = _inputs(z)
    res = []
    for delay in (40.0, 0.0):
        e = _engine(cfg, seed)
        e.set_rng_seed(11)
        _lib.side_delay(delay)
        try:
            e.forward(f, p, c)
            e.backward()
            g = e.grads_state_dict()
            e.set_rng_seed(11)
            loss = e.train_step(f, p, c).item()
            torch.cuda.synchronize()
            w = e.state_dict(False)
        finally:
            _lib.side_delay(0.0)
        res.append((g, loss, w))
    (ga, la, wa), (gb, lb, wb) = res
    lin = [k for k in ga if ga[k].dim() == 2 and k != "decoder.word_embedding.weight"]
    bad = [k for k in lin if not torch.equal(ga[k], gb[k])]
    assert not bad, ("gradients", bad[:8])
    assert la == lb
    bad = [k for k in lin if not torch.equal(wa[k], wb[k])]
    assert not bad, ("weights", bad[:8])
    for k in wa:  # LayerNorm / bias / embedding: f32 atomic sums, last bits only
        torch.testing.assert_close(wa[k], wb[k], atol=1e-5, rtol=0, msg=k)


def test_dp_ranks_with_different_batches_issue_identical_collectives(set_knob):
    """Two RCCL world-1 engines standing in for two ranks (sharded update forced, the world > 1
    forward graph) with DIFFERENT batches -- batch size, caption length and padding differ -- must
    enqueue the same RCCL calls (op, bytes, stream) in the same order, or real ranks deadlock."""
    from capgen.engine import Engine
    from capgen.synthetic import synthetic_batch
    set_knob("ZERO", 2)
    cfg, seed, z = load_fixture("c2s")
    batches = [_inputs(z)]
    fb, pb, cb = synthetic_batch(3, z["feats"].shape[1], cfg.encode_dim_features, cfg.encode_dim_positions,
                                 12, cfg.num_vocab, seed=5, min_valid=3)
    batches.append([t.to(DEV) for t in (fb, pb, cb)])
    logs = []
    for f, p, c in batches:
        e = _engine(cfg, seed)
        e.dp_init(Engine.dp_unique_id(), 0, 1)
        e.collectives_log(1)
        for _ in range(3):
            e.train_step(f, p, c)
        e.forward(f, p, c)
        e.backward()
        torch.cuda.synchronize()
        logs.append(e.collectives_log(2))
        e.collectives_log(0)
    assert logs[0] == logs[1], (logs[0][:2000], logs[1][:2000])
    assert "reduce_scatter" in logs[0] and "all_gather" in logs[0] and "allreduce(count)" in logs[0]


def test_bench_step_runs_from_the_persisted_tune_table():
    """The committed autotune table (capgen/tune_gfx950.txt, tools/tune_table.py) holds every
    GEMM shape of the benchmarked C2 bf16 step: bench, profiles and tests run the same kernels and
    no shape is tuned inside a live step."""
    import os
    from capgen import preset
    from capgen.engine import Engine
    from capgen.params import reference_init_state_dict
    from capgen.synthetic import synthetic_batch
    assert os.path.exists(_lib.TUNE_TABLE), "tune_gfx950.txt missing (tools/tune_table.py)"
    cfg = preset("C2", dtype="bf16", dropout=0.3)
    e = Engine(cfg, DEV)
    e.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
    f, p, c = synthetic_batch(64, 36, cfg.encode_dim_features, cfg.encode_dim_positions, 20, cfg.num_vocab, seed=1000)
    f = f.to(DEV, torch.bfloat16)
    p, c = p.to(DEV), c.to(DEV)
    before = _lib.tune_live_count()
    for _ in range(2):
        e.train_step(f, p, c)
    torch.cuda.synchronize()
    assert _lib.tune_live_count() == before


def test_stream_events_without_system_fence_track_fenced_events(set_knob):
    """The fork / join / bucket events are created without HIP's system-scope fence (Knob EVENT_FENCE = 1,
    the default): they order this device's own streams, whose kernel dispatches carry their own
    device-scope acquire / release.  Against an engine whose events keep the default fence (0), over
    four bucketed bf16 train steps: after the first step every Linear weight bit-identical, the loss
    equal; later steps (the f32-atomic LayerNorm / bias sums differ in the last bits, so they drift)
    losses within 1e-3 and, per tensor, fewer than 1 % of the elements apart by lr / 2 -- a stale
    read across a stream edge (gradients before their weight-gradient group, weights before their
    bucket's Adam, the next forward before the update) moves whole tensors by ~lr."""
    cfg, seed, z = load_fixture("c2s")
    f, p, c = _inputs(z)
    engines = []
    for fence in (1, 0):
        set_knob("EVENT_FENCE", fence)
        e = _engine(cfg, seed)
        e.set_rng_seed(5)
        engines.append(e)
    a, b = engines
    for step in range(4):
        la, lb = a.train_step(f, p, c).item(), b.train_step(f, p, c).item()
        torch.cuda.synchronize()
        sa, sb = a.state_dict(False), b.state_dict(False)
        if step == 0:
            assert la == lb, (la, lb)
            for k in sa:
                if sa[k].dim() == 2 and k != "decoder.word_embedding.weight":
                    assert torch.equal(sa[k], sb[k]), k
        else:
            assert abs(la - lb) < 1e-3 * abs(lb), (step, la, lb)
            for k in sa:
                frac = ((sa[k] - sb[k]).abs() > 0.5 * cfg.learning_rate).float().mean().item()
                assert frac < 0.01, (step, k, frac)
