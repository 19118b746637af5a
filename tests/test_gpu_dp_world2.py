"""The engine's data-parallel path with several ranks: the RCCL count / partial-CE
all-reduces and the per-bucket gradient all-reduce (ZERO=0) or ZeRO-1 reduce-scatter + all-gather
(ZERO=1, the default at world > 1) of engine.hip, run by `world` processes through one communicator.
Needs that many GPUs: RCCL refuses two ranks on one device ("Duplicate GPU detected",
tools/rccl_two_ranks_one_gpu.py on the one-GPU box), so on a one-GPU box these skip --
except the world-1 runs of the same launcher and worker, which run everywhere.

- world 2: each rank trains on half of the c1 fixture batch; three fp32 steps must give every rank
  bit-identical parameters (exact checksum), the same global loss (model.py:76's mean over the GLOBAL
  batch), and the parameters of one world-1 engine trained on the whole batch (summation order only).
- world 8 (C3 exactly): the C2 model, 8 ranks x 64 images (bench.py's per-rank synthetic batches),
  fp32, ZERO=1, against ONE engine at B = 512 on the concatenated batch.
Every worker also runs the forced consistency check (capgen_dp_check) after its steps."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from capgen.params import fixture_state_dict
from golden_util import fixture_inputs, load_fixture

pytestmark = pytest.mark.gpu


def _gpus(n):
    return pytest.mark.skipif(torch.cuda.device_count() < n,
                              reason=f"{n} ranks need {n} GPUs (RCCL refuses two ranks on one device)")


HERE = os.path.dirname(os.path.abspath(__file__))
STEPS = 3


def _launch(tmp_path, world, zero, port, tag="c1", steps=STEPS, timeout=100):
    out = str(tmp_path / f"dp_{tag}_w{world}_z{zero}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(HERE, "dp_world2_worker.py"), tag, str(zero), str(steps), out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [np.load(f"{out}.r{k}.npz") for k in range(world)]


def _full_batch():
    """One world-1 engine (no communicator) trained on the whole fixture batch."""
    from capgen.engine import Engine
    cfg, seed, z = load_fixture("c1")
    f, p, c = (t.to("cuda:0") for t in fixture_inputs(z))
    e = Engine(cfg.replace(dtype="fp32"), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_training(False)
    losses = [e.train_step(f, p, c).item() for _ in range(STEPS)]
    torch.cuda.synchronize()
    params = e.params_arena()
    e.close()
    return losses, params


def test_dp_launcher_world1_fp32(tmp_path):
    """The launcher + worker of the multi-rank tests at world 1 (runs on a one-GPU box): the engine's
    communicator has one rank, the step equals the plain engine's, and the forced consistency check
    (capgen_dp_check -- the exchange the first step runs by itself at world > 1) passes through its
    RCCL max / min all-reduces with both loss forms."""
    (r0,) = _launch(tmp_path, 1, 1, 29620)
    assert int(r0["comm"][0]) == 1
    losses, params = _full_batch()
    np.testing.assert_allclose(r0["losses"], losses, rtol=1e-5, atol=0)
    np.testing.assert_allclose(r0["params"], params, atol=1e-6, rtol=0)


def test_dp_check_needs_a_communicator():
    """capgen_dp_check without capgen_dp_init is an error (non-zero status -> RuntimeError), not a
    silent pass."""
    from capgen.engine import Engine
    cfg, seed, z = load_fixture("c1")
    e = Engine(cfg.replace(dtype="fp32"), "cuda:0")
    try:
        f, p, c = (t.to("cuda:0") for t in fixture_inputs(z))
        e.train_step(f, p, c)
        with pytest.raises(RuntimeError, match="communicator"):
            e.dp_check(None)
    finally:
        e.close()


def test_dp_check_world1_forced():
    """The forced check in-process at world 1 after a train step (and a step of the indexed path,
    which now runs the same first-step check at world > 1): passes, and it does not disturb the
    engine (the next step's loss is the plain engine's)."""
    from capgen.engine import Engine
    cfg, seed, z = load_fixture("c1")
    sd = fixture_state_dict(cfg, seed=seed, with_buffer=False)
    f, p, c = (t.to("cuda:0") for t in fixture_inputs(z))
    runs = []
    for dp in (False, True):
        e = Engine(cfg.replace(dtype="fp32"), "cuda:0")
        e.load_state_dict(sd)
        e.set_training(False)
        if dp:
            e.dp_init(Engine.dp_unique_id(), 0, 1)
        l0 = e.train_step(f, p, c).item()
        if dp:
            e.dp_check(e._loss)
            e.dp_check(None)
        idx = torch.arange(c.shape[0], dtype=torch.int32, device="cuda:0")
        e.train_step_indexed(f.contiguous(), p.contiguous(), idx, c)
        if dp:
            e.dp_check(None)
        l2 = e.train_step(f, p, c).item()
        runs.append((l0, l2))
        e.close()
    assert runs[0][0] == pytest.approx(runs[1][0], rel=1e-5)
    assert runs[0][1] == pytest.approx(runs[1][1], rel=1e-5)


@_gpus(2)
@pytest.mark.parametrize("zero,port", [(0, 29621), (1, 29622)])
def test_dp_world2_equals_full_batch_fp32(tmp_path, zero, port):
    ranks = _launch(tmp_path, 2, zero, port)
    for z in ranks:
        assert int(z["comm"][0]) == 2
    assert ranks[0]["checksum"][0] == ranks[1]["checksum"][0]
    np.testing.assert_array_equal(ranks[0]["params"], ranks[1]["params"])
    np.testing.assert_array_equal(ranks[0]["losses"], ranks[1]["losses"])
    losses, params = _full_batch()
    np.testing.assert_allclose(ranks[0]["losses"], losses, rtol=1e-5, atol=0)
    # three Adam steps (lr 5e-4): the halves' gradient sum differs from the full batch's by
    # summation order only
    np.testing.assert_allclose(ranks[0]["params"], params, atol=2e-6, rtol=0)


@_gpus(8)
def test_dp_world8_c3_equals_global_batch_512_fp32(tmp_path):
    """C3 exactly (BASELINE configs[2]): 8 ranks x 64 images of the C2 model, fp32, ZeRO-1, three
    steps, against one engine at B = 512 on the concatenated batch.  Every rank: the same global loss
    at every step and bit-identical parameters (exact checksum); the loss of every step within 1e-5 of
    the B = 512 engine's (model.py:76's global mean); after step 1 each parameter within 2e-6 of the
    B = 512 engine's, except where that engine's gradient is within fp32 summation noise of zero
    (|g| <= 1e-5 max|g|): there Adam's first update lr * g / (|g| + eps) can take either sign under a
    different summation order."""
    ranks = _launch(tmp_path, 8, 1, 29623, tag="c3", timeout=600)
    for z in ranks:
        assert int(z["comm"][0]) == 8
        assert z["checksum"][0] == ranks[0]["checksum"][0]
        np.testing.assert_array_equal(z["losses"], ranks[0]["losses"])
    np.testing.assert_array_equal(ranks[0]["params"], ranks[7]["params"])
    from capgen.config import preset
    from capgen.engine import Engine
    from capgen.params import reference_init_state_dict
    sys.path.insert(0, HERE)
    from dp_world2_worker import c3_batch
    cfg = preset("C2")
    parts = [c3_batch(cfg, r) for r in range(8)]
    f, p, c = (torch.cat([x[i] for x in parts]).to("cuda:0") for i in range(3))
    e = Engine(cfg.replace(dtype="fp32"), "cuda:0")
    e.load_state_dict(reference_init_state_dict(cfg, seed=0, with_buffer=False))
    e.set_training(False)
    losses = [e.train_step(f, p, c).item()]
    torch.cuda.synchronize()
    p1, g1 = e.params_arena(), e.grads_arena()
    losses += [e.train_step(f, p, c).item() for _ in range(STEPS - 1)]
    e.close()
    np.testing.assert_allclose(ranks[0]["losses"], losses, rtol=1e-5, atol=0)
    d = np.abs(ranks[0]["params1"] - p1)
    noisy = np.abs(g1) <= 1e-5 * np.abs(g1).max()
    bad = (d > 2e-6) & ~noisy
    assert not bad.any(), (int(bad.sum()), float(d[bad].max()))
    assert d.max() <= 2 * 5e-4 + 1e-6
