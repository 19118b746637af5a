"""The engine's data-parallel path with TWO ranks: the RCCL count / partial-CE
all-reduces and the per-bucket gradient all-reduce (ZERO=0) or ZeRO-1 reduce-scatter + all-gather
(ZERO=1, the default at world > 1) of engine.hip, run by two processes through one communicator.
Needs two GPUs: RCCL refuses two ranks on one device ("Duplicate GPU detected",
tools/rccl_two_ranks_one_gpu.py on the one-GPU box), so on a one-GPU box this skips.

Each rank trains on half of the c1 fixture batch; three fp32 steps must give every rank bit-identical
parameters (exact checksum), the same global loss (model.py:76's mean over the GLOBAL batch), and
the parameters of one world-1 engine trained on the whole batch (summation order only)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from capgen.params import fixture_state_dict
from golden_util import fixture_inputs, load_fixture

pytestmark = pytest.mark.gpu
two_gpus = pytest.mark.skipif(torch.cuda.device_count() < 2,
                              reason="two ranks need two GPUs (RCCL refuses two ranks on one device)")

HERE = os.path.dirname(os.path.abspath(__file__))
STEPS = 3


def _launch(tmp_path, world, zero, port):
    out = str(tmp_path / f"dp_w{world}_z{zero}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(HERE, "dp_world2_worker.py"), "c1", str(zero), str(STEPS), out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100)
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
    """The launcher + worker of the world-2 test at world 1 (runs on a one-GPU box): the engine's
    communicator has one rank and the step equals the plain engine's."""
    (r0,) = _launch(tmp_path, 1, 1, 29620)
    assert int(r0["comm"][0]) == 1
    losses, params = _full_batch()
    np.testing.assert_allclose(r0["losses"], losses, rtol=1e-5, atol=0)
    np.testing.assert_allclose(r0["params"], params, atol=1e-6, rtol=0)


@two_gpus
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
