"""One rank of a data-parallel run of the engine (launched by tests/test_gpu_dp_world2.py
through torch.distributed.run; rank r on GPU r).

Each rank trains the fp32 engine for three steps on its half of a fixture batch through the engine's
own RCCL communicator (count all-reduce, per-bucket gradient all-reduce or ZeRO-1 reduce-scatter /
all-gather, engine.hip) and writes its parameters, losses, checksum and communicator size to
<out>.r<rank>.npz.  torch.distributed (gloo) is only the bootstrap channel for the unique id."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "image-caption_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    tag, zero, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    from capgen import _lib
    from capgen.dp import init_engine_dp
    from capgen.engine import Engine
    from capgen.params import fixture_state_dict
    from golden_util import fixture_inputs, load_fixture

    _lib.set_knob("ZERO", zero)
    dev = f"cuda:{rank}"
    cfg, seed, z = load_fixture(tag)
    f, p, c = (t.to(dev) for t in fixture_inputs(z))
    e = Engine(cfg.replace(dtype="fp32"), dev)
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_training(False)
    init_engine_dp(e, rank, world)
    h = c.shape[0] // world
    sl = slice(rank * h, (rank + 1) * h)
    losses = [e.train_step(f[sl], p[sl], c[sl]).item() for _ in range(steps)]
    torch.cuda.synchronize()
    np.savez(f"{out}.r{rank}.npz", params=e.params_arena(), losses=np.array(losses),
             checksum=np.array([e.params_checksum()], dtype=np.uint64),
             comm=np.array([e.dp_comm_info()[0]]))
    dist.barrier()
    e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
