"""Build the persisted GEMM autotune table (image-caption_amd/capgen/tune_gfx950.txt) on an MI355X.

Runs every workload whose kernels bench.py, the profiles and the GPU tests time -- the C2 bf16 train
step (also under the DP paths' shapes, which are the same), C4 decode (greedy and beam 5 at B=256),
the SCST sample/finish at C2, the c2s / C1 bf16 test shapes -- with no table loaded, so each GEMM
shape is tuned once on an idle device (gemm_bf16.hip launch_bf16_tiles), then saves the choices.
Afterwards every process loads the table at its first GEMM and tunes nothing live.

  CAPGEN_TUNE_TABLE=0 python tools/tune_table.py [--out PATH]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("CAPGEN_TUNE_TABLE", "0")  # start from nothing
import torch  # noqa: E402

from capgen import _lib, preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict, reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402


def dev_batch(cfg, B, N, T, seed, dev):
    f, p, c = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab, seed=seed)
    return f.to(dev, torch.bfloat16).contiguous(), p.to(dev).contiguous(), c.to(dev).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=_lib.TUNE_TABLE)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    # C2 / C3 / C5 model: train step, SCST, decode
    cfg = preset("C2", dtype="bf16", dropout=0.3)
    eng = Engine(cfg, dev)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
    f, p, c = dev_batch(cfg, 64, 36, 20, 1000, dev)
    for _ in range(2):
        eng.train_step(f, p, c)
    eng.forward(f, p, c)
    eng.backward()
    eng.rl_sample(f, p, c)
    eng.rl_finish(torch.zeros(64), 0.5)
    fg, pg, _ = dev_batch(cfg, 256, 36, 20, 7, dev)
    eng.set_training(False)
    eng.greedy(fg, pg, want_attention=False)
    eng.beam(fg, pg, 5)
    torch.cuda.synchronize()
    print(f"C2/C4/C5 shapes: {_lib.tune_live_count()} tuned", flush=True)
    del eng
    # test shapes (bf16): the c2s fixture config and C1
    from golden_util import load_fixture
    for tag in ("c2s", "c1"):
        fcfg, seed, z = load_fixture(tag)
        e = Engine(fcfg.replace(dtype="bf16", dropout=0.3, attention_dropout=0.3), dev)
        e.load_state_dict(fixture_state_dict(fcfg, seed=seed, with_buffer=False))
        fi, pi, ci = (torch.from_numpy(z[k]).to(dev) for k in ("feats", "pos", "caps"))
        e.train_step(fi, pi, ci)
        e.forward(fi, pi, ci)
        e.backward()
        e.set_training(False)
        e.greedy(fi, pi)
        e.beam(fi, pi, 5)
        torch.cuda.synchronize()
        del e
    print(f"all: {_lib.tune_live_count()} tuned", flush=True)
    n = _lib.tune_save(args.out)
    print(f"wrote {n} entries to {args.out}", flush=True)


if __name__ == "__main__":
    main()
