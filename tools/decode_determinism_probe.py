"""Probe: are two fresh bf16 engines' C4 decodes (beam 5 and greedy, B = 256, fixture weights)
bit-identical, and is one engine's decode identical across repeated calls?"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-caption_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from capgen.config import preset  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402

cfg = preset("C2")
f, p, _ = synthetic_batch(256, 36, cfg.encode_dim_features, cfg.encode_dim_positions, 20, cfg.num_vocab, seed=1000)
sd = fixture_state_dict(cfg, seed=0, with_buffer=False)
fd, pd = f.to("cuda:0").bfloat16(), p.to("cuda:0")
outs = []
for i in range(2):
    e = Engine(cfg.replace(dtype="bf16"), "cuda:0")
    e.load_state_dict(sd)
    e.set_training(False)
    b1, b2 = e.beam(fd, pd, 5), e.beam(fd, pd, 5)
    g1, _ = e.greedy(fd, pd)
    outs.append((b1, b2, g1))
    e.close()
same = lambda a, b: int((a == b).all(1).sum().item())
print("beam same engine twice:", same(outs[0][0], outs[0][1]), "/ 256")
print("beam two engines:", same(outs[0][0], outs[1][0]), "/ 256")
print("greedy two engines:", same(outs[0][2], outs[1][2]), "/ 256")
