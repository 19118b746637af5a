"""C5-style SCST train step on 1 GPU (BASELINE.json configs[4] runs it on 8): B=64 images,
36 x 2048 regions, T=20, the C2 model, bf16; one step = rl_sample (GPU) -> host CIDEr-D +
BLEU-4 scoring (capgen/scst.py) -> rl_finish (GPU: loss, backward, Adam).  Synthetic
vocabulary "w<i>" (V=10000) and random-init weights.  Prints one JSON line with the step
time split into GPU-sample, host-scoring and GPU-finish parts."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from capgen import preset  # noqa: E402
from capgen.models import SelfCriticNetwork  # noqa: E402
from capgen.params import reference_init_state_dict  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402


def main(steps=20, warmup=3):
    cfg = preset("C2", dtype="bf16", dropout=0.3)
    vocab = {"<NULL>": 0, "<START>": 1, "<END>": 2}
    vocab.update({f"w{i}": i for i in range(3, cfg.num_vocab)})
    sd = {k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()}
    m = SelfCriticNetwork(config=cfg, word_to_idx=vocab, device="cuda:0", state_dict=sd)
    B, N, T = 64, 36, 20
    f, p, c = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab, seed=1000)
    f = f.cuda().bfloat16()
    p, c = p.cuda(), c.cuda()
    eng = m.model.engine
    t_s = t_h = t_f = 0.0
    for i in range(warmup + steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        seq, ent, _ = eng.rl_sample(f, p, c)
        seq_h, ent_h = seq.cpu().numpy(), ent.cpu().numpy()
        t1 = time.perf_counter()
        reward = np.broadcast_to(m.scorer.scores(c[:, 1:].cpu().numpy(), seq_h), (B,))
        total = m.scorer.total(reward, ent_h)
        t2 = time.perf_counter()
        out = eng.rl_finish(total, m.structure_loss_weight, train=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if i >= warmup:
            t_s, t_h, t_f = t_s + t1 - t0, t_h + t2 - t1, t_f + t3 - t2
    ms = 1e3 * (t_s + t_h + t_f) / steps
    print(json.dumps({"metric": "SCST train images/sec (C5 step on 1 GPU: B=64, 36x2048 feats, T=20)",
                      "value": round(B / (ms / 1e3), 1), "unit": "images/s", "ms_per_step": round(ms, 3),
                      "split_ms": {"gpu_sample": round(1e3 * t_s / steps, 3), "host_reward": round(1e3 * t_h / steps, 3),
                                   "gpu_finish": round(1e3 * t_f / steps, 3)},
                      "final_loss": round(float(out[0].item()), 4), "dtype": "bf16", "data": "synthetic"}))


if __name__ == "__main__":
    main()
