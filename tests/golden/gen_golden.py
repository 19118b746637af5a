"""Generate the golden fixtures from the REFERENCE implementation (build container only).

Run:  python tests/golden/gen_golden.py        (needs /root/reference; not run on the GPU box)

It imports shao-chi/Image-Caption's `core.TRANSFORMER.model.Transformer` from
/root/reference with two un-vendored imports stubbed (coco-caption's
`core.metrics.*`, imported by loss.py:7-9 but unused on this path, and `hickle`,
imported by core/utils.py:7), loads the deterministic fixture weights
(capgen.params.fixture_state_dict), and records, in eval mode (dropout off):
  * loss and full logits of Transformer.forward (model.py:79-98; logits via a hook
    on `classifer`),
  * per-parameter gradient sums / abs-sums / sampled values after loss.backward(),
  * the loss after a second Adam(lr) step and per-parameter deltas after two steps
    (models.py:111-126),
  * greedy ids + attention_list (model.py:101-132) and beam-5 ids (model.py:135-200).
Only inputs and outputs are written (tests/golden/*.npz); the reference source never
leaves this container.
"""
from __future__ import annotations

import os
import sys
import types
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))

from capgen.config import preset  # noqa: E402
from capgen.params import fixture_state_dict, reference_param_specs  # noqa: E402
from capgen.synthetic import synthetic_batch  # noqa: E402

REF = "/root/reference"
N_SAMPLES = 8


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    for name in ["hickle", "core.metrics", "core.metrics.cider", "core.metrics.cider.cider",
                 "core.metrics.ciderD", "core.metrics.ciderD.ciderD", "core.metrics.bleu",
                 "core.metrics.bleu.bleu"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["core.metrics.cider.cider"].Cider = object
    sys.modules["core.metrics.ciderD.ciderD"].CiderD = object
    sys.modules["core.metrics.bleu.bleu"].Bleu = object
    from core.TRANSFORMER.model import Transformer
    return Transformer


def sample_index(name, numel):
    r = np.random.default_rng(zlib.crc32(name.encode()))
    return np.sort(r.choice(numel, size=min(N_SAMPLES, numel), replace=False))


def build(Transformer, cfg):
    return Transformer(
        num_vocab=cfg.num_vocab, max_length=cfg.max_length,
        encode_dim_positions=cfg.encode_dim_positions, encode_dim_features=cfg.encode_dim_features,
        device="cpu", output_name=cfg.output_name, encode_mask=cfg.encode_mask, pad_idx=cfg.pad_idx,
        dropout=cfg.dropout, encode_input_size=cfg.encode_input_size, encode_q_k_dim=cfg.encode_q_k_dim,
        encode_v_dim=cfg.encode_v_dim, encode_hidden_size=cfg.encode_hidden_size,
        encode_num_blocks=cfg.encode_num_blocks, encode_num_heads=cfg.encode_num_heads,
        dim_word_embedding=cfg.dim_word_embedding, decode_input_size=cfg.decode_input_size,
        decode_q_k_dim=cfg.decode_q_k_dim, decode_v_dim=cfg.decode_v_dim,
        decode_hidden_size=cfg.decode_hidden_size, decode_num_blocks=cfg.decode_num_blocks,
        decode_num_heads=cfg.decode_num_heads)


def make_fixture(tag, cfg, B, N, T, seed, beam_k=5, min_valid=None):
    Transformer = import_reference()
    torch.manual_seed(0)
    model = build(Transformer, cfg)
    sd = {k: torch.from_numpy(v) for k, v in fixture_state_dict(cfg, seed=seed).items()}
    model.load_state_dict(sd, strict=True)
    model.eval()
    feats, pos, caps = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions,
                                       T, cfg.num_vocab, seed=seed + 100, min_valid=min_valid)
    out = {"feats": feats.numpy(), "pos": pos.numpy(), "caps": caps.numpy()}

    logits_box = {}
    h = model.classifer.register_forward_hook(lambda m, i, o: logits_box.__setitem__("x", o.detach()))
    opt = torch.optim.Adam((p for p in model.parameters() if p.requires_grad), lr=cfg.learning_rate)
    before = {k: v.detach().clone() for k, v in model.named_parameters()}

    opt.zero_grad()
    loss = model(object_features=feats, position_features=pos, target_caption=caps)["loss"]
    loss.backward()
    out["loss"] = np.float64(loss.item())
    out["logits"] = logits_box["x"].numpy()
    names = [n for n, _ in reference_param_specs(cfg)]
    params = dict(model.named_parameters())
    assert sorted(names) == sorted(params), "param spec drift vs reference"
    gsum, gabs, gsamp = [], [], []
    for n in names:
        g = params[n].grad.detach().double().reshape(-1)
        gsum.append(g.sum().item())
        gabs.append(g.abs().sum().item())
        gsamp.append(g[sample_index(n, g.numel())].numpy())
    out["grad_sum"], out["grad_abs"] = np.array(gsum), np.array(gabs)
    out["grad_samples"] = np.concatenate(gsamp)
    opt.step()
    opt.zero_grad()
    loss2 = model(object_features=feats, position_features=pos, target_caption=caps)["loss"]
    loss2.backward()
    opt.step()
    out["loss_after_step1"] = np.float64(loss2.item())
    dsum, dabs, dsamp = [], [], []
    for n in names:
        dlt = (params[n].detach() - before[n]).double().reshape(-1)
        dsum.append(dlt.sum().item())
        dabs.append(dlt.abs().sum().item())
        dsamp.append(dlt[sample_index(n, dlt.numel())].numpy())
    out["delta2_sum"], out["delta2_abs"] = np.array(dsum), np.array(dabs)
    out["delta2_samples"] = np.concatenate(dsamp)
    h.remove()

    model.load_state_dict(sd, strict=True)
    model.eval()
    ids, attn = model.generate_caption_vector(object_features=feats, position_features=pos)
    out["greedy_ids"] = ids.numpy()
    out["greedy_attn"] = np.stack(attn).astype(np.float32)
    if beam_k:
        out["beam_ids"] = model.beam_search(object_features=feats, position_features=pos,
                                            beam_size=beam_k).numpy()
        out["beam_k"] = np.int64(beam_k)
    out["seed"] = np.int64(seed)
    out["cfg"] = np.array(repr(cfg))
    path = os.path.join(HERE, f"{tag}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: loss={out['loss']:.6f} loss_after_step1={out['loss_after_step1']:.6f}")


FIXTURES = {
    # tag: (cfg, B, N, T, seed, beam_k, min_valid)
    "c1": (preset("C1"), 8, 8, 10, 0, 5, 4),
    "c1_encmask": (preset("C1", encode_mask=True), 4, 8, 10, 1, 3, 4),
    "c1_focal": (preset("C1", output_name="FocalLoss_Transformer"), 4, 8, 10, 2, 0, 4),
    "c2s": (preset("C2", num_vocab=1000), 2, 36, 20, 3, 5, 12),
}


def main(tags=None):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for tag, (cfg, B, N, T, seed, k, mv) in FIXTURES.items():
        if tags and tag not in tags:
            continue
        make_fixture(tag, cfg, B, N, T, seed, beam_k=k, min_valid=mv)


if __name__ == "__main__":
    main(sys.argv[1:])
