"""CPU: host-side logic of the boundary (synthetic data, decode_captions, vocab loading,
checkpoint mapping, DP exact-mean rule over gloo)."""
import os
import pickle
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from capgen import preset
from capgen.params import fixture_state_dict, reference_init_state_dict, reference_param_specs, sinusoid_table
from capgen.synthetic import synthetic_batch
from capgen.utils import decode_captions, load_word_to_idx


def test_synthetic_batch_structure():
    f, p, c = synthetic_batch(64, 36, 2048, 84, 20, 10000, seed=0)
    assert f.shape == (64, 36, 2048) and p.shape == (64, 36, 84) and c.shape == (64, 20)
    assert (f >= 0).all()
    pad = torch.count_nonzero(p, dim=2) == 0
    assert pad.any() and not pad[:, 0].any()                # row 0 = whole image, never padding
    assert (f[pad] == 0).all()                              # padded regions zero in both tensors
    nv = (~pad).sum(1)
    assert nv.min() >= 12 and nv.max() <= 36
    assert (c[:, 0] == 1).all()
    assert ((c == 2).sum(1) == 1).all()                     # exactly one <END>
    assert (c[c > 2] >= 4).all()
    f2, _, _ = synthetic_batch(64, 36, 2048, 84, 20, 10000, seed=0)
    assert torch.equal(f, f2)


def test_decode_captions_rules():
    idx = {0: "<NULL>", 1: "<START>", 2: "<END>", 3: "a", 4: "cat", 5: "sits"}
    caps = np.array([[1, 3, 4, 5, 2, 3, 0], [1, 3, 0, 4, 0, 0, 0]])
    assert decode_captions(caps, idx) == ["a cat sits .", "a cat"]
    assert decode_captions(np.array([1, 4, 2]), idx) == ["cat ."]


def test_vocab_loader_accepts_data_pickle_and_refuses_code():
    with tempfile.TemporaryDirectory() as d:
        good = os.path.join(d, "word_index.pkl")
        with open(good, "wb") as f:
            pickle.dump({"<NULL>": 0, "<START>": 1, "<END>": 2}, f)
        assert load_word_to_idx(good)["<END>"] == 2
        bad = os.path.join(d, "evil.pkl")
        with open(bad, "wb") as f:
            pickle.dump(np.zeros(3), f)   # needs find_class -> refused
        with pytest.raises(pickle.UnpicklingError):
            load_word_to_idx(bad)


def test_state_dict_specs_and_inits():
    cfg = preset("C1")
    for sd in (fixture_state_dict(cfg, 0), reference_init_state_dict(cfg, 0)):
        names = [n for n, _ in reference_param_specs(cfg)] + ["decoder.position_embedding.pos_table"]
        assert list(sd) == names
        assert np.all(sd["decoder.word_embedding.weight"][0] == 0)
        assert sd["decoder.position_embedding.pos_table"].shape == (1, cfg.max_length - 1, 128)
    t = sinusoid_table(5, 8)
    assert np.allclose(t[0, 0::2], 0) and np.allclose(t[0, 1::2], 1)


def _dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from capgen.dp import global_target_count, local_target_count
    from oracle import capgen_oracle as O
    cfg = preset("C1")
    f, p, c = synthetic_batch(8, 8, 512, 84, 10, 1000, seed=5, min_valid=4)
    sl = slice(rank * 4, rank * 4 + 4)
    P = O.make_params(fixture_state_dict(cfg, 0, with_buffer=False))
    logits = O.forward_logits(P, cfg, f[sl], p[sl], c[sl], training=False)
    tgt = c[sl].long()[:, 1:].reshape(-1)
    summed = torch.nn.functional.cross_entropy(logits.reshape(-1, 1000), tgt, ignore_index=0, reduction="sum")
    n_glob = global_target_count(c[sl])
    (summed / n_glob).backward()            # exact-mean rule: local sum / GLOBAL count
    g = torch.cat([v.grad.reshape(-1) for v in P.values()])
    dist.all_reduce(g)
    loss = torch.tensor([summed.item() / n_glob])
    dist.all_reduce(loss)
    if rank == 0:
        out.put((loss.item(), g.numpy(), local_target_count(c[sl])))
    dist.destroy_process_group()


def test_dp_exact_mean_gloo_world2_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    loss_dp, g_dp, _ = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    from oracle import capgen_oracle as O
    cfg = preset("C1")
    f, p, c = synthetic_batch(8, 8, 512, 84, 10, 1000, seed=5, min_valid=4)
    P = O.make_params(fixture_state_dict(cfg, 0, with_buffer=False))
    loss, _ = O.forward_loss(P, cfg, f, p, c, training=False)
    loss.backward()
    g = torch.cat([v.grad.reshape(-1) for v in P.values()]).numpy()
    assert abs(loss.item() - loss_dp) < 1e-5
    np.testing.assert_allclose(g_dp, g, atol=1e-6, rtol=1e-4)


def _boot_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from capgen.dp import global_target_count, init_engine_dp, local_target_count, shard_seed

    class RecEngine:  # stands in for Engine.dp_init (the RCCL side needs a GPU per rank)
        def dp_init(self, uid, r, w):
            self.args = (uid, r, w)

    made = []

    def unique_id():  # rank 0 only: the RCCL unique id's 128 bytes
        made.append(rank)
        return bytes((7 * i + 3) % 256 for i in range(128))

    eng = RecEngine()
    init_engine_dp(eng, rank, world, unique_id=unique_id)
    _, _, caps = synthetic_batch(4 + 3 * rank, 6, 16, 84, 12, 1000, seed=shard_seed(1000, rank), min_valid=2)
    out.put((rank, eng.args, made, local_target_count(caps), global_target_count(caps)))
    dist.destroy_process_group()


def test_dp_bootstrap_gloo_world2():
    """capgen/dp.py's bootstrap over a real process group (gloo, world 2): rank 0 alone makes the
    unique id, every rank's dp_init receives rank 0's 128 bytes with its own rank and the world size,
    and the global non-pad count (the CE denominator, model.py:76) is the sum of the ranks' local
    counts on both ranks, for ranks with different batch sizes and caption padding."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_boot_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    uid0 = bytes((7 * i + 3) % 256 for i in range(128))
    locals_ = [r[3] for r in res]
    assert locals_[0] != locals_[1]
    for rank, (uid, r, w), made, _, glob in res:
        assert uid == uid0 and r == rank and w == 2
        assert made == ([0] if rank == 0 else [])
        assert glob == sum(locals_)


def test_train_loop_cadence_matches_main_py(tmp_path):
    """capgen.train.train restates main.py:25-153: train_step per batch, compute_loss on the two
    fixed eval batches every 100 steps, a greedy sample every 2500, per-epoch valid captions +
    checkpoint.  Driven here with a recording stand-in model on the CPU (no engine calls)."""
    import pickle
    import numpy as np
    import torch
    from capgen.train import train

    class Rec:
        def __init__(self):
            self.calls = []

        def train_step_resident(self, store, idx, caps):
            self.calls.append(("step", int(idx.shape[0])))

        def compute_loss(self, object_features, position_features, target_caption):
            self.calls.append(("loss", int(object_features.shape[0])))
            return {"loss": torch.tensor(float(target_caption.shape[0]))}

        def generate_caption(self, object_features, position_features, beam_size=None):
            self.calls.append(("gen", int(object_features.shape[0])))
            return [f"c{k}" for k in range(object_features.shape[0])], None

        def decode_captions(self, ids):
            return [str(r) for r in ids.tolist()]

        def save(self, path):
            open(path, "wb").close()
            self.calls.append(("save", os.path.basename(path)))

    def split(n_img, n_cap, seed):
        r = np.random.default_rng(seed)
        return {"features": r.random((n_img, 3, 8), dtype=np.float32),
                "positions": r.random((n_img, 3, 5), dtype=np.float32),
                "captions": r.integers(1, 9, (n_cap, 6)).astype(np.int32),
                "image_idxs": r.integers(0, n_img, n_cap).astype(np.int32)}

    m = Rec()
    logs = []
    hist = train(m, split(5, 23, 0), split(4, 9, 1), num_epoch=2, batch_size=4, output_path=str(tmp_path),
                 eval_every=2, sample_every=5, log=logs.append, device="cpu", feature_dtype=torch.float32)
    steps = [c for c in m.calls if c[0] == "step"]
    assert len(steps) == 2 * 6 and steps[5] == ("step", 3)     # 23 captions / 4 -> 6 batches, last partial
    # epoch 1: eval at steps 2,4,6 (2 losses each), a sample at step 5, then 3 zipped eval batches
    e1 = m.calls[:m.calls.index(("save", "model_1.pt")) + 1]
    assert sum(c[0] == "loss" for c in e1) == 3 * 2 + 3 * 2
    assert ("gen", 1) in e1 and sum(c[0] == "gen" for c in e1) == 1 + 3
    assert ("save", "model_2.pt") in m.calls and os.path.exists(tmp_path / "model" / "model_2.pt")
    with open(tmp_path / "valid" / "valid.candidate.captions.pkl", "rb") as fh:
        caps = pickle.load(fh)  # written by this test's own run
    assert len(caps) == 4 and all(c.startswith("c") for c in caps if c)
    assert len(hist) == 2 and hist[0]["loss"]["valid"] > 0
