"""Pin the CPU oracle (oracle/capgen_oracle.py) against golden vectors produced by the
reference implementation itself (tests/golden/gen_golden.py)."""
import numpy as np
import pytest
import torch

from capgen.params import fixture_state_dict, reference_param_specs, sinusoid_table
from golden_util import fixture_inputs, load_fixture, sample_index
from oracle import capgen_oracle as O

TAGS = ["c1", "c1_encmask", "c1_focal", "c2s", "c1_splitpos", "c1_imgobj", "c1_movefirst"]


def _setup(tag):
    cfg, seed, z = load_fixture(tag)
    P = O.make_params(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    x = [torch.from_numpy(z[k]) for k in ("feats", "pos", "caps")]
    return cfg, P, x, z


@pytest.mark.parametrize("tag", TAGS)
def test_forward_loss_logits(tag):
    cfg, P, (f, p, c), z = _setup(tag)
    loss, logits = O.forward_loss(P, cfg, f, p, c, training=False)
    assert abs(loss.item() - float(z["loss"])) < 1e-5
    np.testing.assert_allclose(logits.detach().numpy(), z["logits"], atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("tag", TAGS)
def test_grads_and_adam(tag):
    cfg, P, (f, p, c), z = _setup(tag)
    before = {k: v.detach().clone() for k, v in P.items()}
    opt = O.make_adam(P, cfg)
    opt.zero_grad()
    loss, _ = O.forward_loss(P, cfg, f, p, c, training=False)
    loss.backward()
    names = [n for n, _ in reference_param_specs(cfg)]
    samples = []
    for i, n in enumerate(names):
        g = P[n].grad.double().reshape(-1)
        assert abs(g.sum().item() - z["grad_sum"][i]) <= 1e-4 * max(1.0, z["grad_abs"][i]), n
        assert abs(g.abs().sum().item() - z["grad_abs"][i]) <= 1e-4 * max(1.0, z["grad_abs"][i]), n
        samples.append(g[sample_index(n, g.numel())].numpy())
    np.testing.assert_allclose(np.concatenate(samples), z["grad_samples"], atol=1e-5, rtol=1e-3)
    opt.step()
    opt.zero_grad()
    loss2, _ = O.forward_loss(P, cfg, f, p, c, training=False)
    loss2.backward()
    opt.step()
    assert abs(loss2.item() - float(z["loss_after_step1"])) < 1e-4
    for i, n in enumerate(names):
        d = (P[n].detach() - before[n]).double().reshape(-1)
        assert abs(d.abs().sum().item() - z["delta2_abs"][i]) <= 1e-3 * max(1e-6, z["delta2_abs"][i]) + 1e-6, n


@pytest.mark.parametrize("tag", ["c1", "c1_encmask", "c2s"])
def test_greedy_and_beam(tag):
    cfg, P, (f, p, c), z = _setup(tag)
    P = {k: v.detach() for k, v in P.items()}
    ids, attn = O.greedy(P, cfg, f, p)
    np.testing.assert_array_equal(ids.numpy(), z["greedy_ids"])
    np.testing.assert_allclose(np.stack(attn), z["greedy_attn"], atol=1e-5)
    k = int(z["beam_k"])
    np.testing.assert_array_equal(O.beam(P, cfg, f, p, k).numpy(), z["beam_ids"])


@pytest.mark.parametrize("tag", ["c1_policy", "c2s_policy"])
def test_policy_network_greedy_and_beam(tag):
    """PolicyNetwork decoding (model_RL.py:100-199, log-softmax scoring) vs the reference's own
    output; c1_policy also differs from the Transformer's probability beam on some images."""
    cfg, seed, z = load_fixture(tag)
    P = O.make_params(fixture_state_dict(cfg, seed=seed, with_buffer=False), requires_grad=False)
    f, p = (torch.from_numpy(z[k]) for k in ("feats", "pos"))
    ids, attn = O.greedy(P, cfg, f, p, log_softmax=True)
    np.testing.assert_array_equal(ids.numpy(), z["greedy_ids"])
    np.testing.assert_allclose(np.stack(attn), z["greedy_attn"], atol=1e-5)
    k = int(z["beam_k"])
    np.testing.assert_array_equal(O.beam(P, cfg, f, p, k, log_softmax=True).numpy(), z["beam_ids"])
    np.testing.assert_array_equal(O.beam(P, cfg, f, p, k).numpy(), z["transformer_beam_ids"])
    if tag == "c1_policy":
        assert (z["beam_ids"] != z["transformer_beam_ids"]).any()


def test_sinusoid_table_matches_oracle():
    np.testing.assert_array_equal(sinusoid_table(19, 512), O.sinusoid_table(19, 512).numpy())


def test_masks_fire_in_fixtures():
    """The fixtures exercise padded regions and padded captions."""
    for tag in TAGS:
        _, _, z = load_fixture(tag)
        assert (np.count_nonzero(z["pos"], axis=2) == 0).any(), tag
        assert (z["caps"] == 0).any(), tag


def rl_setup(tag):
    """SCST fixtures: fixture weights (+ the pad-id bias boost the generator applied)."""
    cfg, seed, z = load_fixture(tag)
    sd = fixture_state_dict(cfg, seed=seed, with_buffer=False)
    sd["classifer.bias"] = sd["classifer.bias"].copy()
    sd["classifer.bias"][0] += float(z["pad_bias_boost"])
    x = fixture_inputs(z)
    base = float(z["cider_reward_weight"]) * z["inj_cider"] + float(z["bleu_reward_weight"]) * z["inj_bleu"]
    return cfg, sd, x, z, base


@pytest.mark.parametrize("tag", ["c5_rl", "c5_rl_pad", "c5_rl_c2s", "c5_rl_c5"])
def test_rl_loss_and_grads(tag):
    """SelfCriticNetwork step mechanics (model_RL.py:75-97, loss.py:31-220) with injected rewards."""
    cfg, sd, (f, p, c), z, base = rl_setup(tag)
    P = O.make_params(sd)
    logits = O.forward_logits(P, cfg, f, p, c, training=False)
    out = O.rl_loss_from_logits(logits, c, base, float(z["structure_loss_weight"]),
                                float(z["entropy_reward_weight"]), float(z["self_cider_reward_weight"]))
    assert (out["sample"].numpy() == z["sample"]).all()
    np.testing.assert_allclose(out["reward"].numpy(), z["reward"], rtol=1e-6)
    for k in ("loss", "language_model_loss", "structure_loss"):
        assert abs(out[k].item() - float(z[k])) < 1e-4 * max(1.0, abs(float(z[k]))), k
    out["loss"].backward()
    names = [n for n, _ in reference_param_specs(cfg)]
    for i, n in enumerate(names):
        g = P[n].grad.double().reshape(-1)
        assert abs(g.abs().sum().item() - z["grad_abs"][i]) <= 1e-4 * max(1.0, z["grad_abs"][i]), n
