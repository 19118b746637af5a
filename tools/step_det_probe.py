"""Repeat test_train_step_equals_forward_backward_adam_bf16's comparison (bf16 train_step vs
forward -> backward -> adam_step on c2s) and report every 2-D weight that is not bit-identical."""
import os
import sys

sys.path.insert(0, "image-caption_amd")
sys.path.insert(0, "tests")
import torch  # noqa: E402

from golden_util import load_fixture  # noqa: E402
from capgen.engine import Engine  # noqa: E402
from capgen.params import fixture_state_dict  # noqa: E402

cfg, seed, z = load_fixture("c2s")
f, p, c = [torch.from_numpy(z[k]).to("cuda") for k in ("feats", "pos", "caps")]


def mk():
    e = Engine(cfg.replace(dtype="bf16"), "cuda:0")
    e.load_state_dict(fixture_state_dict(cfg, seed=seed, with_buffer=False))
    e.set_training(False)
    return e


def diff(sa, sb):
    return [(k, int((sa[k] != sb[k]).sum().item()), (sa[k] - sb[k]).abs().max().item()) for k in sa
            if sa[k].dim() == 2 and k != "decoder.word_embedding.weight" and not torch.equal(sa[k], sb[k])]


if os.environ.get("PROBE_PROTO"):  # split-K hand-off protocol bits (capgen_debug_splitk_protocol)
    from capgen import _lib
    _lib.check(_lib.load().capgen_debug_splitk_protocol(int(os.environ["PROBE_PROTO"])))
n_diff = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    a, b, c2 = mk(), mk(), mk()
    if os.environ.get("PROBE_GRAPH") == "1":
        a.set_graph(True)          # the whole step as one captured graph
    a.train_step(f, p, c)          # bucketed step
    if os.environ.get("PROBE_SYNC") == "1":
        torch.cuda.synchronize()   # no overlap between the engines
    grads = []
    for e in (b, c2):              # forward -> backward -> adam_step, twice independently
        e.forward(f, p, c)
        e.backward()
        grads.append(e.grads_state_dict())
        e.adam_step()
        if os.environ.get("PROBE_SYNC") == "1":
            torch.cuda.synchronize()
    gb, gc = grads
    worst = max(((gb[k].double() - gc[k].double()).norm() / (gb[k].double().norm() + 1e-30)).item() for k in gb
                if k.startswith("encoder.") or k.startswith("decoder.decoder."))
    print(f"iter {it}: unfused-vs-unfused gradient max rel L2 diff {worst:.2e}", flush=True)
    torch.cuda.synchronize()
    sa, sb, sc = a.state_dict(False), b.state_dict(False), c2.state_dict(False)
    dab, dbc = diff(sa, sb), diff(sb, sc)
    def short(d):
        return sorted({k.replace("encoder.encoder.", "e").replace("decoder.decoder.", "d").split(".")[0]
                       if "coder." in k else k for k, _, _ in d})
    print(f"iter {it}: step-vs-unfused {len(dab)} {short(dab)} | unfused-vs-unfused {len(dbc)} {short(dbc)}",
          flush=True)
    n_diff += bool(dab or dbc)
    if os.environ.get("PROBE_PROTO"):
        import ctypes as C
        from capgen import _lib
        d4 = (C.c_int * 4)()
        _lib.check(_lib.load().capgen_debug_splitk_diag(d4, 1))
        print(f"iter {it}: split-K diag: out-of-range tickets {d4[0]}, tiles combined {d4[1]}", flush=True)
    if dbc and n_diff <= 3:  # which gradients of the two unfused engines differ, in arena order
        for k in gb:
            r = ((gb[k].double() - gc[k].double()).norm() / (gb[k].double().norm() + 1e-30)).item()
            if r > 0:
                print(f"    grad {k}: rel {r:.2e}", flush=True)
    del a, b, c2
print(f"SUMMARY proto={os.environ.get('PROBE_PROTO', 'default')} diverging iterations {n_diff}/{it + 1}", flush=True)
