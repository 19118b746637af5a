"""In-step tuning of the NN input-gradient (dX) GEMM shapes of the C2 bf16 train step.

The persisted tune table ranks every variant on an idle device (cold L2).  In the step the dX
GEMMs run beside the weight-gradient groups and the bucketed Adam on the side streams, and the
idle-box ranking need not hold there.  This tool measures each dX shape's
launches IN the step (capgen_debug_stamps: first workgroup start -> last workgroup end), once
per candidate variant forced on every dX shape at once (CAPGEN_GEMM_FORCE, one child process per
candidate), and picks per shape the variant with the smallest in-step time.

  python tools/dx_incontention_tune.py [--fwd]    -> JSON lines: per candidate, per shape us; then
                                                     the choice per shape and the CAPGEN_GEMM_FORCE
                                                     string that pins it (--fwd: the NT forward
                                                     GEMMs instead of the dX ones)
  python tools/dx_incontention_tune.py --worker   (child: one measurement, env set by the parent)
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))

# bf16-output variants (whole 128-B lines) without k-groups, + split-K forms for K = 2048
CANDIDATES = [6, 7, 12, 13, 17, 20, 21, 4, 5, 8, 14, 15, 1, 3, 23, 24, 25, 26, 27, 28, 29, 30,
              206, 217, 221, 406, 417]


FWD = "--fwd" in sys.argv
CLASS, TA, TB = ("fwd", 0, 0) if FWD else ("dX", 0, 1)


def worker():
    import torch
    from capgen import preset, _lib
    from capgen.engine import Engine
    from capgen.params import reference_init_state_dict
    from capgen.synthetic import synthetic_batch
    dev = torch.device("cuda", 0)
    cfg = preset("C2", dtype="bf16", dropout=0.3)
    eng = Engine(cfg, dev)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
    B, N, T = 64, 36, 20
    f, p, c = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab, seed=1000)
    f, p, c = f.to(dev, torch.bfloat16).contiguous(), p.to(dev).contiguous(), c.to(dev).contiguous()
    loss = torch.zeros(1, device=dev)
    args = (f, _lib.BF16, p, c, B, N, T, loss)
    for _ in range(5):
        eng.train_step_raw(*args)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        eng.train_step_raw(*args)
    ev1.record()
    torch.cuda.synchronize()
    step_ms = ev0.elapsed_time(ev1) / 20
    eng.stamps(1)
    for _ in range(2):
        eng.train_step_raw(*args)
    torch.cuda.synchronize()
    shapes, steps = {}, 5
    for _ in range(steps):
        eng.stamps(3)
        eng.train_step_raw(*args)
        torch.cuda.synchronize()
        for name, t0, t1 in eng.stamps(2):
            w = name.split()
            if len(w) >= 4 and w[1] == "gemm" and w[2] == CLASS and t1 > t0 > 0:
                s = shapes.setdefault(w[-1], [0, 0.0])
                s[0] += 1
                s[1] += t1 - t0
    eng.stamps(0)
    print(json.dumps({"step_ms": round(step_ms, 4), "shapes": {k: [v[0] / steps, round(v[1] / steps, 2)]
                                                               for k, v in shapes.items()}}), flush=True)


def run_child(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--worker"] + (["--fwd"] if FWD else []),
                       env=env, capture_output=True,
                       text=True, timeout=240)
    if r.returncode != 0:
        raise RuntimeError(f"worker failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    base = run_child({})
    print(json.dumps({"candidate": "tuned", **base}), flush=True)
    shapes = sorted(base["shapes"])  # "MxNxK" of the dX launches (layout NN: ta = 0, tb = 1)
    best = {s: ("tuned", base["shapes"][s][1]) for s in shapes}
    for v in CANDIDATES:
        force = ";".join(f"{s.replace('x', ',')},{TA},{TB},{v}" for s in shapes
                         if v < 100 or int(s.split("x")[2]) >= 1024)
        if not force:
            continue
        try:
            r = run_child({"CAPGEN_GEMM_FORCE": force})
        except Exception as e:  # (a variant the shape cannot take: skip it)
            print(json.dumps({"candidate": v, "error": str(e)[-300:]}), flush=True)
            continue
        print(json.dumps({"candidate": v, **r}), flush=True)
        for s, (n, us) in r["shapes"].items():
            if s in best and us < best[s][1] and (v < 100 or int(s.split("x")[2]) >= 1024):
                best[s] = (v, us)
    print(json.dumps({"choice": {s: {"variant": b[0], "us_per_step": b[1], "tuned_us": base["shapes"][s][1]}
                                 for s, b in best.items()}}), flush=True)
    force = ";".join(f"{s.replace('x', ',')},{TA},{TB},{b[0]}" for s, b in best.items() if b[0] != "tuned")
    print(json.dumps({"CAPGEN_GEMM_FORCE": force}), flush=True)


if __name__ == "__main__":
    if "--worker" in sys.argv:
        worker()
    else:
        main()
