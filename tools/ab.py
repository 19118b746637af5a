"""Alternating A/B runs of bench.py (one parameterised driver for every step-time comparison).

  python tools/ab.py --rounds 3 --arm base:CAPGEN_LIB_PATH=image-caption_amd/capgen/libcapgen_base.so \
                     --arm new: [--steps 50] [--out gpurun_out/ab.jsonl]

Each arm is `name:ENV=VAL,ENV=VAL` (empty after the colon = the default build and settings).  The arms
run in turn, `rounds` times, each bench a child process with its own time limit (a box that
misbehaves ends the run instead of looping).  Prints per arm the ms/step of every round and the
in-step kernel classes (bench.py dominant_kernel) of its last round; appends every line to --out.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", action="append", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--timeout", type=int, default=150)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "ab.jsonl"))
    args = ap.parse_args()
    arms = []
    for a in args.arm:
        name, _, envs = a.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        arms.append((name, env))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    res = {n: [] for n, _ in arms}
    last = {}
    for r in range(args.rounds):
        for name, env in arms:
            e = dict(os.environ)
            e.update(env)
            cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--steps", str(args.steps), "--warmup",
                   str(args.warmup), "--no-cpu-baseline", "--no-host-batches"]
            p = subprocess.run(cmd, env=e, cwd=REPO, capture_output=True, text=True, timeout=args.timeout)
            if p.returncode != 0:
                print(f"[{name}] round {r}: rc {p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            res[name].append(line["ms_per_step"])
            last[name] = line.get("dominant_kernel", {}).get("classes_us_per_step")
            with open(args.out, "a") as fh:
                fh.write(json.dumps({"arm": name, "env": env, "round": r, "line": line}) + "\n")
            print(f"[{name}] round {r}: {line['ms_per_step']:.4f} ms/step  loss {line.get('final_loss')}", flush=True)
    for name, _ in arms:
        print(json.dumps({"arm": name, "ms_per_step": res[name], "classes_us_per_step": last[name]}), flush=True)


if __name__ == "__main__":
    main()
