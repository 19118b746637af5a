"""Headline benchmark (BASELINE.json `metric`): train images/sec at batch 64 per GPU,
36x2048 region features, seq_len 20, the 6+6-block d_model=512 h=8 Transformer (C2),
bf16 MFMA path, synthetic data resident in HBM, random-init weights.

One step = TRANSFORMER.train_step (forward + backward + [RCCL all-reduce] + Adam) over
one 64-image batch per GPU.  N>1: launched by torch.distributed.run, one rank per GPU,
weak scaling (64 images per rank), exact global-mean CE.

Prints ONE JSON line (rank 0).  `roofline` is the whole train step on the MFMA roof
(519.9157 GFLOP per 64-image step), plus the step's dominant kernel class timed in
the step (in-kernel timestamps);
`cpu_baseline` times the CPU oracle (fp32 eager torch, train mode) on this host.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "image-caption_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train images/sec @ batch=64, 36×2048 feats, seq_len=20; 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2516.6          # 256 CU x 4096 FLOP/clk x 2.4 GHz (dense)
GFLOP_PER_IMAGE = 8.12368          # SURVEY §8(d) closed form == torch.profiler count
B, N, T = 64, 36, 20


def step_flops_per_image(cfg, N, T):
    """SURVEY §8(d) closed form: train = 3*fwd - 2BN(F+P)d (no dX for the feature embed)."""
    d, f, V = cfg.encode_input_size, cfg.encode_hidden_size, cfg.num_vocab
    F, P, L = cfg.encode_dim_features, cfg.encode_dim_positions, T - 1
    Le, Ld = cfg.encode_num_blocks, cfg.decode_num_blocks
    emb = 2 * N * (F + P) * d
    fwd = (emb + Le * (N * (8 * d * d + 4 * d * f) + 4 * N * N * d) + 2 * L * d * d
           + Ld * (L * (8 * d * d + 4 * d * f) + 4 * L * L * d + 4 * L * d * d + 4 * N * d * d + 4 * L * N * d)
           + 2 * L * d * V)
    return 3 * fwd - emb


def dominant_class(eng, args, steps=3):
    """The step's dominant kernel class measured IN the step: every GEMM / LayerNorm / attention launch
    of a train step records the GPU's 100 MHz real-time counter at its first workgroup's start and its
    last workgroup's end (capgen_debug_stamps, no profiler); run `steps` stamped steps after the timed
    region, group the launches by class, and price the class with the largest summed time per step
    (the NN input-gradient GEMMs at C2) at its algorithmic FLOPs / its summed launch durations -- only when
    every launch of the class ran on one stream (launches on different streams overlap, and their summed
    durations would overstate the class's time).  Runs train steps: call it after every measurement that
    needs the engine's state."""
    from collections import defaultdict
    eng.stamps(1)
    for _ in range(2):
        eng.train_step_raw(*args)
    torch.cuda.synchronize()
    cls = defaultdict(lambda: [0, 0.0, 0.0, set()])  # launches, us, flops, streams
    for _ in range(steps):
        eng.stamps(3)
        eng.train_step_raw(*args)
        torch.cuda.synchronize()
        for name, t0, t1 in eng.stamps(2):
            if t1 <= 0 or t0 <= 0 or t1 < t0:
                continue
            words = name.split()  # "<stream> gemm dX MxNxK" / "<stream> ln_bwd M" / ...
            if len(words) < 2:
                continue
            kind = " ".join(words[1:3]) if words[1] == "gemm" and len(words) >= 3 else words[1]
            if words[0] != "crit":  # launches off the critical stream form classes of their own
                kind = words[0] + " " + kind
            fl = 0.0
            if words[1] == "gemm" and "x" in words[-1]:
                m, n_, k = (int(x) for x in words[-1].split("x"))
                fl = 2.0 * m * n_ * k
            c = cls[kind]
            c[0] += 1
            c[1] += t1 - t0
            c[2] += fl
            c[3].add(words[0])
    eng.stamps(0)
    kind, (n, us, fl, streams) = max(cls.items(), key=lambda kv: kv[1][1])
    avg_us = us / n
    tf = fl / (us * 1e-6) / 1e12 if fl and len(streams) == 1 else None
    names = {"gemm dX": "gemm_bf16_kernel NN input-gradient GEMMs (dX = dY . W)", "gemm fwd": "gemm_bf16_kernel NT forward GEMMs"}
    return {"kernel": names.get(kind, kind) + ", in-step class (stamped launches: first workgroup start -> last workgroup end)",
            "streams": sorted(streams),
            "launches_per_step": round(n / steps, 1), "us_per_step": round(us / steps, 1), "avg_us": round(avg_us, 2),
            "achieved": round(tf, 1) if tf else None, "unit": "TFLOP/s",
            "frac": round(tf / PEAK_BF16_TFLOPS, 4) if tf else None,
            "classes_us_per_step": {k: round(v[1] / steps, 1) for k, v in sorted(cls.items(), key=lambda kv: -kv[1][1])}}


def _pmc_traffic():
    """HBM bytes per train step from the COMMITTED rocprofv3 PMC passes (FETCH_SIZE x2 per the
    gfx950 correction + WRITE_SIZE, summed over one step's kernels; tools/pmcsum.py) -- a file
    measured on this code by tools/round_profile.sh, not in this run (PMC needs its own passes)."""
    import glob
    found = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]_pmc_traffic.json")))
    if not found:
        return None
    path = found[-1]  # the newest round's passes
    with open(path) as fh:
        d = json.load(fh)
    return {"bytes_per_step": d["hbm_bytes_per_step"], "source": os.path.relpath(path, REPO),
            "commit": d.get("commit", "unrecorded")}


def cpu_baseline(cfg, steps=5, warmup=2, c1_steps=50):
    """The pinned CPU oracle (fp32 eager torch, train mode = dropout on) on this host's cores:
    a bounded sample of the same workload (same B/N/T/model) -> images/s, SURVEY §8(d): 2 warm-up +
    5 timed steps at C2 (the reported value) and 2 + 50 at C1 (reported beside it).  Threads: torch's
    intra-op pool as configured for this box (OMP_NUM_THREADS; os.cpu_count() reports the whole host,
    of which one GPU box owns a share)."""
    sys.path.insert(0, REPO)
    from oracle import capgen_oracle as O
    from capgen import preset
    from capgen.params import reference_init_state_dict
    from capgen.synthetic import synthetic_batch
    threads = torch.get_num_threads()

    def time_steps(c, b, n, t, warm, timed):
        f, p, cap = synthetic_batch(b, n, c.encode_dim_features, c.encode_dim_positions, t, c.num_vocab, seed=1000)
        P = O.make_params(reference_init_state_dict(c.replace(dtype="fp32"), seed=0))
        opt = O.make_adam(P, c)
        for _ in range(warm):
            O.train_step(P, opt, c, f, p, cap, training=True)
        t0 = time.perf_counter()
        for _ in range(timed):
            O.train_step(P, opt, c, f, p, cap, training=True)
        return (time.perf_counter() - t0) / timed

    dt = time_steps(cfg, B, N, T, warmup, steps)
    c1 = preset("C1", dropout=0.3)
    dt1 = time_steps(c1, 8, 8, 10, warmup, c1_steps)
    return {"value": round(B / dt, 2), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{warmup} warm-up + {steps} timed C2 train steps (B={B}, fp32 eager torch CPU, dropout on), "
                      f"{dt:.3f} s/step; C1 (B=8): {warmup} + {c1_steps} steps, {dt1 * 1e3:.1f} ms/step",
            "c1_value": round(8 / dt1, 1)}


def host_batches(eng, cfg, dev, steps=20, warmup=5):
    """Secondary line: the unchanged-main.py rate -- TRANSFORMER.train_step's host path
    (capgen/staging.py: pageable CPU f32 batches -> pinned slot -> side-stream H2D overlapped with
    the previous step -> indexed step), wall-clock over `steps` steps.  PCIe and the host copy
    are inside the timed region, so this is never `value`."""
    from capgen.staging import HostBatchStager
    from capgen.synthetic import synthetic_batch
    batches = [synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab,
                               seed=2000 + i) for i in range(3)]
    batches = [(f.float().contiguous(), p.float().contiguous(), c) for f, p, c in batches]
    st = HostBatchStager(dev, B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T)
    for i in range(warmup):
        st.run(eng, *batches[i % 3])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        st.run(eng, *batches[i % 3])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(B * steps / el, 1), "unit": "images/s", "ms_per_step": round(el / steps * 1e3, 4),
            "steps": steps, "kind": "TRANSFORMER.train_step host path (pageable CPU f32 batches; pinned "
                                    "double-buffered staging, side-stream H2D, PCIe inclusive)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", action="store_true", help="replay the step as one hipGraph (slower on ROCm 7)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-host-batches", action="store_true", help="skip the secondary host-batch line")
    ap.add_argument("--dp1", action="store_true",
                    help="diagnostic: run the engine's RCCL data-parallel step at world size 1 (its collectives and, with CAPGEN_ZERO=2, the sharded update) to price the DP machinery on one GPU")
    args = ap.parse_args()

    from capgen import preset
    from capgen.engine import Engine
    from capgen.params import reference_init_state_dict
    from capgen.synthetic import synthetic_batch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = preset("C2", dtype=args.dtype, dropout=0.3)   # config.py:61 DROPOUT; attention 0.1
    eng = Engine(cfg, dev)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in reference_init_state_dict(cfg, seed=0).items()})
    eng.set_graph(args.graph)
    if world > 1 or args.dp1:
        from capgen.dp import init_engine_dp
        init_engine_dp(eng, rank, world)

    f, p, c = synthetic_batch(B, N, cfg.encode_dim_features, cfg.encode_dim_positions, T, cfg.num_vocab,
                              seed=1000 + rank)
    fdt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    f = f.to(dev, fdt).contiguous()
    p = p.to(dev).contiguous()
    c = c.to(dev).contiguous()
    loss = torch.zeros(1, device=dev)
    from capgen import _lib
    ft = _lib.BF16 if fdt == torch.bfloat16 else _lib.F32

    for _ in range(args.warmup):
        eng.train_step_raw(f, ft, p, c, B, N, T, loss)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the stream the step is launched on (the engine forks its side streams
    # off this one and joins them back, so the events bracket the whole step)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        eng.train_step_raw(f, ft, p, c, B, N, T, loss)
    ev1.record(stream)
    issue_s = time.perf_counter() - t0  # host time to enqueue the K steps (no sync inside)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    final_loss = loss.item()
    step_ms_events = ev0.elapsed_time(ev1) / args.steps
    # correctness of a data-parallel run (after the timed region): the communicator the engine's
    # collectives ran on, parameters bit-identical on every rank (exact checksum, min == max over the
    # ranks), every rank holding the same global loss (model.py:76's mean over the global batch)
    comm_n, _ = eng.dp_comm_info()
    dp = {"rccl_ranks": comm_n if comm_n else 1, "engine_communicator": bool(comm_n)}
    if world > 1:
        ck = eng.params_checksum()
        ck = ck - (1 << 64) if ck >= (1 << 63) else ck
        t = torch.tensor([ck, -ck], device=dev, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lt = torch.tensor([final_loss, -final_loss], device=dev, dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        dp["params_equal_across_ranks"] = bool(t[0].item() == -t[1].item())
        dp["global_loss"] = round(final_loss, 6)
        dp["loss_equal_across_ranks"] = bool(lt[0].item() == -lt[1].item())

    images = B * world * args.steps
    value = images / elapsed
    ms = elapsed / args.steps * 1e3
    gfl_img = step_flops_per_image(cfg, N, T) / 1e9
    # roofline unit = one train step: algorithmic FLOP per step
    # (64 images x GFLOP/image) / the event-timed average step on this GPU
    achieved = B * gfl_img / step_ms_events   # GFLOP/ms == TFLOP/s
    traffic = _pmc_traffic()
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (region feats/positions/captions, SURVEY §8(d))",
        "config": {"workload": "C2 train step: B=64/GPU, N=36 regions x F=2048, P=84, T=20, 6+6 blocks d=512 h=8 "
                               "f=2048, V=10000, dropout 0.3/0.1, Adam lr 5e-4",
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 5),
                     "traffic": traffic["bytes_per_step"] if traffic else None,
                     # the commit of the tree the PMC passes profiled: a train path changed since then
                     # makes `traffic` stale, visibly
                     "traffic_commit": traffic["commit"] if traffic else None,
                     "scope": f"one train step = {B} images x {gfl_img:.5f} GFLOP/image "
                              f"algorithmic (SURVEY §8(d)); step time {step_ms_events:.4f} ms from HIP events "
                              f"on the launch stream" + (f"; traffic = HBM bytes/step from the committed PMC "
                                                         f"summary {traffic['source']} (not measured in this run; "
                                                         f"profiled tree: commit {traffic['commit']})"
                                                         if traffic else "")},
        "final_loss": round(final_loss, 5),
        "dp_check": dp,
        # diagnostic: host enqueue time per step; close to ms_per_step means the host issue rate,
        # not the GPU, sets the step time
        "host_issue_ms_per_step": round(issue_s / args.steps * 1e3, 4),
    }
    if rank == 0 and world == 1:
        if not args.no_host_batches:
            out["host_batches"] = host_batches(eng, cfg, dev)
        # (runs stamped train steps: after everything else that uses the engine)
        out["dominant_kernel"] = dominant_class(eng, (f, ft, p, c, B, N, T, loss))
        if not args.no_cpu_baseline:
            del eng
            torch.cuda.empty_cache()
            out["cpu_baseline"] = cpu_baseline(cfg, steps=args.cpu_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
