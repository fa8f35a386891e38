"""Benchmark: SegFormer/MiT-b2-EVP LFB feature extraction (generate_evp_LFB.py's hot loop) on
MI355X — frames/s at 224x224 with optical-flow fusion, return_features=True ([B, 2048]).

One step = one forward of a B-frame batch (default B = 256) whose frames, segmaps and flow are
already resident in HBM.  Multi-GPU: one process per GPU (torchrun), frames shard across ranks
with no data-path collective: weak scaling, value = all ranks' frames / the
slowest rank's time.  Rank 0 prints ONE JSON line.

Roofline: the dominant kernel (the MFMA GEMM / implicit-GEMM conv instantiation with the most
device time) is timed live with HIP events around each of its launches inside the timed region;
achieved = its algorithmic 2*M*N*K flops / its measured time.  cpu_baseline: the oracle (the
reference's op graph restated on torch CPU ops, fp32) on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"))

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}     # MI355X dense MFMA (MI355X_MICROARCH.md)


def synthetic_batch(B, dev, seed):
    """Cholec80-shaped synthetic inputs generated on the device."""
    g = torch.Generator(device=dev).manual_seed(seed)
    mean = torch.tensor([0.41757566, 0.26098573, 0.25888634], device=dev).view(1, 1, 3, 1, 1)
    std = torch.tensor([0.21938758, 0.1983, 0.19342837], device=dev).view(1, 1, 3, 1, 1)
    x = (torch.randint(0, 256, (B, 1, 3, 224, 224), generator=g, device=dev).float() / 255. - mean) / std
    yy = torch.arange(224, device=dev).view(1, 224, 1).float()
    xx = torch.arange(224, device=dev).view(1, 1, 224).float()
    cy, cx = torch.rand(B, 1, 1, generator=g, device=dev) * 224, torch.rand(B, 1, 1, generator=g, device=dev) * 224
    m = ((((yy - cy) / 40.) ** 2 + ((xx - cx) / 60.) ** 2) <= 1).float()
    y = (m.view(B, 1, 1, 224, 224).expand(B, 1, 3, 224, 224) - mean) / std
    flow = 2.0 * torch.randn(B, 1, 2, 224, 224, generator=g, device=dev)
    return x.contiguous(), y.contiguous(), flow


def cpu_baseline(variant, budget_s=20.0, batch=4):
    """Oracle (torch CPU, fp32, the reference's op order) on a bounded sample of the same workload."""
    from oracle import inputs as I, params as P, mit_evp as M, shapes as SH
    cores = torch.get_num_threads()
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 0)
    x, y, fl = I.frames(batch, 1), I.segmaps(batch, 1), I.flow(batch, 1)
    with torch.no_grad():
        M.forward(x, y, sd, variant, fl, return_features=True)          # warm-up
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s or n == 0:
            M.forward(x, y, sd, variant, fl, return_features=True)
            n += 1
        dt = time.perf_counter() - t0
    return {"value": round(n * batch / dt, 3), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{n} batches x {batch} frames ({variant} + flow, fp32, return_features) in {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--variant", default="mit_b2_evp")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-flow", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump-gemm", default=None, help="write per-shape GEMM timings to this file (rank 0)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import svk
    from svk import ops
    from models import mix_transformer_evp as mte

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)                      # random-init weights of the real architecture
    model = getattr(mte, args.variant)()
    model.svk_dtype = dtype
    model = model.to(dev).eval()
    for p in model.parameters():
        p.requires_grad_(False)
    x, y, fl = synthetic_batch(args.batch, dev, seed=1234 + rank)
    if args.no_flow:
        fl = None

    def step():
        return model(x, y, fl, return_features=True)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        records = []
        ops.set_profiler(records)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ops.set_profiler(None)
    assert out.shape == (args.batch, 2048) and torch.isfinite(out).all()

    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    elapsed = float(dt.item())
    frames = world * args.batch * args.steps
    value = frames / elapsed

    # dominant kernel: the GEMM instantiation with the most measured device time
    per, shapes = {}, {}
    for name, flops, nbytes, s, e, shape in records:
        ms = s.elapsed_time(e)
        for key, d in ((name, per), ((name, str(shape)), shapes)):
            tot = d.setdefault(key, [0.0, 0.0, 0.0, 0])
            tot[0] += ms
            tot[1] += flops
            tot[2] += nbytes
            tot[3] += 1
    if args.dump_gemm and rank == 0:
        with open(args.dump_gemm, "w") as f:
            for (name, shape), (ms, fl, nb, n) in sorted(shapes.items(), key=lambda kv: -kv[1][0]):
                f.write(f"{ms / args.steps:8.3f} ms/step n={n // args.steps:3d} {fl / ms / 1e9:8.1f} TF/s "
                        f"{nb / ms / 1e6:8.1f} GB/s  {shape:28s} {name}\n")
    gemm_ms = sum(v[0] for v in per.values())
    name, (ms, flops, nbytes, n) = max(per.items(), key=lambda kv: kv[1][0])
    achieved = flops / (ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    roofline = {"bound": "mfma", "kernel": name, "achieved": round(achieved, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None,
                "launches_per_step": n // args.steps, "avg_launch_us": round(ms * 1e3 / n, 2),
                "algorithmic_flop_per_launch": flops / n,
                "all_gemm_tflops": round(sum(v[1] for v in per.values()) / (gemm_ms * 1e-3) / 1e12, 2),
                "gemm_share_of_step": round(gemm_ms / (elapsed * 1e3), 3)}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.variant, args.cpu_baseline_seconds)
        line = {"metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                "data": "synthetic (seeded Cholec80-shaped frames/segmaps/flow, resident in HBM; random-init weights)",
                "config": {"workload": f"generate_evp_LFB feature extraction: {args.variant} + "
                                       f"{'no flow' if args.no_flow else 'optical-flow cross-attn fusion'}, "
                                       f"224x224, return_features -> [B, 2048]",
                           "model": args.variant, "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                           "parallelism": f"dp{world} (frame shards, no collective)"},
                "roofline": roofline, "cpu_baseline": cpu, "svk": svk.version()}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
