"""Benchmark of the surgical-phase hot path on MI355X.

Default workload (the headline, BASELINE.json metric): SegFormer/MiT-b2-EVP LFB feature
extraction (generate_evp_LFB.py's hot loop) — frames/s at 224x224 with optical-flow fusion,
return_features=True ([B, 2048]).  One step = one forward of a B-frame batch (default B = 256)
whose frames, segmaps and flow are already resident in HBM.  Other workloads (``--workload``):
``mstcn`` (config 3: MultiStageModel_S(4,10,64,256) over 40 full-length videos), ``mamba``
(config 3 as tecno.py instantiates it at HEAD: CausalMambaModel, the selective-scan path), ``preproc``
(generate_evp_LFB.py's eval transform on decoded 480x854 uint8 frames, Pillow-exact), ``e2e``
(config 5: SegFormer -> MS-TCN(2,8,32,2048) -> Transformer(len 30) on 256-frame chunks) and
``train`` (configs 2/4: the train_evp.py stage-1 step, B = 88 per GPU, DDP over RCCL when N > 1).

Multi-GPU: one process per GPU (torchrun); units shard across ranks with no data-path collective
(SURVEY.md §8(e)): weak scaling, value = all ranks' units / the slowest rank's time.  Rank 0
prints ONE JSON line.

The extraction and train steps replay as HIP graphs (svk.graphs.GraphedForward / EVPTrainStep.capture):
the timed region is graph launches only, no instrumentation.  Roofline: the dominant kernel (the MFMA
GEMM / implicit-GEMM conv instantiation with the most device time) is timed with HIP events around each
of its launches on eager iterations of the same step run right after the timed region (identical
launches); achieved = its algorithmic flops or bytes / its measured time; the rocprofv3 summaries in
profiles/ time the graph-replayed launches themselves.  cpu_baseline: the oracle (the
reference's op graph restated on torch CPU ops, fp32) on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import ast
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"))

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}     # MI355X dense MFMA (MI355X_MICROARCH.md)
TORCH_DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}
# algorithmic work of one extraction frame: the reference formulation of MiT-b2 + flow
# minus the dead head work that the exact resize-first rewrite removes (10.77 - 1.08)
EXTRACT_GFLOP_PER_FRAME = 9.69
# per variant (b3 + flow 16.66 in the reference formulation; the head is the same, so the
# resize-first rewrite removes the same 1.08): the callers' extraction model is mit_b3_evp
# (generate_evp_LFB.py:412)
EXTRACT_GFLOP = {"mit_b2_evp": EXTRACT_GFLOP_PER_FRAME, "mit_b3_evp": 16.66 - 1.08}
# one train_evp stage-1 frame (forward + backward through every frozen block + SGD):
# the count profiles/r03/bench_train.jsonl prices the train step against
TRAIN_GFLOP_PER_FRAME = 25.94
HBM_PEAK_GBS = 8000.0                              # MI355X HBM3E
# on-chip operand-fetch ceiling of an LDS-DMA tile loader: rows served from the XCD's L2 into LDS at 66-73 GB/s
# per CU = 16.8-18.8 TB/s chip-wide (MI355X_MICROARCH.md, 'Indexed rows: gather into LDS'); from the Infinity
# Cache 8.6 TB/s.  The persistent GEMMs stream their A / W tiles through exactly that path.
L2_LDS_PEAK_GBS = 18800.0
DATA = "synthetic (seeded Cholec80-shaped frames/segmaps/flow, resident in HBM; random-init weights)"


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


def _profile_jsons(name):
    """Committed profiles/rNN/<name>, newest round first."""
    base = os.path.join(REPO, "profiles")
    for r in sorted((d for d in os.listdir(base) if d.startswith("r")), reverse=True) if os.path.isdir(base) else []:
        path = os.path.join(base, r, name)
        if os.path.exists(path):
            yield path


def _profile_entry(name, key):
    """(entry, path) of the newest committed profiles/rNN/<name> that holds ``key`` (a round's collection may
    cover only some workloads: older rounds fill the rest)."""
    for path in _profile_jsons(name):
        try:
            with open(path) as f:
                table = json.load(f)
        except (OSError, ValueError):
            continue
        if key in table:
            return table[key], path
    return None, None


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC passes of this workload
    (FETCH_SIZE / WRITE_SIZE in separate passes, gfx950 FETCH correction; tools/pmc_traffic.py)."""
    ent, path = _profile_entry("pmc_traffic.json", workload)
    if ent is None or "kernels" not in ent:
        return None, None
    table = ent["kernels"]
    src = os.path.relpath(path, REPO)
    if kernel in table:
        return table[kernel]["hbm_bytes_per_launch"], src
    # a name without template arguments (e.g. "wgrad_kernel") covers all of its instantiations:
    # dispatch-weighted mean over them
    ents = [v for k, v in table.items() if k.startswith(kernel + "<")]
    n = sum(v["dispatches"] for v in ents)
    if not n:
        return None, None
    return round(sum(v["hbm_bytes_per_launch"] * v["dispatches"] for v in ents) / n), src + " (all instantiations)"


def pmc_mfma_busy(workload, dtype, variant="mit_b2_evp"):
    """Whole-step MFMA busy fraction from the committed rocprofv3 counter pass (tools/pmc_mfma.py):
    sum of SQ_VALU_MFMA_BUSY_CYCLES over the step's kernels / (SIMDs x the step's GPU-active cycles)."""
    rec, path = _profile_entry("pmc_mfma.json",
                               f"{workload}_{dtype}" if variant == "mit_b2_evp" else f"{workload}_{variant}_{dtype}")
    if rec is None:
        return None
    return dict(rec, source=os.path.relpath(path, REPO))


def video_lengths(n=40, seed=0):
    """Seeded test-split-like video lengths, U[1000, 6000] frames at 1 fps."""
    return [int(t) for t in np.random.default_rng(6000 + seed).integers(1000, 6001, size=n)]


# ---------------------------------------------------------------------------------------------
def host_cpus():
    """The host cores the CPU baseline may use, stated the way SURVEY.md §8(d) asks: the CPUs in this
    process's affinity mask (os.sched_getaffinity), the distinct physical cores behind them
    (/proc/cpuinfo physical id + core id), and the cgroup CPU quota (/sys/fs/cgroup/cpu.max) and the job's CPU share (OMP_NUM_THREADS: the GPU box gives a one-GPU job
    16 of its host CPUs).  The baseline runs one thread per usable physical core."""
    aff = sorted(os.sched_getaffinity(0))
    phys, cur = {}, {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if ":" not in line:
                    if "processor" in cur:
                        phys[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                    cur = {}
                    continue
                k, v = (t.strip() for t in line.split(":", 1))
                cur[k] = v
        if "processor" in cur:
            phys[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
    except OSError:
        pass
    cores = len({phys[c] for c in aff if c in phys}) or len(aff)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    usable = min(cores, quota) if quota else cores
    # the GPU box states the job's CPU share in OMP_NUM_THREADS (16 per GPU): never oversubscribe it
    share = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    if share:
        usable = min(usable, share)
    return {"affinity_cpus": len(aff), "physical_cores": cores, "cgroup_cpu_quota": quota, "job_cpu_share": share,
            "threads": usable}


def _cpu_threads():
    info = host_cpus()
    torch.set_num_threads(info["threads"])
    return info


def cpu_baseline_extract(variant, budget_s, batch=4):
    """Oracle (torch CPU, fp32, the reference's op order) on a bounded sample of the same workload."""
    host = _cpu_threads()
    from oracle import inputs as I, params as P, mit_evp as M, shapes as SH
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 0)
    x, y, fl = I.frames(batch, 1), I.segmaps(batch, 1), I.flow(batch, 1)
    with torch.no_grad():
        M.forward(x, y, sd, variant, fl, return_features=True)          # warm-up
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s or n == 0:
            M.forward(x, y, sd, variant, fl, return_features=True)
            n += 1
        dt = time.perf_counter() - t0
    return {"value": round(n * batch / dt, 3), "unit": "frames/s", "cores": torch.get_num_threads(), "host_cpus": host, "kind": "port",
            "sample": f"{n} batches x {batch} frames ({variant} + flow, fp32, return_features) in {dt:.1f} s"}


def cpu_baseline_mstcn(budget_s, T=2456):
    host = _cpu_threads()
    from oracle import params as P, mstcn as MS, shapes as SH, inputs as I
    sd = P.make_state_dict(SH.mstcn_shapes(4, 10, 64, 256, 14), 1)
    x = I.lfb(T, 256, 7).transpose(2, 1)
    with torch.no_grad():
        MS.multi_stage_s(x, sd, 4, 10, True)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s or n == 0:
            MS.multi_stage_s(x, sd, 4, 10, True)
            n += 1
        dt = time.perf_counter() - t0
    return {"value": round(n * T / dt, 1), "unit": "frames/s", "cores": torch.get_num_threads(), "host_cpus": host, "kind": "port",
            "sample": f"{n} videos x {T} frames (MultiStageModel_S(4,10,64,256,14,causal), fp32) in {dt:.1f} s"}


def cpu_baseline_mamba(budget_s, T=2456):
    host = _cpu_threads()
    from oracle import mamba as OM, inputs as I
    sd = OM.init_state_dict(OM.mamba_shapes(256, 64, 10, 14), 1)
    x = I.lfb(T, 256, 7).transpose(2, 1)
    with torch.no_grad():
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s or n == 0:
            OM.causal_mamba(x, sd, 10, dtype=torch.float32)
            n += 1
        dt = time.perf_counter() - t0
    return {"value": round(n * T / dt, 1), "unit": "frames/s", "cores": torch.get_num_threads(), "host_cpus": host, "kind": "port",
            "sample": f"{n} videos x {T} frames (CausalMambaModel(4,10,64,256,14), 10 Mamba blocks d_state 64, "
                      f"fp32 restatement of mamba_ssm's reference scan) in {dt:.1f} s"}


# ---------------------------------------------------------------------------------------------
def workload_extract(args, dev, rank, dtype):
    from models import mix_transformer_evp as mte
    torch.manual_seed(0)                      # random-init weights of the real architecture
    model = getattr(mte, args.variant)()
    model.svk_dtype = dtype
    model = model.to(dev).eval()
    for p in model.parameters():
        p.requires_grad_(False)
    x, y, fl = synthetic_batch(args.batch, dev, seed=1234 + rank)
    if args.no_flow:
        fl = None

    def eager():
        return model(x, y, fl, return_features=True)

    if args.no_graph:
        step = eager
    else:
        from svk.graphs import GraphedForward
        graphed = GraphedForward(model, x, y, fl, return_features=True)   # one graph launch per batch

        def step():
            return graphed()

        step.profile = eager

    def set_dtype(dt):
        model.svk_dtype = dt                   # GraphedForward re-captures on the next call

    step.set_dtype = set_dtype

    def check(out):
        assert out.shape == (args.batch, 2048) and torch.isfinite(out).all()

    config = {"workload": f"generate_evp_LFB feature extraction: {args.variant} + "
                          f"{'no flow' if args.no_flow else 'optical-flow cross-attn fusion'}, "
                          f"224x224, return_features -> [B, 2048]",
              "model": args.variant, "per_gpu_batch": args.batch, "hip_graph": not args.no_graph}
    return step, args.batch, config, check, (lambda: cpu_baseline_extract(args.variant, args.cpu_baseline_seconds))


def workload_lfb(args, dev, rank, dtype):
    """generate_evp_LFB.py's loop end to end from host memory (PCIe-inclusive; not the headline): decoded
    uint8 frames / segmaps [250, 250, 3] and raw f32 flows [250, 250, 2] in pinned host batches -> H2D on a
    copy stream -> GPU frame / flow transforms -> the graph-replayed forward -> features D2H into a pinned
    host bank (svk.lfb.LFBExtractor).  One step = 8 batches of --batch frames; the host-side JPEG decode is
    not part of it (synthetic decoded frames)."""
    from models import mix_transformer_evp as mte
    from svk.lfb import LFBExtractor
    torch.manual_seed(0)
    model = getattr(mte, args.variant)()
    model.svk_dtype = dtype
    model = model.to(dev).eval()
    for p in model.parameters():
        p.requires_grad_(False)
    B, H, W, nb, chunk = args.batch, 250, 250, 4, 8
    g = torch.Generator().manual_seed(1234 + rank)
    batches = []
    for _ in range(nb):
        fr = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8).pin_memory()
        sg = ((torch.rand(B, H, W, 1, generator=g) < 0.2).to(torch.uint8) * 255).expand(B, H, W, 3).contiguous().pin_memory()
        fl = (2.0 * torch.randn(B, H, W, 2, generator=g)).pin_memory()
        batches.append((fr, sg, fl))
    ex = LFBExtractor(model, B, dev, graph=not args.no_graph)
    ex_eager = LFBExtractor(model, B, dev, graph=False)

    def step():
        return ex.run([batches[i % nb] for i in range(chunk)], chunk * B, to_host=True)

    def profile():
        return ex_eager.run(batches[:1], B, to_host=True)

    step.profile = profile

    def check(out):
        assert out.shape == (chunk * B, 2048) and out.is_pinned() and torch.isfinite(out).all()

    per_frame = H * W * 3 * 2 + H * W * 2 * 4
    config = {"workload": f"generate_evp_LFB loop from pinned host memory: decoded uint8 {H}x{W} frames + segmaps and "
                          f"raw f32 flows -> H2D (copy stream, double-buffered) -> GPU Resize(250)/CenterCrop(224)/"
                          f"Normalize + cv2 flow resize -> {args.variant} + flow forward (HIP graph) -> features D2H "
                          f"(pinned bank); {chunk} batches per step",
              "model": args.variant, "per_gpu_batch": B, "h2d_bytes_per_frame": per_frame,
              "d2h_bytes_per_frame": 2048 * 4, "pcie_inclusive": True}
    return step, chunk * B, config, check, (lambda: cpu_baseline_extract(args.variant, args.cpu_baseline_seconds))


def workload_mstcn(args, dev, rank, dtype):
    from models import mstcn
    torch.manual_seed(0)
    model = mstcn.MultiStageModel_S(4, 10, 64, 256, 14, True).to(dev).eval()
    lens = video_lengths(40, seed=rank)
    bank = torch.randn(sum(lens), 256, device=dev)      # the videos' LFB rows, concatenated time-major
    feats = [f[None] for f in torch.split(bank, lens)]

    def step():           # all 40 videos in one ragged pass: one launch per layer (MultiStageModel_S.forward_videos)
        return model.forward_videos(bank, lens)

    def per_video():      # the callers' loop (trans_SV_output.py:251-291): one forward per video
        out = None
        for f in feats:
            out = model(f.transpose(2, 1))
        return out

    def check(out):
        assert out.shape == (4, sum(lens), 14) and torch.isfinite(out).all()
        last = per_video()
        torch.testing.assert_close(model.split_videos(out, lens)[-1], last, rtol=1e-5, atol=1e-5)
        with torch.no_grad():
            for _ in range(2):
                per_video()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            per_video()
            torch.cuda.synchronize()
        config["per_video_loop_frames_s"] = round(sum(lens) / (time.perf_counter() - t0), 1)

    config = {"workload": "tecno.py MS-TCN MultiStageModel_S(4 stages x 10 layers, f_maps 64, f_dim 256, causal) "
                          "over 40 full-length videos (T ~ U[1000, 6000]) per step, one ragged pass "
                          "(forward_videos: one launch per layer for all videos)",
              "model": "MultiStageModel_S(4,10,64,256,14,True)", "videos_per_step": 40}
    return step, sum(lens), config, check, (lambda: cpu_baseline_mstcn(args.cpu_baseline_seconds))


def workload_mamba(args, dev, rank, dtype):
    from models import mstcn
    torch.manual_seed(0)
    model = mstcn.CausalMambaModel(4, 10, 64, 256, 14, True).to(dev).eval()     # tecno.py:153
    lens = video_lengths(40, seed=rank)
    bank = torch.randn(sum(lens), 256, device=dev)      # the videos' LFB rows, concatenated time-major
    feats = [f[None] for f in torch.split(bank, lens)]

    def step():           # all 40 videos in one ragged pass (CausalMambaModel.forward_videos)
        return model.forward_videos(bank, lens)

    def per_video():      # the callers' loop: one forward per video
        out = None
        for f in feats:
            out = model(f.transpose(2, 1))
        return out

    def check(out):
        assert out.shape == (sum(lens), 14) and torch.isfinite(out).all()
        last = per_video()
        torch.testing.assert_close(model.split_videos(out, lens)[-1], last, rtol=1e-4, atol=1e-4)
        with torch.no_grad():
            per_video()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            per_video()
            torch.cuda.synchronize()
        config["per_video_loop_frames_s"] = round(sum(lens) / (time.perf_counter() - t0), 1)

    config = {"workload": "tecno.py CausalMambaModel(f_maps 64, f_dim 256, 10 Mamba blocks: d_state 64, d_conv 4, "
                          "expand 2) over 40 full-length videos (T ~ U[1000, 6000]) per step, one ragged pass "
                          "(forward_videos: one launch per kernel for all videos)",
              "model": "CausalMambaModel(4,10,64,256,14,True)", "videos_per_step": 40}
    return step, sum(lens), config, check, (lambda: cpu_baseline_mamba(args.cpu_baseline_seconds))


def cpu_baseline_preproc(budget_s, H=480, W=854):
    from oracle import preproc as OP
    img = np.random.default_rng(0).integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        OP.frame_transform(img)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} frames {H}x{W} (numpy restatement of Pillow's resize + torch crop/normalise) in {dt:.1f} s"}


def workload_preproc(args, dev, rank, dtype):
    from svk.preproc import frame_transform
    H, W = 480, 854                                           # Cholec80 frame size (854x480 video)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    frames = torch.randint(0, 256, (args.batch, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(args.batch, 3, 224, 224, device=dev)

    def step():
        return frame_transform(frames, out=out)

    def check(o):
        assert o.shape == (args.batch, 3, 224, 224) and torch.isfinite(o).all()

    config = {"workload": "generate_evp_LFB.py eval transform on decoded frames: Resize((250, 250)) [Pillow bilinear, "
                          "bit-exact] -> CenterCrop(224) -> ToTensor -> Normalize, 480x854 uint8 RGB -> [B, 3, 224, 224] f32",
              "per_gpu_batch": args.batch}
    return step, args.batch, config, check, (lambda: cpu_baseline_preproc(min(args.cpu_baseline_seconds, 10.0)))


def cpu_baseline_augment(budget_s, H=480, W=854):
    """One training sample as the reference's DataLoader worker makes it (decoded frame + segmap through Pillow:
    Resize, RandomCrop, ColorJitter, flip, rotate, ToTensor, Normalize; the flow through cv2-style resize + the
    tensor crop / flip / rotation) with the drop-in synced classes, one host thread."""
    import random
    from PIL import Image
    from models import data_process as DP
    from oracle import preproc as OP
    rng = np.random.default_rng(0)
    img, seg = (rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8) for _ in range(2))
    flow = rng.normal(size=(H, W, 2)).astype(np.float32)
    crop, jit, flip, rot = DP.RandomCrop(224), DP.ColorJitter(0.1, 0.1, 0.1, 0.05), DP.RandomHorizontalFlip(), DP.RandomRotation(5)
    m, s = torch.tensor(DP.MEAN)[:, None, None], torch.tensor(DP.STD)[:, None, None]

    def pil(a):
        im = Image.fromarray(a).resize((250, 250), Image.BILINEAR)
        for t in (crop, jit, flip, rot):
            im = t(im)
        return torch.from_numpy(np.array(im)).permute(2, 0, 1).float().div(255).sub_(m).div_(s)

    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        pil(img)
        pil(seg)
        r = OP.cv2_resize_linear(flow, (250, 250))
        t = torch.from_numpy(np.ascontiguousarray(r.transpose(2, 0, 1)))
        rot(flip(crop(t)))
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} samples {H}x{W} (frame + segmap through Pillow, flow through the host tensor path; "
                      f"train_evp.py use_flip=1 transform, one worker thread) in {dt:.1f} s"}


def workload_augment(args, dev, rank, dtype):
    """train_evp.py's training transform (use_flip=1) on a B-sample batch of decoded 480x854 frames, RGB segmaps
    and RAFT flows resident in HBM (svk.augment.TrainAugment: synced parameter draws on the host, bit-exact
    Pillow arithmetic on the GPU); one step = one batch."""
    from svk.augment import TrainAugment
    H, W = 480, 854
    g = torch.Generator(device=dev)
    g.manual_seed(4321 + rank)
    frames = torch.randint(0, 256, (args.batch, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    segs = torch.randint(0, 256, (args.batch, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    flows = torch.randn(args.batch, H, W, 2, device=dev, generator=g)
    aug = TrainAugment(use_flip=1)

    def step():
        return aug(frames, segs, flows)[0]

    def check(o):
        assert o.shape == (args.batch, 3, 224, 224) and torch.isfinite(o).all()

    config = {"workload": "train_evp.py training transform (use_flip=1): Resize(250) -> RandomCrop(224) -> ColorJitter -> "
                          "flip -> RandomRotation(5) -> ToTensor -> Normalize on decoded 480x854 frames + RGB segmaps "
                          "(Pillow-exact), crop / flip / rotation on the RAFT flow; synced host draws per sample",
              "per_gpu_batch": args.batch}
    return step, args.batch, config, check, (lambda: cpu_baseline_augment(min(args.cpu_baseline_seconds, 10.0)))


def cpu_baseline_e2e(variant, budget_s, modules, inputs, chunk=32):
    """Config 5's chain restated on the oracle (torch CPU, fp32) on a bounded sample: ``chunk`` frames of
    the benched inputs through the SAME weights as the GPU modules.  The GPU chain runs once on the same
    chunk (outside the timed region) and the record carries the comparison (per-frame logits max |d|,
    phase argmax agreement): the one-off parity check of the benched configuration."""
    host = _cpu_threads()
    from oracle import mit_evp as M, mstcn as MS, trans_sv as TS
    seg, tc, tr = modules
    x, y, fl = (t[:chunk] for t in inputs)
    with torch.no_grad():
        f = seg(x, y, fl, return_features=True)[None]
        got = tr.original_forward(tc(f.transpose(2, 1))[-1], f).float().cpu()
    torch.cuda.synchronize()
    sd = {k: v.detach().float().cpu() for k, v in seg.state_dict().items()}
    sd_tc = {k: v.detach().cpu() for k, v in tc.state_dict().items()}
    sd_tr = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    xc, yc, fc = (t.float().cpu() for t in (x, y, fl))
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while time.perf_counter() - t0 < budget_s or n == 0:
            rf = M.forward(xc, yc, sd, variant, fc, return_features=True)[None]
            ro = MS.multi_stage_s(rf.transpose(2, 1), sd_tc, 2, 8, True)[-1]
            rp = TS.original_forward(ro, rf, sd_tr, 32)
            n += 1
    dt = time.perf_counter() - t0
    agree = float((got[:, 0, :7].argmax(-1) == rp[:, 0, :7].argmax(-1)).float().mean())
    return {"value": round(n * chunk / dt, 3), "unit": "frames/s", "cores": torch.get_num_threads(), "host_cpus": host,
            "kind": "port",
            "sample": f"{n} chains x {chunk} frames ({variant} + flow -> MS-TCN(2,8,32,2048) -> Transformer, fp32) "
                      f"in {dt:.1f} s",
            "check_vs_gpu": {"frames": chunk, "logits_max_abs_diff": float((got - rp).abs().max()),
                             "phase_argmax_agreement": agree}}


def workload_e2e(args, dev, rank, dtype):
    """BASELINE config 5 (trans_SV_output.py:276-291): MiT features -> MultiStageModel_S(2,8,32,2048,causal)
    -> Transformer(32, 2048, 14, 30).original_forward on B-frame chunks, the whole chain replayed as one HIP
    graph (--no-graph: eager)."""
    from models import mix_transformer_evp as mte, mstcn, adapter_transformer
    torch.manual_seed(0)
    seg = getattr(mte, args.variant)()
    seg.svk_dtype = dtype
    seg = seg.to(dev).eval()
    tc = mstcn.MultiStageModel_S(2, 8, 32, 2048, 14, True).to(dev).eval()
    tr = adapter_transformer.Transformer(32, 2048, 14, 30).to(dev).eval()
    for mod in (seg, tc, tr):
        for p in mod.parameters():
            p.requires_grad_(False)
    x, y, fl = synthetic_batch(args.batch, dev, seed=1234 + rank)

    def eager():
        f = seg(x, y, fl, return_features=True)[None]          # [1, T, 2048] LFB rows
        out = tc(f.transpose(2, 1))[-1]                          # [1, 14, T]
        return tr.original_forward(out, f)                       # [T, 1, 14]

    step = eager
    if not args.no_graph:
        with torch.no_grad():
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                eager()                                          # weight packs + allocator pool
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                static_out = eager()

        def step():
            g.replay()
            return static_out

        step.profile = eager

    def check(out):
        assert out.shape == (args.batch, 1, 14) and torch.isfinite(out).all()

    config = {"workload": f"trans_SV_output end-to-end: {args.variant}+flow features -> MS-TCN(2,8,32,2048,causal) "
                          f"-> Transformer(len_q 30) on {args.batch}-frame chunks",
              "model": f"{args.variant} + MultiStageModel_S(2,8,32,2048) + Transformer(32,2048,14,30)",
              "per_gpu_batch": args.batch, "hip_graph": not args.no_graph}
    return step, args.batch, config, check, (lambda: cpu_baseline_e2e(args.variant, args.cpu_baseline_seconds,
                                                                      (seg, tc, tr), (x, y, fl)))


def cpu_baseline_train(variant, budget_s, batch=8):
    """Oracle train step (torch CPU autograd, fp32, train mode, SGD) on a bounded sample."""
    host = _cpu_threads()
    from oracle import inputs as I, params as P, shapes as SH, train_evp as TR
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 0)
    x, y, fl = I.frames(batch, 1), I.segmaps(batch, 1), I.flow(batch, 1)
    lab = torch.randint(0, 7, (batch,), generator=torch.Generator().manual_seed(0))
    at = torch.rand(batch, 7, generator=torch.Generator().manual_seed(1))
    masks = TR.make_masks(batch, variant, seed=0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        _, _, grads, _ = TR.loss_and_grads(x, y, fl, lab, at, sd, variant, masks, dtype=torch.float32)
        TR.sgd_step({k: sd[k] for k in grads}, grads)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * batch / dt, 3), "unit": "frames/s", "cores": torch.get_num_threads(), "host_cpus": host, "kind": "port",
            "sample": f"{n} train steps x {batch} frames ({variant} + flow, fp32 autograd + SGD) in {dt:.1f} s"}


def workload_train(args, dev, rank, dtype):
    """train_evp.py stage-1 step (config 2 / 4): frozen backbone, trainable head + prompts + flow
    encoder + cross-attention, train mode, CE(sum) + SmoothL1(sum), SGD; DDP when world > 1."""
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    torch.manual_seed(0)
    model = getattr(mte, args.variant)().to(dev)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    tr = EVPTrainStep(model, dtype=dtype, seed=rank, process_group=dist.group.WORLD if world > 1 else None,
                      world_size=world, grad_comm=args.grad_comm)
    x, y, fl = synthetic_batch(args.batch, dev, seed=1234 + rank)
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    lab = torch.randint(0, 7, (args.batch,), generator=g, device=dev)
    at = torch.rand(args.batch, 7, generator=g, device=dev)

    if not args.no_graph:
        tr.step(x, y, fl, lab, at)                 # one eager iteration, then the whole step as one HIP graph
        tr.capture(x, y, fl, lab, at)

    def step():
        return tr.step(x, y, fl, lab, at)[0]

    def eager():
        return tr.train_iteration(x, y, fl, lab, at)[0]

    step.profile = eager

    def check(out):
        assert torch.isfinite(out).all()

    config = {"workload": f"train_evp.py stage-1 step: {args.variant} frozen backbone + trainable head/prompts/"
                          f"flow encoder/cross-attn ({tr.n_trainable} params), train mode, CE+SmoothL1 (sum), "
                          f"SGD(lr 5e-4, m 0.9, wd 1e-5)",
              "model": args.variant, "per_gpu_batch": args.batch, "hip_graph": not args.no_graph,
              "grad_allreduce_dtype": args.grad_comm}
    return step, args.batch, config, check, (lambda: cpu_baseline_train(args.variant, args.cpu_baseline_seconds))


def cpu_baseline_tecno_train(kind, budget_s, T=1500):
    """Oracle train step (fp32 CPU autograd through the restatement, dropout draws, the tecno loss,
    clip_grad_norm_ + AdamW) on one video of T frames, repeated within the budget."""
    host = _cpu_threads()
    from oracle import params as P, mstcn as MS, mamba as OM, inputs as I, shapes as SH
    if kind == "mstcn":
        sd = P.make_state_dict(SH.mstcn_shapes(4, 10, 64, 256, 14), 1)
    else:
        sd = OM.init_state_dict(OM.mamba_shapes(256, 64, 10, 14), 1)
    sd = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    opt = torch.optim.AdamW(list(sd.values()), lr=1e-4, weight_decay=1e-3)
    x = I.lfb(T, 256, 7).transpose(2, 1)
    g = torch.Generator().manual_seed(0)
    lab = torch.randint(0, 7, (T,), generator=g)
    ant = torch.rand(T, 7, generator=g)
    cw = torch.ones(7)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        if kind == "mstcn":
            masks = (torch.rand(4, 10, T, 64, generator=g) < 0.5).float() * 2
            y = MS.multi_stage_s(x, sd, 4, 10, True, masks=masks)
        else:
            masks = (torch.rand(10, T, 64, generator=g) < 0.9).float() / 0.9
            y = OM.causal_mamba(x, sd, 10, dtype=torch.float32, masks=masks)
        clc, antl = MS.tecno_loss(y, lab, ant, cw)
        opt.zero_grad()
        (clc + antl).backward()
        torch.nn.utils.clip_grad_norm_(list(sd.values()), 1.0)
        opt.step()
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * T / dt, 2), "unit": "frames/s", "cores": torch.get_num_threads(), "host_cpus": host, "kind": "port",
            "sample": f"{n} optimizer steps on one {T}-frame video ({kind}, fp32 autograd through the oracle "
                      f"restatement + AdamW) in {dt:.1f} s"}


def workload_tecno_train(args, dev, rank, dtype):
    """tecno.py:192-259 training epoch: one optimizer step per video over 40 full-length videos
    (T ~ U[1000, 6000] LFB rows, f_dim 256), weighted CE + SmoothL1 over all stages, clip 1.0, AdamW —
    every step one replay of the HIP graph captured for that video length."""
    from models import mstcn
    from svk.temporal import TemporalTrainStep
    torch.manual_seed(0)
    kind = args.temporal
    lens = video_lengths(40, seed=rank)
    g = torch.Generator(device=dev).manual_seed(99 + rank)
    feats = [torch.randn(T, 256, device=dev, generator=g) for T in lens]
    labels = [torch.randint(0, 7, (T,), device=dev, generator=g) for T in lens]
    ants = [torch.rand(T, 7, device=dev, generator=g) * 5 for T in lens]
    cw = [1.6411019141231247, 0.19090963801041133, 1.0, 0.2502662616859295, 1.9176363911137977,
          0.9840248158200853, 2.174635818337618]                               # tecno.py:124-130

    def build(k):
        if k == "mstcn":
            return mstcn.MultiStageModel_S(4, 10, 64, 256, 14, True).to(dev)
        return mstcn.CausalMambaModel(4, 10, 64, 256, 14, True).to(dev)

    model = build(kind)
    st = TemporalTrainStep(model, class_weights=cw, graphs=not args.no_graph, seed=rank)

    def step():
        out = None
        for x, lab, ant in zip(feats, labels, ants):
            out = st(x, lab, ant)
        return out

    eager_st = TemporalTrainStep(model, class_weights=cw, graphs=False, seed=rank)

    def eager():
        out = None
        for x, lab, ant in zip(feats, labels, ants):
            out = eager_st(x, lab, ant)
        return out

    step.profile = eager

    def check(out):
        assert torch.isfinite(out).all()

    name = ("MultiStageModel_S(4,10,64,256,14,True)" if kind == "mstcn" else
            "CausalMambaModel(4,10,64,256,14,True)")
    config = {"workload": f"tecno.py training epoch: {name}, one optimizer step per video over 40 full-length "
                          "videos (T ~ U[1000, 6000]), train-mode dropout, weighted CE + SmoothL1 (all stages), "
                          "clip_grad_norm_(1.0), AdamW(lr 1e-4, wd 1e-3)",
              "model": name, "videos_per_step": 40, "hip_graph": not args.no_graph}
    return step, sum(lens), config, check, (lambda: cpu_baseline_tecno_train(kind, args.cpu_baseline_seconds))


WORKLOADS = {"extract": workload_extract, "lfb": workload_lfb, "augment": workload_augment, "mstcn": workload_mstcn, "mamba": workload_mamba, "preproc": workload_preproc, "e2e": workload_e2e, "train": workload_train,
             "tecno_train": workload_tecno_train}


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def count_visible_gpus(topology=None, env=None):
    """GPUs this process may use, counted WITHOUT any HIP call (so the launcher parent never
    initialises the runtime before it spawns the ranks): the KFD topology's GPU nodes (a node with
    SIMDs), narrowed by ROCR_VISIBLE_DEVICES and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES the
    way the ROCm runtime applies them (the HIP list indexes into what ROCR left visible)."""
    env = os.environ if env is None else env
    topology = KFD_TOPOLOGY if topology is None else topology
    n = 0
    try:
        for node in os.listdir(topology):
            try:
                with open(os.path.join(topology, node, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = env.get(var)
        if val is None:
            continue
        ids = [t for t in val.split(",") if t.strip() != ""]
        n = min(n, len(ids)) if not any(t.strip().startswith("-") for t in ids) else 0
    return n


def launch_ranks(args):
    """``--gpus N`` without a torchrun environment: start N ranks under torch.distributed.run (one
    process per GPU, rendezvous on 127.0.0.1) as a CHILD process and return its exit code.  The GPU
    count comes from the KFD topology (count_visible_gpus), so the parent makes no HIP call before the
    spawn.  Mismatches fail loudly instead of silently measuring one rank."""
    world_env = os.environ.get("WORLD_SIZE")
    # the "plumbing" workload (launcher test, gloo on CPU) runs without GPUs
    visible = args.gpus if args.workload == "plumbing" else count_visible_gpus()
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
        if int(os.environ.get("LOCAL_WORLD_SIZE", world_env)) > visible:
            sys.exit(f"bench.py: {world_env} ranks on this node but only {visible} visible GPU(s)")
        return None
    if args.gpus > visible:
        sys.exit(f"bench.py: --gpus {args.gpus} but only {visible} visible GPU(s)")
    if args.gpus <= 1:
        return None
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def plumbing(world, rank, local):
    """Launcher self-test (no GPU): every rank reports (rank, local rank, world) over gloo and rank 0
    prints them with the timing barrier's max-over-ranks reduction exercised on CPU tensors."""
    if world > 1:
        dist.init_process_group("gloo")
    me = torch.tensor([rank, local, world], dtype=torch.int64)
    got = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(got, me)
        dist.barrier()
    else:
        got = [me]
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"workload": "plumbing", "n_gpus": world, "ranks": [g.tolist() for g in got],
                          "max_over_ranks": t.item()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="extract", choices=sorted(WORKLOADS) + ["plumbing"])
    ap.add_argument("--batch", type=int, default=None, help="frames per GPU per step (256; train: 88)")
    ap.add_argument("--variant", default="mit_b2_evp")
    ap.add_argument("--dtype", default=None, choices=sorted(TORCH_DT),
                    help="compute dtype (extract / e2e default fp16 = the reference's autocast precision; "
                         "train default bf16 = BASELINE config 2)")
    ap.add_argument("--other-dtypes", default=None,
                    help="comma list of extra dtypes timed on the same inputs and reported as other_dtypes "
                         "(extract default: bf16,fp32; 'none' to skip)")
    ap.add_argument("--no-flow", action="store_true")
    ap.add_argument("--grad-comm", default="f32", choices=["f32", "bf16"],
                    help="train with N > 1: dtype of the gradient all-reduce (bf16 = half the bytes per link)")
    ap.add_argument("--temporal", default="mstcn", choices=["mstcn", "mamba"],
                    help="tecno_train: the temporal model (BASELINE config 3 names the MS-TCN; tecno.py:153 "
                         "trains the CausalMambaModel)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-workloads", action="store_true",
                    help="extract at N = 1: skip the train / config-5 legs reported under other_workloads")
    ap.add_argument("--dump-gemm", default=None, help="write per-shape GEMM timings to this file (rank 0)")
    ap.add_argument("--no-graph", action="store_true", help="extract / train: launch kernels eagerly instead of "
                                                           "replaying the step as a HIP graph")
    args = ap.parse_args(argv)
    if args.batch is None:
        args.batch = 88 if args.workload == "train" else 256      # train_evp.py:28 / extraction chunk
    if args.dtype is None:
        args.dtype = "bf16" if args.workload == "train" else "fp16"
    if args.other_dtypes is None:
        args.other_dtypes = "bf16,fp32" if args.workload == "extract" else "none"
    return args


def timed(step, steps, world):
    """Barrier + synchronize on both sides of exactly ``steps`` steps; max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return out, float(dt.item())


def operand_fetch(name, shapes, prof_steps, ms):
    """The dominant persistent GEMM's on-chip operand traffic: every (BM x BN) tile DMAs its A rows and W rows
    over the whole (64-padded) K into LDS, i.e. tiles x (BM + BN) x K x 2 bytes per launch — L2 / Infinity Cache
    -> LDS, far above the algorithmic HBM bytes — priced against the measured L2-served LDS-DMA ceiling."""
    m = re.match(r"gemm_pk<[^,]+, PkCfg<(\d+), (\d+)", name)
    if not m:
        return None
    bm, bn = int(m.group(1)), int(m.group(2))
    nbytes, n = 0.0, 0
    for (kname, shape), (_, _, _, cnt) in shapes.items():
        if kname != name:
            continue
        try:
            sh = ast.literal_eval(shape)
            M, N, K = int(sh[0]), int(sh[1]), int(sh[2])
        except (ValueError, SyntaxError, TypeError, IndexError):
            return None
        tiles = -(-M // bm) * -(-N // bn)
        nbytes += cnt * tiles * (bm + bn) * (-(-K // 64) * 64) * 2
        n += cnt
    if not n:
        return None
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"bytes_per_launch": round(nbytes / n), "achieved_gbs": round(gbs, 1), "ceiling_gbs": L2_LDS_PEAK_GBS,
            "frac": round(gbs / L2_LDS_PEAK_GBS, 4),
            "note": "tiles x (BM + BN) x K x 2 B per launch over the same HIP-event launch time as roofline.achieved; "
                    "ceiling = L2-served LDS-DMA 73 GB/s per CU (MI355X_MICROARCH.md)"}


def roofline_of(records, prof_steps, elapsed, steps, workload, dtype_name, value, world, dump_gemm=None,
                variant="mit_b2_evp", prof_elapsed=None):
    """Dominant kernel (the GEMM / conv instantiation with the most HIP-event device time over the profiled
    eager iterations) priced against its roof: algorithmic FLOP or bytes per launch / average launch time."""
    per, shapes = {}, {}
    for name, flops, nbytes, s, e, shape in records:
        ms = s.elapsed_time(e)
        for key, d in ((name, per), ((name, str(shape)), shapes)):
            tot = d.setdefault(key, [0.0, 0.0, 0.0, 0])
            tot[0] += ms
            tot[1] += flops
            tot[2] += nbytes
            tot[3] += 1
    if dump_gemm:
        with open(dump_gemm, "w") as f:
            for (name, shape), (ms, fl, nb, n) in sorted(shapes.items(), key=lambda kv: -kv[1][0]):
                f.write(f"{ms / prof_steps:8.3f} ms/step n={n // prof_steps:3d} {fl / ms / 1e9:8.1f} TF/s "
                        f"{nb / ms / 1e6:8.1f} GB/s  {shape:28s} {name}\n")
    gemm_ms = sum(v[0] for v in per.values())
    # the dominant kernel (every GEMM of the step is a hand-written svk kernel: no library backend since round 5)
    name, (ms, flops, nbytes, n) = max(per.items(), key=lambda kv: kv[1][0])
    peak = PEAK_TFLOPS[dtype_name]
    # bound by arithmetic intensity vs the machine balance (peak FLOP/s / 8 TB/s): tall-skinny
    # token GEMMs (K or N <= 128) are HBM-bound, the head / 4096-wide GEMMs MFMA-bound
    intensity = flops / max(nbytes, 1)
    # the selective scan is a VALU recurrence (no MFMA work at all): priced against HBM
    hbm_bound = intensity < peak * 1e12 / (HBM_PEAK_GBS * 1e9) or name.startswith(("mamba_scan", "frame_preproc"))
    tflops = flops / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    roofline = {"bound": "hbm" if hbm_bound else "mfma", "kernel": name,
                "achieved": round(gbs if hbm_bound else tflops, 2), "peak": HBM_PEAK_GBS if hbm_bound else peak,
                "unit": "GB/s" if hbm_bound else "TFLOP/s",
                "frac": round(gbs / HBM_PEAK_GBS if hbm_bound else tflops / peak, 4), "traffic": None,
                "launches_per_step": n // prof_steps, "avg_launch_us": round(ms * 1e3 / n, 2),
                "algorithmic_flop_per_launch": flops / n, "algorithmic_bytes_per_launch": nbytes / n,
                "arith_intensity_flop_per_byte": round(intensity, 1),
                "kernel_tflops": round(tflops, 2), "kernel_gbs": round(gbs, 1),
                "all_gemm_tflops": round(sum(v[1] for v in per.values()) / (gemm_ms * 1e-3) / 1e12, 2),
                # GEMM device time of the profiled EAGER iterations over those iterations' own wall time (round 6:
                # dividing by the graph-replayed step made it exceed 1)
                "gemm_share_of_step": round(gemm_ms / (prof_elapsed * 1e3) if prof_elapsed
                                            else gemm_ms / prof_steps / (elapsed * 1e3 / steps), 3)}
    if workload in ("extract", "e2e") and variant in EXTRACT_GFLOP:
        # whole-step MFMA utilisation: measured frames/s x algorithmic work / dense peak
        gf = EXTRACT_GFLOP[variant]
        roofline["step_mfma_util"] = round(value / world * gf * 1e9 / (peak * 1e12), 4)
        roofline["step_gflop_per_frame"] = round(gf, 2)
    elif workload == "train":
        roofline["step_mfma_util"] = round(value / world * TRAIN_GFLOP_PER_FRAME * 1e9 / (peak * 1e12), 4)
        roofline["step_gflop_per_frame"] = TRAIN_GFLOP_PER_FRAME
    fetch = operand_fetch(name, shapes, prof_steps, ms)
    if fetch is not None:
        roofline["operand_fetch"] = fetch
    busy = pmc_mfma_busy(workload, dtype_name, variant)
    if busy is not None:
        roofline["mfma_busy_counters"] = busy
    traffic, src = pmc_traffic(workload, name)
    if traffic is not None:
        roofline["traffic"] = traffic
        roofline["traffic_source"] = src + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, per launch)"
    return roofline


def run_leg(args, dev, rank, world, dtype):
    """Build the workload, W warmup steps, EXACTLY K timed steps (barrier + synchronize both sides, max over
    ranks), then the profiled eager iterations for the roofline and the other dtypes."""
    from svk import ops
    step, units, config, check, cpu_fn = WORKLOADS[args.workload](args, dev, rank, dtype)
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        out, elapsed = timed(step, args.steps, world)      # the measured region: no instrumentation
        check(out)
        # roofline: HIP events around every GEMM / conv launch on separate (untimed) iterations of the
        # same step (graph-replayed steps make no host calls: their eager twin, identical launches)
        records = []
        ops.set_profiler(records)
        prof_steps = max(1, min(args.steps, 5))
        torch.cuda.synchronize()
        tp0 = time.perf_counter()
        for _ in range(prof_steps):
            (step.profile if hasattr(step, "profile") else step)()
        torch.cuda.synchronize()
        prof_elapsed = time.perf_counter() - tp0
        ops.set_profiler(None)
        # the same inputs at the other compute dtypes (extraction): fp32 is the precision of the
        # reference's generate_evp_LFB.py, bf16 the narrower 16-bit format
        other = {}
        if hasattr(step, "set_dtype") and args.other_dtypes != "none":
            for name in [d for d in args.other_dtypes.split(",") if d and d != args.dtype]:
                step.set_dtype(TORCH_DT[name])
                for _ in range(2):
                    step()
                n2 = max(2, args.steps // 2)
                o2, el2 = timed(step, n2, world)
                check(o2)
                other[name] = {"value": round(world * units * n2 / el2, 2), "ms_per_step": round(el2 * 1e3 / n2, 3),
                               "steps": n2}
                # this dtype's own dominant-kernel roofline (fp32 = generate_evp_LFB.py's precision,
                # priced against the 157 TF f32 MFMA peak), from profiled eager iterations of the same step
                rec2 = []
                ops.set_profiler(rec2)
                torch.cuda.synchronize()
                tp0 = time.perf_counter()
                for _ in range(prof_steps):
                    (step.profile if hasattr(step, "profile") else step)()
                torch.cuda.synchronize()
                pe2 = time.perf_counter() - tp0
                ops.set_profiler(None)
                other[name]["roofline"] = roofline_of(rec2, prof_steps, el2, n2, args.workload, name,
                                                      world * units * n2 / el2, world, None, args.variant, pe2)
            step.set_dtype(dtype)
    value = world * units * args.steps / elapsed
    f32_only = args.workload in ("mstcn", "mamba", "preproc", "tecno_train", "augment")
    dtype_name = "fp32" if f32_only else args.dtype
    roofline = roofline_of(records, prof_steps, elapsed, args.steps, args.workload, dtype_name, value, world,
                           args.dump_gemm if rank == 0 else None, args.variant, prof_elapsed)
    leg = {"value": round(value, 2), "unit": "frames/s", "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "dtype": dtype_name, "config": config,
           "roofline": roofline}
    if other:
        leg["other_dtypes"] = other
    return leg, cpu_fn


def other_workloads(args, dev, rank, world):
    """BASELINE.json's metric has two halves and config 5 a chain: on the headline run (N = 1) the same box
    also times the train_evp step (config 2: B = 88, bf16, graph-replayed) and the config-5 chain (fp16,
    256-frame chunks, graph-replayed), each with its own dominant-kernel roofline and CPU baseline (the
    chain's carries the one-off GPU-vs-oracle check of the benched configuration), and the callers' own
    extraction model, mit_b3_evp (generate_evp_LFB.py:412; 18 stage-3 blocks), at fp16 and fp32 on the same
    B = 256 synthetic batch, each dtype with its own roofline."""
    legs = {}
    b3 = "mit_b3_evp"
    # 30 timed / 10 warm-up steps each (round 6: at 10 / 3 two back-to-back default runs on one box read the train leg
    # at 5 758 and 6 467 frames/s)
    for name, argv in (("train", ["--workload", "train", "--steps", "30", "--warmup", "10", "--variant", args.variant]),
                       ("e2e_config5", ["--workload", "e2e", "--steps", "30", "--warmup", "10",
                                        "--variant", args.variant]),
                       ("extract_" + b3, ["--workload", "extract", "--steps", "30", "--warmup", "10", "--variant", b3,
                                          "--other-dtypes", "fp32"])):
        if name.startswith("extract_") and args.variant == b3:
            continue                                 # the headline already is b3
        a = parse_args(argv + ["--cpu-baseline-seconds", str(min(args.cpu_baseline_seconds, 10.0))])
        try:
            leg, cpu_fn = run_leg(a, dev, rank, world, TORCH_DT[a.dtype])
            if not args.no_cpu_baseline:
                leg["cpu_baseline"] = cpu_fn()
            if name == "train":
                leg["config"]["steps_per_s"] = round(a.steps / (leg["ms_per_step"] * a.steps * 1e-3), 3)
            legs[name] = leg
        except Exception as e:                       # a failing extra leg must not cost the headline line
            legs[name] = {"error": f"{type(e).__name__}: {e}"[:400]}
        torch.cuda.empty_cache()
    return legs


def main():
    args = parse_args()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.workload == "plumbing":
        return plumbing(world, rank, local)
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import svk

    dtype = TORCH_DT[args.dtype]
    leg, cpu_fn = run_leg(args, dev, rank, world, dtype)
    extra = None
    if args.workload == "extract" and world == 1 and not args.no_other_workloads:
        extra = other_workloads(args, dev, rank, world)

    if rank == 0:
        cpu = cpu_fn() if (world == 1 and not args.no_cpu_baseline) else None
        par = (f"dp{world} (DDP: RCCL all-reduce of the f32 gradient in two buckets, the head bucket overlapped "
               f"with the backbone backward)" if args.workload == "train"
               else f"dp{world} (shards of independent units, no collective)")
        config = leg["config"]
        config.update({"global_units_per_step": round(leg["value"] * leg["ms_per_step"] * 1e-3), "parallelism": par})
        if args.workload == "train":
            config["steps_per_s"] = round(1e3 / leg["ms_per_step"], 3)
        line = {"metric": METRIC if args.workload == "extract" else f"frames/s ({args.workload})",
                **({"metric": "generate_evp_LFB frames/s from pinned host memory (PCIe-inclusive; not the headline)"}
                   if args.workload == "lfb" else {}),
                **({"metric": "train_evp frames/s (step/s x 88 frames/GPU)"} if args.workload == "train" else {}),
                "value": leg["value"], "unit": "frames/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": leg["ms_per_step"],
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": leg["dtype"], "data": DATA, "config": config,
                "roofline": leg["roofline"], "cpu_baseline": cpu, "svk": svk.version()}
        if "other_dtypes" in leg:
            line["other_dtypes"] = leg["other_dtypes"]
        if extra:
            line["other_workloads"] = extra
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
