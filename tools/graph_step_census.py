"""Kernel census of the graph-replayed extraction step (launches per replayed step, glue
kernels inside the graph).  Two modes:
  run:     python tools/graph_step_census.py run [--batch 256] [--replays 6]
           builds MiT-b2 + flow at fp16, captures the step (svk.graphs.GraphedForward), synchronises, then
           replays it --replays times and nothing else (run it under rocprofv3 --kernel-trace).
  analyse: python tools/graph_step_census.py analyse KERNEL_TRACE_CSV [--replays 6]
           takes the dispatches after the last host synchronisation gap, splits them into replays at the
           step's last kernel (mean_rows), prints launches per step, the kernels that are not svk's, and
           the sum of in-step gaps."""
import argparse
import collections
import csv
import os
import sys


def run(args):
    import torch
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "deep-learning-for-surgical-video-analysis_amd"), repo]
    from bench import synthetic_batch
    from models import mix_transformer_evp as mte
    from svk.graphs import GraphedForward
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = mte.mit_b2_evp()
    m.svk_dtype = torch.float16
    m = m.to(dev).eval()
    for p in m.parameters():
        p.requires_grad_(False)
    x, y, fl = synthetic_batch(args.batch, dev, 1234)
    with torch.no_grad():
        g = GraphedForward(m, x, y, fl, return_features=True)
        for _ in range(3):
            g()
        torch.cuda.synchronize()
        import time
        time.sleep(0.05)                       # a host gap the analyser uses as the boundary
        for _ in range(args.replays):
            g()
        torch.cuda.synchronize()
    print("replays done", flush=True)


def analyse(args):
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # last gap > 20 ms = the sleep before the measured replays
    cut = 0
    for i in range(1, len(rows)):
        if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 20_000_000:
            cut = i
    tail = rows[cut:]
    steps, cur = [], []
    for r in tail:
        cur.append(r)
        if "mean_rows" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    print(f"{len(steps)} replayed steps after the host gap ({len(tail)} dispatches)")
    for k, st in enumerate(steps):
        s0, e1 = int(st[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in st)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st)
        foreign = collections.Counter(r["Kernel_Name"][:90] for r in st if "svk" not in r["Kernel_Name"])
        print(f"step {k}: {len(st)} launches, span {(e1 - s0) / 1e6:.3f} ms, sum of kernel times {busy / 1e6:.3f} ms, "
              f"non-svk: {dict(foreign) if foreign else 'none'}")
    if steps:   # critical path: per queue, the union of its kernels' intervals vs the step's span
        use = steps[1:] or steps
        tot = collections.defaultdict(float)
        span_sum = 0.0
        for st in use:
            s0, e1 = int(st[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in st)
            span_sum += e1 - s0
            byq = collections.defaultdict(list)
            for r in st:
                byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            allq = [iv for v in byq.values() for iv in v]
            for q, ivs in list(byq.items()) + [("any", allq)]:
                ivs.sort()
                busy, cs, ce = 0, None, None
                for a, b in ivs:
                    if ce is None or a > ce:
                        busy += 0 if ce is None else ce - cs
                        cs, ce = a, b
                    else:
                        ce = max(ce, b)
                busy += ce - cs
                tot[q] += busy
        n = len(use)
        span = span_sum / n / 1e3
        main_q = max((q for q in tot if q != "any"), key=lambda q: tot[q])   # the queue carrying most of the step
        print(f"critical path: span {span:.1f} us per step; main queue q{main_q} busy {tot[main_q] / n / 1e3:.1f} us "
              f"({tot[main_q] / span_sum:.3f} of the span, idle {(span_sum - tot[main_q]) / n / 1e3:.1f} us); "
              + "; ".join(f"q{q} busy {v / n / 1e3:.1f} us" for q, v in sorted(tot.items()) if q not in (main_q, "any"))
              + f"; any queue busy {tot['any'] / n / 1e3:.1f} us ({tot['any'] / span_sum:.3f} of the span: the GPU idles "
              f"{(span_sum - tot['any']) / n / 1e3:.1f} us per step between kernels)")
    if args.by_kernel and steps:   # per-kernel time per replayed step (all replays but the first)
        use = steps[1:] or steps
        agg, cnt = collections.Counter(), collections.Counter()
        for st in use:
            for r in st:
                agg[r["Kernel_Name"][:100]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                cnt[r["Kernel_Name"][:100]] += 1
        tot = sum(agg.values()) / len(use) / 1e3
        print(f"per replayed step: {sum(cnt.values()) / len(use):.1f} launches, kernel time {tot:.1f} us")
        for k, v in agg.most_common():
            print(f"{v / len(use) / 1e3:9.1f} us {cnt[k] / len(use):6.1f}x  {k}")
    if args.seq and steps:   # the last step's launch sequence: start offset, duration (us), queue, kernel
        st = steps[-1]
        s0 = int(st[0]["Start_Timestamp"])
        with open(args.seq, "w") as f:
            for r in st:
                t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                f.write(f"{(t0 - s0) / 1e3:8.1f} {(t1 - t0) / 1e3:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:90]}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "analyse"])
    ap.add_argument("trace", nargs="?")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--replays", type=int, default=6)
    ap.add_argument("--seq", default="", help="analyse: write the last step's launch sequence here")
    ap.add_argument("--by-kernel", action="store_true", help="analyse: per-kernel time per replayed step")
    args = ap.parse_args()
    (run if args.mode == "run" else analyse)(args)


if __name__ == "__main__":
    main()
