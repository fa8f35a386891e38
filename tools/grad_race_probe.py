"""Run-to-run determinism probe for the f32 train step (VERDICT r04 "next" #1).

The same f32 EVPTrainStep.forward_backward is repeated on identical inputs; every svk.ops call's
outputs (returned tensors and the in-place gradient outputs) of iteration 0 are kept and every later
iteration is compared call by call.  f32 atomics make a few calls non-bit-exact (~1e-7 relative); a call
whose output moves by more than ``--tol`` relative is reported with its index, op name and shapes, which
names the first kernel whose result is not reproducible.  ``--load`` runs an MFMA-heavy bf16 GEMM loop
on a second stream during the steps (other waves issuing MFMAs on the same SIMDs).

    python tools/grad_race_probe.py --variant mit_b3_evp --iters 40 [--load]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"), REPO]

from svk import ops  # noqa: E402

OUT_ARGS = {"gemm_wgrad": ("dw", "db"), "conv2d_wgrad": ("dw", "db"), "bn_bwd": ("dgamma", "dbeta"),
            "layernorm_bwd": ("dgamma", "dbeta"), "resize_bilinear_bwd": ("dx",), "colstats": ("s", "sq"),
            "unpatchify": ("out",), "attention_bwd": ("dk", "dv", "dq")}


class Recorder:
    def __init__(self):
        self.calls = []          # per iteration: list of (name, [tensors])
        self.ref = None
        self.cur = None
        self.cur_in = None
        self.cur_ptr = None

    def wrap(self, name, fn):
        import inspect
        sig = inspect.signature(fn)

        def w(*a, **k):
            if self.cur is not None:
                ins = [(i, t) for i, t in enumerate(list(a) + list(k.values())) if isinstance(t, torch.Tensor)]
                self.cur_in.append((name, [(i, t.data_ptr(), t.numel() * t.element_size(), tuple(t.shape),
                                            t.detach().float().clone()) for i, t in ins]))
            r = fn(*a, **k)
            if self.cur is not None:
                outs = []
                rs = r if isinstance(r, (tuple, list)) else (r,)
                outs += [t for t in rs if isinstance(t, torch.Tensor)]
                if name in OUT_ARGS:
                    ba = sig.bind_partial(*a, **k)
                    for an in OUT_ARGS[name]:
                        t = ba.arguments.get(an)
                        if isinstance(t, torch.Tensor):
                            outs.append(t)
                shapes = [tuple(t.shape) for t in outs]
                self.cur.append((name, shapes, [t.detach().float().clone() for t in outs]))
                self.cur_ptr.append([(t.data_ptr(), t.numel() * t.element_size()) for t in outs])
            return r
        return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="mit_b3_evp")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--B", type=int, default=3)
    ap.add_argument("--tol", type=float, default=1e-5)
    ap.add_argument("--load", action="store_true")
    ap.add_argument("--no-record", action="store_true", help="compare only the final gradients")
    args = ap.parse_args()
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = getattr(mte, args.variant)().to(dev)
    tr = EVPTrainStep(m, dtype=torch.float32, drop=True, seed=5)
    B = args.B
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, 1, 3, 224, 224, generator=g).to(dev)
    y = torch.randn(B, 1, 3, 224, 224, generator=g).to(dev)
    fl = (2 * torch.randn(B, 1, 2, 224, 224, generator=g)).to(dev)
    lab = torch.randint(0, 7, (B,), generator=g).to(dev)
    at = torch.rand(B, 7, generator=g).to(dev)
    rec = Recorder()
    if not args.no_record:
        for name in list(OUT_ARGS) + ["gemm", "layernorm", "attention", "bn_apply", "mean_rows", "mul_f32",
                                      "bcast_rows", "cast", "resize_bilinear", "dwconv3x3", "conv2d_nhwc",
                                      "conv2d_dgrad", "conv2d_dgrad_col2im", "phase_loss", "gemm_unpatchify",
                                      "conv2d_ln_nhwc", "act_bwd", "gauss5x5_reflect", "nchw_to_nhwc"]:
            if hasattr(ops, name):
                setattr(ops, name, rec.wrap(name, getattr(ops, name)))
    stop = [False]
    if args.load:
        ls = torch.cuda.Stream(device=dev)
        a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)

        def spin():
            with torch.cuda.stream(ls):
                for _ in range(40):
                    a @ a
    grads0 = None
    worst = {}
    for it in range(args.iters):
        if args.load:
            spin()
        rec.cur = [] if not args.no_record else None
        rec.cur_in, rec.cur_ptr = [], []
        tr.forward_backward(x, y, fl, lab, at)
        gsnap = tr.grad.detach().clone()
        torch.cuda.synchronize()
        if it == 0:
            grads0 = gsnap
            rec.ref = rec.cur
            rec.ref_in = rec.cur_in
            continue
        gd = {n: ((gsnap[tr.off[n]:tr.off[n] + p.numel()] - grads0[tr.off[n]:tr.off[n] + p.numel()]).abs().max()
                  / grads0[tr.off[n]:tr.off[n] + p.numel()].abs().max().clamp_min(1e-30)).item()
              for n, p in tr.params.items()}
        bad = sorted(((v, n) for n, v in gd.items() if v > args.tol), reverse=True)
        first = None
        if rec.cur is not None:
            assert len(rec.cur) == len(rec.ref), (len(rec.cur), len(rec.ref))
            for ci, ((nm, sh, ts), (_, _, rs)) in enumerate(zip(rec.cur, rec.ref)):
                for j, (t, r) in enumerate(zip(ts, rs)):
                    d = ((t - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
                    key = (ci, nm, str(sh), j)
                    worst[key] = max(worst.get(key, 0.0), d)
                    if d > args.tol and first is None:
                        first = (ci, nm, sh, j, d)
        first_in = None
        if first is not None:          # were the first differing call's INPUTS already different?
            ci = first[0]
            nm, ins = rec.cur_in[ci]
            for (i, ptr, nb, sh, t), (_, _, _, _, r) in zip(ins, rec.ref_in[ci][1]):
                d = (t - r).abs()
                print(f"  call #{ci} {nm} arg{i} {sh}: max|in - ref in| {d.max().item():.3e} "
                      f"(ref max {r.abs().max().item():.3e})", flush=True)
                if first_in is None and d.max().item() > args.tol * r.abs().max().clamp_min(1e-30).item():
                    first_in = (ci, nm, i, ptr, nb, sh, d)
        if first is not None and os.environ.get("PROBE_DUMP"):
            ci = first[0]
            torch.save({"name": first[1], "it": it,
                        "in": [t.cpu() for (_, _, _, _, t) in rec.cur_in[ci][1]],
                        "ref_in": [t.cpu() for (_, _, _, _, t) in rec.ref_in[ci][1]],
                        "out": [t.cpu() for t in rec.cur[ci][2]], "ref_out": [t.cpu() for t in rec.ref[ci][2]]},
                       os.environ["PROBE_DUMP"])
        if first_in is not None and (first is None or first_in[0] <= first[0]):
            ci, nm, i, ptr, nb, sh, d = first_in
            badm = d.flatten() > 0
            idx = badm.nonzero().flatten()
            esz = nb // max(1, d.numel())
            lo, hi = ptr + idx.min().item() * esz, ptr + (idx.max().item() + 1) * esz
            print(f"  INPUT corrupted before call #{ci} {nm} arg{i} {sh} ptr {ptr:#x}+{nb}: {idx.numel()} elements, "
                  f"bytes [{lo:#x}, {hi:#x})", flush=True)
            # earlier calls (this iteration) whose outputs overlap or border the corrupted range
            for cj in range(ci):
                for k2, (p2, n2) in enumerate(rec.cur_ptr[cj]):
                    if p2 < hi + 4096 and p2 + n2 > lo - 4096:
                        print(f"    call #{cj} {rec.cur[cj][0]} out{k2} {rec.cur[cj][1][k2] if k2 < len(rec.cur[cj][1]) else ''} "
                              f"[{p2:#x}, {p2 + n2:#x})", flush=True)
        print(f"iter {it}: {len(bad)} params over {args.tol:g}"
              + (f" (worst {bad[0][1]} {bad[0][0]:.3e})" if bad else "")
              + (f"; first differing call #{first[0]} {first[1]} {first[2]} out{first[3]} rel {first[4]:.3e}"
                 if first else ""), flush=True)
    if worst:
        print("calls with the largest run-to-run relative deviation:")
        for (ci, nm, sh, j), d in sorted(worst.items(), key=lambda kv: -kv[1])[:25]:
            print(f"  #{ci:4d} {nm:22s} out{j} {sh:40s} {d:.3e}")
    stop[0] = True


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"done in {time.time() - t0:.1f}s")
