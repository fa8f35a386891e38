"""Attention backward (bf16, the train step's shapes at B = 88) per kernel: the transposed-score dQ kernel
(SVK_ATTN_BWD_T=1) vs the round-5 one (=0), interleaved passes, median.  Only the svk_attention_bwd call is timed
(dQ kernel + two batched dK / dV reductions + the f32 -> bf16 store).  Usage: python tools/attn_bwd_bench.py [--only I]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402

SHAPES = [(3136, 49, 1), (784, 49, 2), (196, 49, 5), (49, 49, 8), (196, 196, 8), (196, 196, 5)]   # (Nq, Nk, heads), hd 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", type=int, default=-1)
    ap.add_argument("--variants", default="1,0")
    args = ap.parse_args()
    dev, dt, B, hd = torch.device("cuda:0"), torch.bfloat16, 88, 64
    shapes = SHAPES if args.only < 0 else [SHAPES[args.only]]
    for Nq, Nk, heads in shapes:
        C = heads * hd
        g = torch.Generator(device=dev).manual_seed(0)
        q, k, v, do = (torch.randn(B, n, C, device=dev, generator=g).to(dt) for n in (Nq, Nk, Nk, Nq))
        o = ops.attention(q, k, v, heads, hd ** -0.5)
        dkv = torch.empty(B, Nk, 2 * C, device=dev, dtype=dt)
        dq = torch.empty_like(q)
        t = {vv: [] for vv in args.variants.split(",")}

        def run(vv):
            os.environ["SVK_ATTN_BWD_T"] = vv
            ops.attention_bwd(q, k, v, o, do, heads, hd ** -0.5, dkv[:, :, :C], dkv[:, :, C:], dq)
        for _ in range(args.rounds):
            for vv in t:
                t[vv].append(timeit(lambda: run(vv), args.reps))
        print(f"B={B} Nq={Nq} Nk={Nk} heads={heads}: " +
              " | ".join(f"T={vv} {sorted(x)[len(x) // 2] * 1e3:7.1f}us" for vv, x in t.items()), flush=True)


if __name__ == "__main__":
    main()
