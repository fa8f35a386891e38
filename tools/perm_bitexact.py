"""Runs a set of extended-epilogue GEMMs (bias, residual, DropPath row scale, activation backward from U; bf16) and
saves the outputs, so two runs under SVK_PK_PERM=1 / 0 can be compared bit for bit.
Usage: python tools/perm_bitexact.py OUT.pt | python tools/perm_bitexact.py --compare A.pt B.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))

SHAPES = [(50176, 320, 320, 196), (200704, 128, 512, 784), (12544, 512, 512, 49), (275968, 256, 64, 3136), (68992, 512, 128, 784), (17248, 1280, 320, 196), (17248, 320, 1280, 196),
          (2000, 136, 72, 25), (4312, 512, 2048, 49), (1003, 64, 96, 17)]


def main():
    if sys.argv[1] == "--compare":
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        for k in a:
            same = torch.equal(a[k], b[k])
            print(f"{k}: {'bit-identical' if same else 'DIFFERENT max ' + str(float((a[k].float() - b[k].float()).abs().max()))}")
            assert same, k
        return
    from svk import ops
    dev, dt = torch.device("cuda:0"), torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    for M, N, K, rpf in SHAPES:
        a = torch.randn(M, K, device=dev, generator=g).to(dt)
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
        bias = torch.randn(N, device=dev, generator=g)
        u = torch.randn(M, N, device=dev, generator=g).to(dt)
        r = torch.randn(M, N, device=dev, generator=g).to(dt)
        rs = (torch.rand((M + rpf - 1) // rpf, device=dev, generator=g) < 0.9).float() / 0.9
        out[f"{M}x{N}x{K}_u"] = ops.gemm(a, w, bias, row_scale=rs, rows_per=rpf, dact="gelu", dact_src=u).cpu()
        out[f"{M}x{N}x{K}_ur"] = ops.gemm(a, w, bias, residual=r, row_scale=rs, rows_per=rpf, dact="gelu",
                                          dact_src=u).cpu()
        out[f"{M}x{N}x{K}_r"] = ops.gemm(a, w, None, residual=r, row_scale=rs, rows_per=rpf).cpu()
        out[f"{M}x{N}x{K}_k"] = ops._last_kernel()
        a16, w16, r16 = a.to(torch.float16), w.to(torch.float16), r.to(torch.float16)
        out[f"{M}x{N}x{K}_p16"] = ops.gemm(a16, w16, bias, residual=r16).cpu()      # plain residual epilogue
        out[f"{M}x{N}x{K}_pk"] = ops._last_kernel()
    torch.save({k: v for k, v in out.items() if torch.is_tensor(v)}, sys.argv[1])
    print({k: v for k, v in out.items() if not torch.is_tensor(v)})


if __name__ == "__main__":
    main()
