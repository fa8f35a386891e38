"""Run torch.matmul (hipBLASLt) on the MFMA-bound MiT-b2 (B = 256) GEMM shapes, f16, so that a
rocprofv3 kernel trace names the library kernels that win there (tile, MFMA shape, waves, LDS use
are encoded in the Tensile kernel name).  Usage (GPU box):
  rocprofv3 --kernel-trace --stats -d gpurun_out/blaslt -o run -- python tools/blaslt_names.py"""
import torch

SHAPES = [(12544, 2048, 1024, "head"), (12544, 512, 2048, "s4 fc2"), (50176, 320, 1280, "s3 fc2"),
          (12544, 1024, 512, "s4 kv"), (50176, 1280, 320, "s3 fc1"), (12544, 2048, 512, "s4 fc1")]


def main():
    dev = torch.device("cuda:0")
    for M, N, K, what in SHAPES:
        a = torch.randn(M, K, device=dev).half()
        w = torch.randn(N, K, device=dev).half()
        out = torch.empty(M, N, device=dev, dtype=torch.half)
        for _ in range(3):
            torch.matmul(a, w.t(), out=out)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            torch.matmul(a, w.t(), out=out)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        print(f"{what:8s} ({M},{N},{K}) {ms * 1e3:7.1f}us {2 * M * N * K / ms / 1e9:6.0f}TF", flush=True)


if __name__ == "__main__":
    main()
