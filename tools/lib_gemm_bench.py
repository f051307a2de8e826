"""What the vendor GEMM (torch.matmul -> hipBLASLt / rocBLAS on ROCm) reaches on the
prefill's GEMM shapes (Llama-3.2-3B, T = 4096, f16 in, f32 accumulate, f16 out): the
ceiling a library call would set for our fused 8-phase kernels (prefill_gemm.h).
Timing only -- nothing here is on the product path.

usage: python tools/lib_gemm_bench.py [--iters 20]"""
import argparse

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    shapes = {"qkv (q | k | v)": (4096, 5120, 3072), "qkv k|v over [hi|lo]": (4096, 2048, 6144),
              "wo": (4096, 3072, 3072), "w1|w3": (4096, 16384, 3072), "w2": (4096, 3072, 8192),
              "logits": (4096, 128256, 3072)}
    dev = torch.device("cuda:0")
    for name, (m, n, k) in shapes.items():
        a = torch.randn(m, k, device=dev, dtype=torch.float16)
        w = torch.randn(n, k, device=dev, dtype=torch.float16)
        for _ in range(3):
            torch.nn.functional.linear(a, w)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.nn.functional.linear(a, w)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        ms = ts[len(ts) // 2]
        print(f"{name:22s} M {m} N {n:6d} K {k}: {ms * 1e3:8.1f} us  {2 * m * n * k / ms / 1e9:7.1f} TFLOP/s",
              flush=True)
        del a, w


if __name__ == "__main__":
    main()
