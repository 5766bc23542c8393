#!/usr/bin/env python3
"""Decode-GEMM microbenchmark (Llama-3-8B projections at decode batch M): library variants."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="128,256")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for M in [int(x) for x in a.m.split(",")]:
        for name, (N, K) in SHAPES.items():
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            res = {}
            res["linear"] = timeit(lambda: F.linear(x, w))
            res["swapped"] = timeit(lambda: torch.mm(w, x.t()))
            for lib in ("cublaslt", "cublas"):
                try:
                    torch.backends.cuda.preferred_blas_library(lib)
                    res[f"linear[{lib}]"] = timeit(lambda: F.linear(x, w))
                except Exception as e:  # noqa: BLE001
                    res[f"linear[{lib}]"] = float("nan")
            torch.backends.cuda.preferred_blas_library("cublaslt")
            wb = N * K * 2
            print(f"M={M:4d} {name:8s} " + "  ".join(f"{k}={v:6.1f}us({wb / v / 1e6:4.2f}TB/s)" for k, v in res.items()),
                  flush=True)


if __name__ == "__main__":
    main()
