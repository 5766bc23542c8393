#!/usr/bin/env python3
"""Decode-shaped GEMMs (Llama-3-8B projections at M decode rows): ``ome_skinny_gemm`` at several
split-K factors vs hipBLASLt (F.linear).  Prints time, weight-streaming TB/s and max error vs an
fp32 reference."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

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
    dev = torch.device("cuda")
    for M in (64, 128, 256):
        for name, (N, K) in SHAPES.items():
            torch.manual_seed(0)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            ref = (x.float() @ w.float().t())
            wb = N * K * 2
            line = [f"M={M:4d} {name:8s} hipblaslt={timeit(lambda: F.linear(x, w)):7.1f}us"]
            for sp in sorted({1, 2, 4, 8, ops.skinny_splits(M, N, K)}):
                if sp > K // 64:
                    continue
                out = ops.skinny_gemm(x, w, splits=sp)
                err = (out.float() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                t = timeit(lambda: ops.skinny_gemm(x, w, splits=sp, out=out))
                tag = "*" if sp == ops.skinny_splits(M, N, K) else ""
                line.append(f"s{sp}{tag}={t:7.1f}us({wb / t / 1e6:4.2f}TB/s,err {err:.1e})")
            print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
