"""Decode-GEMM diagnosis: the planned ``ops.gemm_sk`` configuration (what ``quant.linear`` runs)
on the Llama-3-8B projections at M = 256, with weights COLD (rotating copies, > 600 MB, as in a
layer stack) and WARM (one copy re-read: served from the 256 MB Infinity Cache / L2).  A large
warm / cold gap means the kernel waits on HBM latency / bandwidth rather than on its MFMA loop.

    python scripts/gemm_warm_cold_probe.py [--m 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ome_amd import ops  # noqa: E402
from ome_amd.models.quant import linear  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timed(fn, n, iters=40):
    for i in range(4):
        fn(i % n)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    a = ap.parse_args()
    M = a.m
    for name, (N, K) in SHAPES.items():
        n_cold = max(2, -(-(600 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_cold)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        plan = ops.gemm_sk_plan(M, N, K, 0)
        cold = timed(lambda i: linear(x, ws[i]), n_cold)
        warm = timed(lambda i: linear(x, ws[0]), 1)
        gb = N * K * 2 / 1e9
        print(f"{name:8s} M={M} N={N} K={K} plan={plan}  cold {cold:6.1f} us ({gb / cold * 1e3:5.2f} TB/s)  "
              f"warm {warm:6.1f} us ({gb / warm * 1e3:5.2f} TB/s)  cold/warm {cold / warm:4.2f}", flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
