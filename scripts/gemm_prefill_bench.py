#!/usr/bin/env python3
"""Mixed/prefill-step GEMM microbenchmark (Llama-3-8B projections at M = decode rows + prefill
chunk): hipBLASLt heuristic vs TunableOp-tuned, to decide whether M should be bucketed (padded)
onto tuned shapes.  Prints TF/s per (M, projection)."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--m", default="320,512,737,1024,1237,1536,2048,3000,4096,8448")
    ap.add_argument("--tune", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    tun = torch.cuda.tunable
    ws = {k: torch.randn(N, K, device=dev, dtype=torch.bfloat16) for k, (N, K) in SHAPES.items()}
    tot = {"heur": 0.0, "tuned": 0.0}
    for M in [int(x) for x in a.m.split(",")]:
        row = []
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = ws[name]
            tun.enable(False)
            t0 = timeit(lambda: F.linear(x, w))
            t1 = float("nan")
            if a.tune:
                tun.enable(True)
                tun.tuning_enable(True)
                tun.set_max_tuning_duration(30)
                tun.set_max_tuning_iterations(20)
                F.linear(x, w)
                tun.tuning_enable(False)
                t1 = timeit(lambda: F.linear(x, w))
                tun.enable(False)
            fl = 2 * M * N * K
            tot["heur"] += t0
            tot["tuned"] += t1 if t1 == t1 else t0
            row.append(f"{name}={fl / t0 / 1e6:5.0f}/{fl / t1 / 1e6 if t1 == t1 else 0:5.0f}TF")
        print(f"M={M:5d} " + "  ".join(row), flush=True)
    print(f"sum us heuristic {tot['heur']:.0f} tuned {tot['tuned']:.0f}", flush=True)


if __name__ == "__main__":
    main()
