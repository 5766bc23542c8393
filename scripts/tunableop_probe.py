#!/usr/bin/env python3
"""How much does TunableOp's per-shape search buy over the hipBLASLt heuristic at mixed-step M?
Llama-3-8B projections, warm weights, F.linear timed with hipGraph replay."""
import os
import sys

import torch
import torch.nn.functional as F


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (5 * reps)


shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
Ms = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "512,768,1024,1280,2048").split(",")]
W = {k: torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
res = {}
for M in Ms:
    for k, w in W.items():
        x = torch.randn(M, w.shape[1], device="cuda", dtype=torch.bfloat16)
        res[(M, k, "heur")] = timed(lambda: F.linear(x, w))
tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(60)
tun.set_max_tuning_iterations(40)
tun.set_filename("/tmp/tunable_probe.csv", insert_device_ordinal=False)
for M in Ms:
    for k, w in W.items():
        x = torch.randn(M, w.shape[1], device="cuda", dtype=torch.bfloat16)
        F.linear(x, w)    # tunes this shape
        torch.cuda.synchronize()
tun.tuning_enable(False)
for M in Ms:
    tot_h = tot_t = 0.0
    line = [f"M={M:5d}"]
    for k, w in W.items():
        x = torch.randn(M, w.shape[1], device="cuda", dtype=torch.bfloat16)
        t = timed(lambda: F.linear(x, w))
        h = res[(M, k, "heur")]
        tot_h += h
        tot_t += t
        line.append(f"{k} {h:6.1f}->{t:6.1f}us")
    line.append(f"layer {tot_h:6.1f}->{tot_t:6.1f}us ({100 * (tot_h - tot_t) / tot_h:+.1f}%)")
    print(" | ".join(line), flush=True)
