#!/usr/bin/env python3
"""Sampling kernel per decode step (256 rows x 128256 vocab, bf16 logits; HIP-graph replay):
greedy (the headline's temperature 0) and temperature 0.8 / top-p 0.9 / top-k 50."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

B, V = 256, 128256
dev = torch.device("cuda")
logits = (torch.randn(B, V, device=dev) * 3).to(torch.bfloat16)
seeds = torch.arange(B, device=dev, dtype=torch.int64)


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


for name, t, k, p in (("greedy", 0.0, -1, 1.0), ("T0.8 top_p 0.9", 0.8, -1, 0.9), ("T0.8 top_k 50 top_p 0.9", 0.8, 50, 0.9)):
    temp = torch.full((B,), t, device=dev)
    tk = torch.full((B,), k, device=dev, dtype=torch.int32)
    tp = torch.full((B,), p, device=dev)
    mp = torch.zeros(B, device=dev)
    us = timed(lambda: ops.sample(logits, temp, tk, tp, mp, seeds, 0))
    ids, _ = ops.sample(logits, temp, tk, tp, mp, seeds, 0)
    ok = bool((ids == logits.float().argmax(-1).int()).all()) if t == 0 else True
    print(f"{name:26s} {us:8.1f} us per step (B={B}, V={V})" + ("  argmax ok" if ok and t == 0 else ""), flush=True)

# kept-set sizes on this synthetic row distribution (how much the Gumbel pass must hash)
z = logits[0].float() / 0.8
p = torch.softmax(z, 0)
srt = torch.sort(p, descending=True).values
print(f"tokens kept by top_p 0.9 on row 0: {int((torch.cumsum(srt, 0) < 0.9).sum()) + 1} of {V}")
