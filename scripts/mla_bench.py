"""Time ``ops.mla_attn`` (csrc/kernels/mla.hip) on DeepSeek-V3 decode shapes: T sequences of L
cached tokens each, H = 128 heads, DK = 576 / DV = 512 latent rows.  Prints one JSON line per shape
with microseconds per call and the effective latent-KV read bandwidth (every sequence's KV once).

    python scripts/mla_bench.py                 # all-heads kernel
    OME_MLA_ALL=0 python scripts/mla_bench.py   # 16-head kernel (A/B)
    OME_MLA_ALL_MIN_T=0 python scripts/mla_bench.py   # all-heads even at T <= 4 (A/B of the cutover)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ome_amd import ops  # noqa: E402


def run(T, L, H=128, iters=50):
    dev = "cuda"
    ppr = -(-L // 16)
    cache = (torch.randn(T * ppr + 1, 16, 576, device=dev) * 0.5).to(torch.bfloat16)
    bt = (torch.randperm(T * ppr, device=dev) + 1).view(T, ppr).to(torch.int32)
    q = (torch.randn(T, H, 576, device=dev) * 0.3).to(torch.bfloat16)
    rows = torch.arange(T, dtype=torch.int32, device=dev)
    kl = torch.full((T,), L, dtype=torch.int32, device=dev)
    ws = ops.MLAWorkspace(dev)
    out = torch.empty(T, H, 512, dtype=torch.bfloat16, device=dev)
    for _ in range(5):
        ops.mla_attn(q, cache, bt, rows, kl, 0.07, ws=ws, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.mla_attn(q, cache, bt, rows, kl, 0.07, ws=ws, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    kv = T * L * 576 * 2
    flops = 2 * T * H * L * (576 + 512)
    return {"T": T, "L": L, "H": H, "parts": ops.MLAWorkspace.parts(T, H), "us": round(us, 1),
            "kv_GBps": round(kv / us / 1e3, 1), "TFLOPs": round(flops / us / 1e6, 1),
            "kernel": "all-heads" if ops.MLAWorkspace.all_heads(H, 576, T) else "16-head"}


if __name__ == "__main__":
    for T, L in [(1, 4096), (2, 4096), (4, 4096), (6, 2048), (8, 2048), (32, 1024), (64, 1024), (128, 1024), (128, 4096), (256, 2048)]:
        print(json.dumps(run(T, L)), flush=True)
