#!/usr/bin/env python3
"""Decode-attention microbenchmark on one MI355X: kernel variants x split-K partition sizes on
the bench's context distribution (Llama-3-8B heads: Hq=32, Hkv=8, D=128, 16-token pages)."""
import argparse
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--variants", default="1,2,3")
    ap.add_argument("--parts", default="4096,1024,512,256")
    ap.add_argument("--ctx", type=int, default=0, help="fixed context (0 = bench distribution)")
    ap.add_argument("--pool-pages", type=int, default=0, help="scatter pages over a pool this large (TLB test)")
    ap.add_argument("--dyn-parts", default="", help="also per-sequence partitions: comma list of part counts "
                                                   "(the runtime's OME_DECODE_DYN_PARTS layout; 1 = what bs 256 runs)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    rng = random.Random(0)
    B, Hq, Hkv, D, P = a.batch, 32, 8, 128, 16
    lens = []
    for _ in range(B):
        if a.ctx:
            lens.append(a.ctx)
        else:
            i = max(1, min(3800, int(rng.gauss(480, 240))))
            o = max(1, int(rng.gauss(300, 150)))
            lens.append(i + rng.randrange(0, o))
    maxpg = max(-(-L // P) for L in lens) + 1
    npages = max(sum(-(-L // P) for L in lens) + 8, a.pool_pages)
    kc = torch.randn(npages, Hkv, P, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(npages, Hkv, D, P, device=dev, dtype=torch.bfloat16)
    perm = rng.sample(range(1, npages), sum(-(-L // P) for L in lens))
    bt = torch.zeros(B, maxpg, dtype=torch.int32)
    o = 0
    for b, L in enumerate(lens):
        n = -(-L // P)
        bt[b, :n] = torch.tensor(perm[o:o + n])
        o += n
    bt = bt.to(dev)
    sl = torch.tensor(lens, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    kv_bytes = sum(lens) * Hkv * D * 2 * 2
    print(f"B={B} mean ctx={sum(lens) / B:.0f} max={max(lens)} KV bytes/call={kv_bytes / 1e6:.1f} MB")
    ref = None
    cfgs = [(int(x), None) for x in a.parts.split(",") if x] + [(0, int(x)) for x in a.dyn_parts.split(",") if x]
    for part, dyn in cfgs:
        ws = ops.DecodeWorkspace(B, Hq, D, max(lens) + P, part, dev, parts=dyn) if dyn else \
            ops.DecodeWorkspace(B, Hq, D, max(lens) + P, part, dev)
        for v in a.variants.split(","):
            os.environ["OME_DECODE_ATTN"] = v
            out = ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            for _ in range(5):
                ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws, out=out)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws, out=out)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1000 / a.iters
            print(f"variant {v} part {part if not dyn else f'dyn{dyn}':>5}: {us:8.1f} us  {kv_bytes / us / 1e6:6.2f} TB/s  maxerr {err:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
