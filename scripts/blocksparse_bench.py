"""Phi-3-small block-sparse prefill attention vs the dense-masked kernel (verdict r05 item 8).

One layer's attention of Phi-3-small-8k (32 query / 8 kv heads, D 128, blocks of 64 keys, 16
local blocks, vertical stride 8, stripes rotating with the head) over one 8k-token prompt, with
the engine's own work plan (``ops.prefill_plan``, rows from ``ops.prefill_rows``).  Run once per
mode; the kernel switches are read once per process:

    python scripts/blocksparse_bench.py                                    # skip + FAST body (default)
    OME_BS_SKIP=0 OME_PREFILL_FAST=0 python scripts/blocksparse_bench.py   # r05: mask only, generic body
    python scripts/blocksparse_bench.py --dense                            # no sparsity at all
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ome_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=8192)
    ap.add_argument("--dense", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--decode-batch", type=int, default=32)
    a = ap.parse_args()
    Hq, Hkv, D, P, L = 32, 8, 128, 16, a.len
    dev = "cuda"
    npages = L // P + 2
    kc = torch.randn(npages, Hkv, P, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(npages, Hkv, D, P, device=dev, dtype=torch.bfloat16)
    bt = (torch.arange(npages - 1, device=dev, dtype=torch.int32) + 1).view(1, -1)
    q = torch.randn(L, Hq, D, device=dev, dtype=torch.bfloat16)
    cu = torch.tensor([0, L], dtype=torch.int32, device=dev)
    kl = torch.tensor([L], dtype=torch.int32, device=dev)
    rows = ops.prefill_rows(Hq, Hkv, D, P)
    items, split, comb, chunk, parts = ops.prefill_plan([L], [L], tile=rows, kv_heads=Hkv)
    t = lambda x, c: torch.tensor(x, dtype=torch.int32, device=dev).view(-1, c) if x else None  # noqa: E731
    plan = ops.PrefillPlan(t(items, 2), t(split, 4), t(comb, 4), chunk, parts, rows)
    bs = None if a.dense else (64, 16, 8, 1, 0)
    scale = 1.0 / D
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, plan, scale, blocksparse=bs)
    for _ in range(3):
        ops.paged_prefill(q, kc, vc, bt, cu, kl, plan, scale, out=out, blocksparse=bs)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(a.iters):
        ops.paged_prefill(q, kc, vc, bt, cu, kl, plan, scale, out=out, blocksparse=bs)
    e[1].record()
    torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / a.iters
    dense_flops = 4 * Hq * D * L * (L + 1) / 2
    mode = "dense" if a.dense else ("mask-only" if os.environ.get("OME_BS_SKIP") == "0" else "skip") + \
        ("" if a.dense else (", generic body" if os.environ.get("OME_PREFILL_FAST") == "0" else ", fast body"))
    print(json.dumps({"op": "prefill", "mode": mode, "len": L, "rows": rows, "split_parts": parts,
                      "ms": round(ms, 3), "dense_equiv_TFs": round(dense_flops / ms / 1e9, 1)}), flush=True)
    # decode: B sequences of L cached keys, one query token each (the same pattern at qpos = L - 1)
    B = a.decode_batch
    kc = torch.randn(B * (L // P) + 2, Hkv, P, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(B * (L // P) + 2, Hkv, D, P, device=dev, dtype=torch.bfloat16)
    bt = (torch.arange(B * (L // P), device=dev, dtype=torch.int32) + 1).view(B, -1)
    qd = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    ws = ops.DecodeWorkspace(B, Hq, D, L, 512, dev)
    od = ops.paged_decode(qd, kc, vc, bt, sl, scale, ws, blocksparse=bs)
    for _ in range(3):
        ops.paged_decode(qd, kc, vc, bt, sl, scale, ws, out=od, blocksparse=bs)
    torch.cuda.synchronize()
    e[0].record()
    for _ in range(a.iters):
        ops.paged_decode(qd, kc, vc, bt, sl, scale, ws, out=od, blocksparse=bs)
    e[1].record()
    torch.cuda.synchronize()
    us = e[0].elapsed_time(e[1]) * 1e3 / a.iters
    kv_bytes = B * L * Hkv * D * 2 * 2
    print(json.dumps({"op": "decode", "mode": mode, "batch": B, "len": L, "us": round(us, 1),
                      "dense_equiv_TBs": round(kv_bytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
