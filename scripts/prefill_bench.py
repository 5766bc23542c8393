#!/usr/bin/env python3
"""Prefill-attention microbenchmark: v1 vs v2 on Llama-3-8B heads (Hq=32, Hkv=8)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    Hq, Hkv, D, P = 32, 8, 128, 16
    for q_lens, kv_lens in (([512] * 2, [512] * 2), ([480] * 4, [480] * 4), ([2048], [2048]), ([8192], [8192])):
        npages = sum(-(-L // P) for L in kv_lens) + 8
        kc = torch.randn(npages, Hkv, P, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn(npages, Hkv, D, P, device=dev, dtype=torch.bfloat16)
        mx = max(-(-L // P) for L in kv_lens) + 1
        bt = torch.zeros(len(kv_lens), mx, dtype=torch.int32)
        o = 1
        for i, L in enumerate(kv_lens):
            n = -(-L // P)
            bt[i, :n] = torch.arange(o, o + n)
            o += n
        bt = bt.to(dev)
        T = sum(q_lens)
        q = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
        cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=dev)
        kvl = torch.tensor(kv_lens, dtype=torch.int32, device=dev)
        items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=dev)
        flops = sum(4 * Hq * D * (ql * (kl - ql) + ql * (ql + 1) / 2) for ql, kl in zip(q_lens, kv_lens))
        ref = None
        for v in ("1", "2"):
            os.environ["OME_PREFILL_ATTN"] = v
            out = ops.paged_prefill(q, kc, vc, bt, cu, kvl, items, D ** -0.5)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float()
            err = (out.float() - ref).abs().max().item()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                ops.paged_prefill(q, kc, vc, bt, cu, kvl, items, D ** -0.5, out=out)
            s.record()
            for _ in range(20):
                ops.paged_prefill(q, kc, vc, bt, cu, kvl, items, D ** -0.5, out=out)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1000 / 20
            print(f"q={q_lens} kv={kv_lens} v{v}: {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s  maxerr {err:.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
