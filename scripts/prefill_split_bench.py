#!/usr/bin/env python3
"""Prefill attention per layer call (Llama-3-8B heads: 32 q / 8 kv, D 128, paged bf16 KV):
classic one-workgroup-per-32-row item vs split-KV chunks + combine (ops.prefill_plan)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

DEV = torch.device("cuda")


def run(q_lens, kv_lens, target):
    D, P, Hq, Hkv = 128, 16, 32, 8
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc = torch.randn(npages, Hkv, P, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(npages, Hkv, D, P, device=DEV, dtype=torch.bfloat16)
    bt = torch.zeros(len(kv_lens), max(-(-L // P) for L in kv_lens), dtype=torch.int32, device=DEV)
    p = 1
    for i, L in enumerate(kv_lens):
        n = -(-L // P)
        bt[i, :n] = torch.arange(p, p + n, dtype=torch.int32)
        p += n
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    items, split, comb, chunk, parts = ops.prefill_plan(q_lens, kv_lens, target=target, force=True)
    t = lambda a, c: torch.tensor(a, dtype=torch.int32, device=DEV).view(-1, c)  # noqa: E731
    classic = t(items, 2)
    plan = ops.PrefillPlan(classic, t(split, 4) if split else None, t(comb, 4) if comb else None, chunk, parts)
    res = {}
    for name, it in (("classic", classic), ("split", plan)):
        for _ in range(3):
            ops.paged_prefill(q, kc, vc, bt, cu, kl, it, 0.0884)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            ops.paged_prefill(q, kc, vc, bt, cu, kl, it, 0.0884)
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) * 1000 / 20
    a = ops.paged_prefill(q, kc, vc, bt, cu, kl, classic, 0.0884)
    b = ops.paged_prefill(q, kc, vc, bt, cu, kl, plan, 0.0884)
    err = (a.float() - b.float()).abs().max().item()
    print(f"q_lens={q_lens} target={target} chunk={chunk} parts={parts} items={len(items)} split_items={len(split)}: "
          f"classic {res['classic']:.1f} us  split {res['split']:.1f} us  max|diff| {err:.3g}", flush=True)


if __name__ == "__main__":
    for target in (64, 128, 256, 512):
        run([480, 420], [480, 420], target)
    run([480, 420, 300], [480, 420, 300], 128)
    run([700], [700], 128)
    run([2000], [2000], 128)
    run([7800], [7800], 128)
    run([256], [4096], 128)
