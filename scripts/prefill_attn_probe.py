#!/usr/bin/env python3
"""Where does a short prefill's attention time go?  Classic paged_prefill_v2 per layer call
(Llama-3-8B heads 32 q / 8 kv, D 128, paged bf16 KV) over (a) ONE sequence of L tokens -- the
grid is tiny, time ~ the longest item's serial chain of 64-key steps -- and (b) 16 sequences of
L tokens -- grid full.  Slope over L gives the per-step latency, intercept the fixed cost."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

DEV = torch.device("cuda")


def run(q_lens, kv_lens, reps=20):
    D, P, Hq, Hkv = 128, 16, 32, 8
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc = torch.randn(npages, Hkv, P, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(npages, Hkv, D, P, device=DEV, dtype=torch.bfloat16)
    bt = torch.zeros(len(kv_lens), max(-(-L // P) for L in kv_lens), dtype=torch.int32, device=DEV)
    perm = torch.randperm(npages - 1) + 1   # pages scattered like a busy pool
    p = 0
    for i, L in enumerate(kv_lens):
        n = -(-L // P)
        bt[i, :n] = perm[p:p + n].to(torch.int32)
        p += n
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens, 32), dtype=torch.int32, device=DEV).view(-1, 2)
    out = torch.empty_like(q)
    for _ in range(3):
        ops.paged_prefill(q, kc, vc, bt, cu, kl, items, 0.0884, out=out)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            ops.paged_prefill(q, kc, vc, bt, cu, kl, items, 0.0884, out=out)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    t = a.elapsed_time(b) * 1000 / reps
    ref = None
    if sum(q_lens) <= 1024:
        from ome_amd.ops import reference as R
        ref = R.paged_prefill(q.cpu().float(), kc.cpu().float(), vc.cpu().float(), bt.cpu(), cu.cpu(), kl.cpu(),
                              0.0884, -1, 1.0, 1.0, 0.0, None, None, None)
        err = (out.float().cpu() - ref.float()).abs().max().item()
    else:
        err = float("nan")
    return t, items.shape[0], err


if __name__ == "__main__":
    for L in (32, 64, 128, 256, 512, 1024):
        t1, n1, e1 = run([L], [L])
        t16, n16, e16 = run([L] * 16, [L] * 16)
        print(f"L={L:5d}  1 seq: {t1:7.1f} us ({n1:3d} items, err {e1:.2g})   16 seqs: {t16:7.1f} us "
              f"({n16:4d} items, err {e16:.2g})", flush=True)
    t, n, e = run([480, 420], [480, 420])
    print(f"[480, 420]: {t:.1f} us ({n} items, err {e:.2g})")
    t, n, e = run([700, 256], [700, 256 + 512])
    print(f"[700, 256 over 512 prefix]: {t:.1f} us ({n} items, err {e:.2g})")
