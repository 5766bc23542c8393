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
    rows = ops.prefill_rows(Hq, Hkv, D, P)   # OME_PREFILL_ROWS=64: the 8-wave kernel over 64-row items
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens, rows), dtype=torch.int32, device=DEV).view(-1, 2)
    if rows != 32:
        items = ops.PrefillPlan(items, items[:0], items[:0], 0, 0, rows)
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
    # fp32 reference on the GPU for (up to) the first two sequences, 512 query rows at a time
    err = 0.0
    for i in range(min(2, len(q_lens))):
        L, ql = kv_lens[i], q_lens[i]
        pages = bt[i, :-(-L // P)].long()
        K = kc[pages].permute(1, 0, 2, 3).reshape(Hkv, -1, D)[:, :L].float()          # [Hkv, L, D]
        V = vc[pages].permute(1, 0, 3, 2).reshape(Hkv, -1, D)[:, :L].float()
        K, V = K.repeat_interleave(Hq // Hkv, 0), V.repeat_interleave(Hq // Hkv, 0)
        q0 = int(cu[i])
        for r0 in range(0, ql, 512):
            r1 = min(ql, r0 + 512)
            qq = q[q0 + r0:q0 + r1].float().transpose(0, 1)                               # [Hq, n, D]
            sc = qq @ K.transpose(1, 2) * 0.0884
            pos = torch.arange(r0, r1, device=DEV)[:, None] + (L - ql)
            sc = sc.masked_fill(torch.arange(L, device=DEV)[None, :] > pos, float("-inf"))
            want = (sc.softmax(-1) @ V).transpose(0, 1)
            err = max(err, (out[q0 + r0:q0 + r1].float() - want).abs().max().item())
    n_items = items.shape[0]
    return t, n_items, err


def tflops(q_lens, kv_lens, us, Hq=32, D=128):
    fl = sum(4 * Hq * D * sum(kl - ql + r + 1 for r in range(ql)) for ql, kl in zip(q_lens, kv_lens))
    return fl / us / 1e6


if __name__ == "__main__":
    for L in (32, 64, 128, 256, 512, 1024):
        t1, n1, e1 = run([L], [L])
        t16, n16, e16 = run([L] * 16, [L] * 16)
        print(f"L={L:5d}  1 seq: {t1:7.1f} us ({n1:3d} items, err {e1:.2g})   16 seqs: {t16:7.1f} us "
              f"({n16:4d} items, err {e16:.2g})", flush=True)
    for B, L in ((16, 1024), (16, 2048), (1, 8192), (4, 4096)):
        t, n, e = run([L] * B, [L] * B, reps=5)
        print(f"{B}x{L} causal: {t:8.1f} us  {tflops([L] * B, [L] * B, t):6.0f} TF  ({n} items, err {e:.2g})",
              flush=True)
    t, n, e = run([480, 420], [480, 420])
    print(f"[480, 420]: {t:.1f} us ({n} items, err {e:.2g})")
    t, n, e = run([700, 256], [700, 256 + 512])
    print(f"[700, 256 over 512 prefix]: {t:.1f} us ({n} items, err {e:.2g})")
