#!/usr/bin/env python3
"""Per-call time of the decode layer's small kernels (rope+KV write, fused add+RMSNorm, SwiGLU)
under their launch-geometry knobs, Llama-3-8B shapes, graph-replayed (20 calls per graph)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.ops._native import call  # noqa: E402


def timed(fn, reps=20, iters=20):
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
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (reps * iters)


def main():
    dev = torch.device("cuda")
    H, Hq, Hkv, D, I = 4096, 32, 8, 128, 14336
    pages = 16384
    kc = torch.zeros(pages, Hkv, 16, D, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros(pages, Hkv, D, 16, dtype=torch.bfloat16, device=dev)
    cs = torch.randn(8192, D, device=dev)
    w = torch.randn(H, dtype=torch.bfloat16, device=dev)
    for T in (256, 1024, 4096):
        qkv = torch.randn(T, (Hq + 2 * Hkv) * D, dtype=torch.bfloat16, device=dev)
        pos = torch.randint(0, 4000, (T,), dtype=torch.int32, device=dev)
        slots = (torch.randperm(pages, device=dev)[:T].to(torch.int32) * 16 + 3).contiguous() if T <= pages else None
        q = torch.empty(T, Hq, D, dtype=torch.bfloat16, device=dev)
        x = torch.randn(T, H, dtype=torch.bfloat16, device=dev)
        r = torch.randn(T, H, dtype=torch.bfloat16, device=dev)
        gu = torch.randn(T, 2 * I, dtype=torch.bfloat16, device=dev)
        out = torch.empty(T, I, dtype=torch.bfloat16, device=dev)
        line = [f"T={T:5d}"]
        for ny in (1, 2, 3, 4):
            call("ome_rope_set_split", ny)
            t = timed(lambda: ops.rope_qkv_cache(qkv, pos, cs, D, q, kc, vc, slots, Hq, Hkv, D))
            line.append(f"rope ny{ny} {t:6.2f}")
        call("ome_rope_set_split", 0)
        for nt in (128, 256, 512):
            call("ome_norm_set_threads", nt)
            t = timed(lambda: ops.fused_add_rmsnorm(x, r, w, 1e-5))
            line.append(f"norm nt{nt} {t:6.2f}")
        call("ome_norm_set_threads", 0)
        t = timed(lambda: ops.act_and_mul(gu, 0, out=out))
        line.append(f"act {t:6.2f}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
