#!/usr/bin/env python3
"""Decode-shaped GEMMs (Llama-3-8B projections at M decode rows): ``ome_stream_gemm`` at several
split-K factors vs hipBLASLt (F.linear).  Prints time, weight-streaming TB/s and max error vs an
fp32 reference; ``*`` marks the default plan.  Weights rotate over copies larger than the
Infinity Cache (cold, HBM-streamed, as inside a layer stack)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, ws, iters=48):
    """Mean time per call, rotating over weight copies whose total exceeds the 256 MB Infinity
    Cache, so every call streams its weight from HBM as in a real layer stack."""
    for w in ws[:3]:
        fn(w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(ws[i % len(ws)])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    dev = torch.device("cuda")
    Ms = [int(v) for v in os.environ.get("BENCH_M", "1,16,64,128,256").split(",")]
    for M in Ms:
        for name, (N, K) in SHAPES.items():
            torch.manual_seed(0)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            ref = x.float() @ w.float().t()
            wb = N * K * 2
            ws = [w] + [w.clone() for _ in range(max(1, -(-640 * 2**20 // wb)) - 1)]
            line = [f"M={M:4d} {name:8s} hipblaslt={timeit(lambda w_: F.linear(x, w_), ws):7.1f}us"]
            if M <= 8:
                og = ops.gemv(x, w)
                err = (og.float() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                t = timeit(lambda w_: ops.gemv(x, w_, out=og), ws)
                line.append(f"gemv={t:6.1f}us({wb / t / 1e6:4.2f}TB/s,err {err:.0e})")
            nf0, s0 = ops.stream_gemm_plan(M, N, K)
            cands = sorted({(nf0, s0), (1, 1), (1, 2), (1, 4), (1, 8), (1, max(1, s0 // 2)), (1, s0 * 2)})
            if M <= 128 and N % 256 == 0:
                cands += [(2, 1), (2, 2)]
            for nf, sp in cands:
                if sp > K // 64:
                    continue
                out = ops.stream_gemm(x, w, splits=sp, nf=nf)
                err = (out.float() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                t = timeit(lambda w_: ops.stream_gemm(x, w_, splits=sp, nf=nf, out=out), ws)
                tag = "*" if (nf, sp) == (nf0, s0) else ""
                line.append(f"n{nf}s{sp}{tag}={t:6.1f}us({wb / t / 1e6:4.2f}TB/s,err {err:.0e})")
            print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
