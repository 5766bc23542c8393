#!/usr/bin/env python3
"""ome_gemm (csrc/kernels/gemm.hip) vs hipBLASLt (F.linear) on the Llama-3-8B projections.
Cold weights: every call uses the next of several weight copies (> 256 MiB Infinity Cache in
total), as in a layer stack; activations stay warm.  Prints us and TF/s per (M, shape, variant)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
DEV = torch.device("cuda")


def bench(fn, n_w, iters=30):
    for i in range(4):
        fn(i % n_w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


VARS = [int(v) for v in os.environ.get("GEMM_VARS", "1,2,3").split(",")]


def main():
    ms = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "256,512,913,2048").split(",")]
    for name, (N, K) in SHAPES.items():
        n_w = max(2, -(-(600 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_w)]
        for M in ms:
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            ref = F.linear(x, ws[0]).float()
            fl = 2 * M * N * K
            row = [f"M={M:5d} {name:8s}"]
            t = bench(lambda i: F.linear(x, ws[i]), n_w)
            row.append(f"hipblaslt {t:7.1f}us {fl / t / 1e6:5.0f}TF")
            for var in VARS:
                ops.call("ome_gemm_set_variant", var)
                best = None
                for sp in (1, 2, 4, 8):
                    if K % (64 * sp):
                        continue
                    wsb = torch.empty(sp * M * N, dtype=torch.float32, device=DEV) if sp > 1 else None
                    y = ops.gemm(x, ws[0], splits=sp, ws=wsb)
                    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                    t = bench(lambda i: ops.gemm(x, ws[i], splits=sp, ws=wsb), n_w)
                    if err > 1e-2:
                        row.append(f"v{var}s{sp} ERR {err:.2g}")
                    if best is None or t < best[0]:
                        best = (t, sp)
                row.append(f"v{var} s{best[1]} {best[0]:7.1f}us {fl / best[0] / 1e6:5.0f}TF")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
