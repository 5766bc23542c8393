"""Microbenchmark: Llama-3-8B projection shapes, bf16 hipBLASLt vs ome_fp8_gemm (per-channel and
128x128 block scales), including the activation-quant kernel.  Prints one line per shape."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.models.quant import quantize_weight  # noqa: E402


def t(fn, n=50):
    for _ in range(5):
        fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / n


def main():
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
    for M in (256, 913, 2048, 8192):
        for name, N, K in shapes:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            q0, q1 = quantize_weight(w, 0), quantize_weight(w, 128)
            tb = t(lambda: F.linear(x, w))
            qa0, sa0 = ops.fp8_quant(x, 0)
            qa1, sa1 = ops.fp8_quant(x, 128)
            tq = t(lambda: ops.fp8_quant(x, 0))
            tg0 = t(lambda: ops.fp8_gemm(qa0, sa0, q0.q, q0.scale, 0))
            tg1 = t(lambda: ops.fp8_gemm(qa1, sa1, q1.q, q1.scale, 128))
            fl = 2 * M * N * K
            print(f"M={M:5d} {name:8s} bf16 {tb:8.1f}us ({fl / tb / 1e6:6.0f} TF, {N * K * 2 / tb / 1e3:5.2f} TB/s)"
                  f" | quant {tq:6.1f}us | fp8 pc {tg0:8.1f}us ({fl / tg0 / 1e6:6.0f} TF, {N * K / tg0 / 1e3:5.2f} TB/s)"
                  f" | fp8 blk {tg1:8.1f}us", flush=True)


if __name__ == "__main__":
    main()
