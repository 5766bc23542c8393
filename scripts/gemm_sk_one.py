#!/usr/bin/env python3
"""Run one ome_gemm_sk configuration (or hipBLASLt) back to back, for rocprofv3 counter passes.
usage: gemm_sk_one.py SHAPE M BN NWG [ITERS]   (BN 0 = hipBLASLt F.linear)"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    name, M, bn, nwg = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 50
    N, K = SHAPES[name]
    dev = torch.device("cuda")
    n_w = max(2, -(-(600 << 20) // (N * K * 2)))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_w)]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    epi = 2 if name == "gate_up" and bn else 0
    out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
    for i in range(iters):
        if bn:
            ops.gemm_sk(x, ws[i % n_w], out=out, epi=epi, bn=bn, nwg=nwg)
        else:
            F.linear(x, ws[i % n_w])
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
