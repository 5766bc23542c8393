#!/usr/bin/env python3
"""Selective-scan kernel timing at NemotronH-8B shapes (H=128, P=64, N=128, G=8): decode (256 one-row
sequences: bound by the 2 x 4 MB fp32 state per sequence and layer) and prefill (2 x 512 rows:
bound by the sequential row loop).  OME_SSM_NT=1 switches the state I/O to non-temporal."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

H, P, N, G = 128, 64, 128, 8
dev = "cuda"


def run(S, L):
    T = S * L
    x = torch.randn(T, H * P, device=dev, dtype=torch.bfloat16)
    dt = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    B = torch.randn(T, G * N, device=dev, dtype=torch.bfloat16)
    C = torch.randn(T, G * N, device=dev, dtype=torch.bfloat16)
    A, D, db = -torch.rand(H, device=dev), torch.ones(H, device=dev), torch.zeros(H, device=dev)
    st = torch.zeros(S + 1, H, P, N, device=dev)
    cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
    slot = torch.arange(S, dtype=torch.int32, device=dev)
    reset = torch.zeros(S, dtype=torch.int32, device=dev)
    for _ in range(3):
        ops.ssm_scan(x, dt, B, C, A, D, db, 0.001, st, cu, slot, reset, H, P, N, G)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        ops.ssm_scan(x, dt, B, C, A, D, db, 0.001, st, cu, slot, reset, H, P, N, G)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 100
    gb = S * H * P * N * 4 * 2 / 1e9
    print(f"NT={os.environ.get('OME_SSM_NT', '0')} S={S:4d} rows/seq={L:4d}: {us:8.1f} us  "
          f"(state r+w {gb:.2f} GB -> {gb / us * 1e3:.2f} TB/s)", flush=True)


for nt in ("0", "1"):
    os.environ["OME_SSM_NT"] = nt
    run(256, 1)
    run(2, 512)
