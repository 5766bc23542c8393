#!/usr/bin/env python3
"""Diagnostic timings of the ping-pong GEMM body (csrc/kernels/gemm_pp.hip) at square shapes:
OME_PP_PROBE=0 normal, 1 = no LDS-DMA in the K loop (stale LDS data), 2 = no DMA and no LDS
fragment reads (MFMA + barriers only).  Run one probe per process: the launcher reads the
variable once."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

for S in (4096, 8192):
    x = torch.randn(S, S, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(S, S, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        ops.gemm_pp(x, w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        ops.gemm_pp(x, w)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) * 1000 / 20
    print(f"body {os.environ.get('OME_PP_BODY', '5')} probe {os.environ.get('OME_PP_PROBE', '0')} S={S}: {t:8.1f} us {2 * S ** 3 / t / 1e6:6.0f} TF", flush=True)
