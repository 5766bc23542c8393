#!/usr/bin/env python3
"""Per-layer GEMM time of the serving path (``quant.linear`` routing + the gate_up SiLU epilogue)
as a function of the row count M, on Llama-3-8B projections with cold weights.

Question: is the mixed-step GEMM time a staircase in M (tile / wave quantisation)?  If so the
scheduler can size each mixed step's prefill chunk to land on the cheap side of a step
(``runtime/scheduler.py`` M alignment).  Prints ``M us_per_layer us_per_row`` lines and, with
``--json``, writes {M: us} for the planner.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.models.quant import linear  # noqa: E402

DEV = torch.device("cuda")
H, I, QKV = 4096, 14336, 6144


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m0", type=int, default=256)
    ap.add_argument("--m1", type=int, default=2560)
    ap.add_argument("--step", type=int, default=32)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    n_l = 3   # weight copies: 3 x 436 MB > the 256 MB Infinity Cache
    wq = [torch.randn(QKV, H, device=DEV, dtype=torch.bfloat16) / 64 for _ in range(n_l)]
    wo = [torch.randn(H, H, device=DEV, dtype=torch.bfloat16) / 64 for _ in range(n_l)]
    wg = [ops.interleave_gate_up(torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) / 64) for _ in range(n_l)]
    wd = [torch.randn(H, I, device=DEV, dtype=torch.bfloat16) / 120 for _ in range(n_l)]
    xb = torch.randn(a.m1, H, device=DEV, dtype=torch.bfloat16)
    ab = torch.randn(a.m1, I, device=DEV, dtype=torch.bfloat16)

    def layer(M, i):
        x, act = xb[:M], ab[:M]
        linear(x, wq[i])
        linear(x, wo[i])
        w = wg[i]
        plan = ops.gemm_sk_plan(M, w.shape[0], w.shape[1], 2)
        if plan is not None:
            ops.gemm_sk(x, w, epi=2, bn=plan[0], nwg=plan[1], bm=plan[2])
        else:
            ops.act_and_mul(linear(x, w), 0, interleaved=True)
        linear(act, wd[i])

    res = {}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    prev = None
    for M in range(a.m0, a.m1 + 1, a.step):
        for i in range(n_l):
            layer(M, i)
        best = 1e30
        for _ in range(3):
            s.record()
            for j in range(a.iters):
                layer(M, j % n_l)
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) * 1000 / a.iters)
        res[M] = round(best, 2)
        d = "" if prev is None else f"  d/row {(best - prev) / a.step:6.3f}"
        print(f"M={M:5d} {best:8.1f} us/layer  {best / M:6.3f} us/row{d}", flush=True)
        prev = best
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
