#!/usr/bin/env python3
"""ome_gemm_pp (csrc/kernels/gemm_pp.hip) vs hipBLASLt (F.linear) and the stream-K kernel.

Random operands (uniform-ish normal), cold weights for the Llama-3-8B projection shapes (every call
uses the next of several weight copies, > 256 MiB in total), warm for the square shapes.  Each
kernel is checked against an fp32 reference once before it is timed; timings of the variants are
interleaved in one process (cdna_hip_programming.md §5.4 rule 24)."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

DEV = torch.device("cuda")
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def bench(fn, n_w, iters):
    for i in range(3):
        fn(i % n_w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="256,512,1024,2048,2304")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--square", default="4096,8192")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    for S in [int(v) for v in a.square.split(",") if v]:
        x = torch.randn(S, S, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(S, S, device=DEV, dtype=torch.bfloat16) / S ** 0.5
        assert ((ops.gemm_pp(x, w).float() - (x.float() @ w.float().t())).abs().max() < 0.1)
        fl = 2 * S ** 3
        for rnd in range(2):
            tl = bench(lambda i: F.linear(x, w), 1, a.iters)
            tp = bench(lambda i: ops.gemm_pp(x, w), 1, a.iters)
            print(f"square {S}: hipblaslt {tl:8.1f}us {fl / tl / 1e6:6.0f}TF  pp {tp:8.1f}us {fl / tp / 1e6:6.0f}TF"
                  f"  x{tl / tp:.2f}", flush=True)
        del x, w
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        epi = 2 if name == "gate_up" else 0
        n_w = max(2, -(-(600 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_w)]
        wi = [ops.interleave_gate_up(w) for w in ws] if epi else ws
        for M in [int(v) for v in a.m.split(",")]:
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            ref = F.linear(x, ws[0]).float()
            if epi:
                ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            y = ops.gemm_pp(x, wi[0], epi=epi)
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            fl = 2 * M * N * K
            if epi:
                t_lib = bench(lambda i: ops.act_and_mul(F.linear(x, wi[i]), interleaved=True), n_w, a.iters)
            else:
                t_lib = bench(lambda i: F.linear(x, ws[i]), n_w, a.iters)
            t_pp = bench(lambda i: ops.gemm_pp(x, wi[i], epi=epi), n_w, a.iters)
            plan = ops.gemm_sk_plan(M, N, K, epi)
            sk = ""
            if plan:
                bn, nwg, bm = plan
                t_sk = bench(lambda i: ops.gemm_sk(x, wi[i], epi=epi, bn=bn, nwg=nwg, bm=bm), n_w, a.iters)
                sk = f" sk {t_sk:7.1f}us"
            print(f"M={M:5d} {name:8s} lib{'+act' if epi else ''} {t_lib:7.1f}us {fl / t_lib / 1e6:5.0f}TF  "
                  f"pp {t_pp:7.1f}us {fl / t_pp / 1e6:5.0f}TF x{t_lib / t_pp:.2f}{sk} err {err:.1e}", flush=True)
        del ws, wi
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
