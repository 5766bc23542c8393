#!/usr/bin/env python3
"""FP8 weights at decode row counts: W8A16 (csrc/kernels/w8a16.hip, fp8 weight streamed + widened
in registers, bf16 activations) vs W8A8 (activation quant + stream-K fp8) vs the bf16 projection as
``quant.linear`` routes it, with cold weights (rotating copies > the 256 MB Infinity Cache) and
every call replayed from a HIP graph.  W8A16 is checked against the fp32 reference first.

Prints one line per (shape, M) with the best W8A16 split-K factor and its fp8 weight-stream rate;
``--json`` writes {"N,K,block": {M: {"w8a16_us", "splits", "w8a8_us", "bf16_us"}}}."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.models.quant import linear, quantize_weight  # noqa: E402
from ome_amd.ops import reference as ref  # noqa: E402

SHAPES = {
    "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)],
    "dsv3": [("q_a", 1536, 7168), ("kv_a", 576, 7168), ("o", 7168, 16384), ("shared_gu", 4096, 7168)],
}


def timed(fn, n=24):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i)
        with torch.cuda.graph(g, stream=s):
            for i in range(n):
                fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / n)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama8b,dsv3")
    ap.add_argument("--rows", default="1,2,4,8,16,32,64,128,192,256")
    ap.add_argument("--blocks", default="0,128")
    ap.add_argument("--cold-mb", type=int, default=768)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = {}
    for model in a.models.split(","):
        for name, N, K in SHAPES[model]:
            copies = max(2, -(-a.cold_mb * 2**20 // (N * K)))
            wb = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(max(2, copies // 2))]
            for block in (int(b) for b in a.blocks.split(",")):
                qs = [quantize_weight(wb[i % len(wb)], block) for i in range(copies)]
                key = f"{N},{K},{block}"
                res.setdefault(key, {})
                for M in (int(r) for r in a.rows.split(",")):
                    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                    got = ops.w8a16_gemm(x, qs[0].q, qs[0].scale, block)
                    want = F.linear(x.float(), ref.fp8_dequant_weight(qs[0].q, qs[0].scale, block).float())
                    err = ((got.float() - want).norm() / want.norm()).item()
                    assert err < 1e-2, (name, M, block, err)
                    t_b = timed(lambda i: linear(x, wb[i % len(wb)]))
                    t_88 = timed(lambda i: ops.fp8_linear(x, qs[i % copies].q, qs[i % copies].scale, block))
                    mg = ops.w8a16_mgemv_splits(M, N, K)
                    cands = [None] if M <= 8 else ([None] + mg[:4] if mg else [None, 1, 2, 3, 4, 6, 8])
                    best, bs = 1e30, None
                    for sp in cands:
                        if sp is not None and sp > K // 64:
                            continue
                        t = timed(lambda i: ops.w8a16_gemm(x, qs[i % copies].q, qs[i % copies].scale, block,
                                                           splits=sp))
                        if t < best:
                            best, bs = t, sp
                    sp_used = bs if bs is not None else (1 if M <= 8 else mg[0] if mg else ops.skinny_splits(M, N, K))
                    res[key][M] = {"w8a16_us": round(best, 2), "splits": sp_used, "w8a8_us": round(t_88, 2),
                                   "bf16_us": round(t_b, 2)}
                    print(f"{model:8s} {name:9s} blk{block:<3d} M={M:4d}  bf16 {t_b:7.1f}  w8a8 {t_88:7.1f}  "
                          f"w8a16 {best:7.1f} (splits {sp_used}, {N * K / best / 1e6:5.2f} TB/s fp8)  "
                          f"x{t_b / best:4.2f} vs bf16  x{t_88 / best:4.2f} vs w8a8", flush=True)
            del wb
            torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
