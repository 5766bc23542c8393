"""Decode-shaped W8A8: the stream-K fp8 kernel (gemm_sk.hip Q = 1 / 2) against bf16 (hipBLASLt and
the stream-K bf16 kernel) and the previous fp8 kernels (64 x 64 / 256 x 256 MX tiles), with COLD
weights (a rotating set of weight copies larger than the 256 MB Infinity Cache) -- the regime of
a decode step, whose layer stack never fits in cache.  Times include the activation-quant kernel
(the fp8 linear runs it every call).  Prints one line per (M, shape) and a JSON summary."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.models.quant import linear, quantize_weight  # noqa: E402

SHAPES = {
    "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)],
    "llama70b": [("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192), ("down", 8192, 28672)],
    "dsv3": [("q_a", 1536, 7168), ("kv_a", 576, 7168), ("o", 7168, 16384), ("shared_gu", 4096, 7168)],
}


def timed(fns, n=30):
    """Mean us per call of fn(i) over a graph of n calls cycling the weight copies."""
    for i in range(3):
        fns(i)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fns(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama8b,llama70b")
    ap.add_argument("--rows", default="1,32,128,256,512")
    ap.add_argument("--cold-mb", type=int, default=768)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = [int(r) for r in a.rows.split(",")]
    res = []
    for model in a.models.split(","):
        for name, N, K in SHAPES[model]:
            if N % 128 or K % 128:
                continue
            copies = max(2, -(-a.cold_mb * 2**20 // (N * K * 2)))
            ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
            q0 = [quantize_weight(w, 0) for w in ws]
            q1 = [quantize_weight(w, 128) for w in ws]
            for M in rows:
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                c = len(ws)
                r = {"model": model, "shape": name, "M": M, "N": N, "K": K}
                r["bf16_lib"] = timed(lambda i: F.linear(x, ws[i % c]))
                plan = ops.gemm_sk_plan(M, N, K)
                if plan:
                    r["bf16_sk"] = timed(lambda i: ops.gemm_sk(x, ws[i % c], bn=plan[0], nwg=plan[1], bm=plan[2]))
                for blk, qs in ((0, q0), (128, q1)):
                    tag = "pc" if blk == 0 else "blk"
                    ops.FP8_SK_MAX_ROWS = 0
                    r[f"fp8_{tag}_old"] = timed(lambda i: ops.fp8_linear(x, qs[i % c].q, qs[i % c].scale, blk))
                    best = None
                    for bn in ((128, 256) if blk == 0 else (128,)):
                        for nwg in (64, 128, 256):
                            if not ops.gemm_sk_fp8_ok(M, N, K, bn, nwg):
                                continue

                            def run(i, bn=bn, nwg=nwg):
                                qa, sa = ops.fp8_quant(x, blk)
                                ops.gemm_sk_fp8(qa, sa, qs[i % c].q, qs[i % c].scale, blk, bn=bn, nwg=nwg)
                            us = timed(run)
                            r[f"fp8_{tag}_sk_{bn}_{nwg}"] = us
                            if best is None or us < best[0]:
                                best = (us, bn, nwg)
                    ops.FP8_SK_MAX_ROWS = 512
                    r[f"fp8_{tag}_sk"] = best[0]
                    r[f"fp8_{tag}_sk_cfg"] = best[1:]
                # what the model actually runs: quant.linear on the bf16 weight vs on the Fp8Weight
                # (which takes its bf16 copy below fp8_bf16_max_m rows)
                r["bf16_routed"] = timed(lambda i: linear(x, ws[i % c]))
                r["fp8_pc_routed"] = timed(lambda i: linear(x, q0[i % c]))
                r["fp8_blk_routed"] = timed(lambda i: linear(x, q1[i % c]))
                print(f"  routed: bf16 {r['bf16_routed']:7.1f}us  fp8 pc {r['fp8_pc_routed']:7.1f}us "
                      f"({r['bf16_routed'] / r['fp8_pc_routed']:4.2f}x)  fp8 blk {r['fp8_blk_routed']:7.1f}us "
                      f"({r['bf16_routed'] / r['fp8_blk_routed']:4.2f}x)  bf16-copy rows <= {q0[0].bf16_max_m}",
                      flush=True)
                bf = min(r["bf16_lib"], r.get("bf16_sk", 1e9))
                print(f"{model:8s} {name:9s} M={M:4d} bf16 {bf:7.1f}us | fp8 pc: sk {r['fp8_pc_sk']:7.1f} "
                      f"old {r['fp8_pc_old']:7.1f} ({N * K / r['fp8_pc_sk'] / 1e6:4.2f} TB/s, "
                      f"{bf / r['fp8_pc_sk']:4.2f}x bf16) | fp8 blk: sk {r['fp8_blk_sk']:7.1f} "
                      f"old {r['fp8_blk_old']:7.1f} ({bf / r['fp8_blk_sk']:4.2f}x bf16)", flush=True)
                res.append(r)
            del ws, q0, q1
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
