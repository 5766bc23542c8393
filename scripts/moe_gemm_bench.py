#!/usr/bin/env python3
"""Grouped MoE GEMM microbenchmark (gate_up rows compared in token order: the align kernel's
within-expert order is atomic-order dependent) (decode-time shapes): v1 (BK 32, single LDS buffer) vs v2
(double-buffered, BK 64 / 128).  Each variant runs in its own process (OME_MOE_GEMM is read once
by the library); outputs are checked against v1.  Bandwidth = expert weight bytes / time."""
import os
import subprocess
import sys

SHAPES = [  # name, E, H, I, T, k
    ("mixtral-8x7b", 8, 4096, 14336, 256, 2),
    ("qwen3-30b-a3b", 128, 2048, 768, 256, 8),
    ("dsv2-lite", 64, 2048, 1408, 256, 6),
    ("gpt-oss-20b", 32, 2880, 2880, 256, 4),
    ("mixtral-prefill", 8, 4096, 14336, 2048, 2),
    ("qwen3-prefill", 128, 2048, 768, 4096, 8),
    ("mixtral-mid", 8, 4096, 14336, 640, 2),
]


def child():
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ome_amd import ops
    from ome_amd.ops._native import call

    torch.manual_seed(0)
    dev = "cuda"
    for name, E, H, I, T, k in SHAPES:
        x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
        w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
        w2 = torch.randn(E, H, I, device=dev, dtype=torch.bfloat16) * 0.02
        logits = torch.randn(T, E, device=dev)
        tw, tid = ops.moe_route(logits, k, True)
        n = T * k
        offsets = torch.empty(E + 1, dtype=torch.int32, device=dev)
        sorted_ids = torch.empty(n, dtype=torch.int32, device=dev)
        inv = torch.empty(n, dtype=torch.int32, device=dev)
        call("ome_moe_align", tid.data_ptr(), n, E, offsets.data_ptr(), sorted_ids.data_ptr(), inv.data_ptr(),
             ops.stream_ptr())
        tm = int(os.environ["OME_MOE_TILE"])
        mt = -(-n // tm) + E
        gu = torch.empty(n, 2 * I, dtype=torch.bfloat16, device=dev)
        h = torch.randn(n, I, device=dev, dtype=torch.bfloat16)
        y = torch.empty(n, H, dtype=torch.bfloat16, device=dev)

        def g1():
            call("ome_moe_gemm", x.data_ptr(), x.stride(0), sorted_ids.data_ptr(), k, w13.data_ptr(),
                 offsets.data_ptr(), E, 2 * I, H, mt, gu.data_ptr(), gu.stride(0), None, tm, ops.stream_ptr())

        def g2():
            call("ome_moe_gemm", h.data_ptr(), h.stride(0), None, 0, w2.data_ptr(), offsets.data_ptr(), E, H, I, mt,
                 y.data_ptr(), y.stride(0), None, tm, ops.stream_ptr())

        res = []
        for f, nbytes in ((g1, w13.numel() * 2), (g2, w2.numel() * 2)):
            for _ in range(5):
                f()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(30):
                f()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1000 / 30
            res.append(f"{us:8.1f}us {nbytes / us / 1e6:5.2f}TB/s")
        torch.save({"gu": gu.index_select(0, inv.long()).cpu(), "y": y.cpu()}, f"/tmp/moe_{name}_{os.environ['OME_MOE_GEMM']}_{tm}.pt")
        print(f"{os.environ['OME_MOE_GEMM']:>4} tile{tm:<4d}{name:16s} w13 {res[0]} | w2 {res[1]}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        return child()
    import torch

    runs = [("1", "64"), ("2", "64"), ("2", "128")]
    for v, t in runs:
        subprocess.run([sys.executable, __file__, "child"], env={**os.environ, "OME_MOE_GEMM": v, "OME_MOE_TILE": t},
                       check=True)
    for name, *_ in SHAPES:
        ref = torch.load(f"/tmp/moe_{name}_1_64.pt", weights_only=True)
        for v in ("2_64", "2_128"):
            got = torch.load(f"/tmp/moe_{name}_{v}.pt", weights_only=True)
            err = max((got[t].float() - ref[t].float()).abs().max().item() for t in ("gu", "y"))
            print(f"check {name} v{v} max|diff| vs v1 = {err:.3e}")
            assert err < 5e-2


if __name__ == "__main__":
    main()
