"""FP8 grouped MoE GEMM, 64x128 vs 128x128 tiles (``OME_MOE_FP8_TILE``), DeepSeek-V3 expert
shapes (H 7168, I 2048, 256 experts, top-8) at decode and prefill token counts.  Whole
``ops.fused_moe`` call (align + quant + gate_up + SiLU*mul + quant + down + combine), weights cold
(layer copies rotated past the 256 MB Infinity Cache).

    python scripts/fp8_moe_tile_bench.py [--experts 256] [--tokens 64,256,1024,2048,4096,8192]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ome_amd import ops  # noqa: E402
from ome_amd.models.quant import quantize_experts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--experts", type=int, default=256)
    ap.add_argument("--hidden", type=int, default=7168)
    ap.add_argument("--inter", type=int, default=2048)
    ap.add_argument("--topk", type=int, default=8)
    ap.add_argument("--tokens", default="64,256,1024,2048,4096,8192")
    ap.add_argument("--copies", type=int, default=2)
    a = ap.parse_args()
    E, H, I, k = a.experts, a.hidden, a.inter, a.topk
    dev = torch.device("cuda")
    torch.manual_seed(0)
    layers = []
    for _ in range(a.copies):   # 2 x 11 GB of fp8 experts: no layer is cache-resident
        w13 = quantize_experts((torch.randn(E, 2 * I, H, device=dev) * H ** -0.5).to(torch.bfloat16))
        w2 = quantize_experts((torch.randn(E, H, I, device=dev) * I ** -0.5).to(torch.bfloat16))
        layers.append((w13, w2))
        torch.cuda.empty_cache()
    wbytes = sum(t.numel() for t in (layers[0][0].q, layers[0][1].q))
    for T in [int(t) for t in a.tokens.split(",")]:
        x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
        tw, tid = ops.moe_route(torch.randn(T, E, device=dev), k)
        row = {}
        for tile in ("64", "128"):
            os.environ["OME_MOE_FP8_TILE"] = tile
            for i in range(4):
                ops.fused_moe(x, tw, tid, *layers[i % a.copies], 0, 1.0)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 10
            s.record()
            for i in range(n):
                ops.fused_moe(x, tw, tid, *layers[i % a.copies], 0, 1.0)
            e.record()
            torch.cuda.synchronize()
            row[tile] = s.elapsed_time(e) * 1000 / n
        os.environ.pop("OME_MOE_FP8_TILE")
        auto = ops.moe_fp8_tile_m(T * k, E)
        tfl = 2 * T * k * 3 * H * I / 1e12
        print(f"T={T:5d} rows/expert={T * k / E:6.1f}  tile64 {row['64']:8.1f} us  tile128 {row['128']:8.1f} us  "
              f"128/64 {row['128'] / row['64']:4.2f}  auto={auto}  best {tfl / min(row.values()) * 1e6:6.1f} TF/s  "
              f"weights {wbytes / 1e9:.1f} GB -> {wbytes / min(row.values()) / 1e6:5.2f} TB/s-equiv", flush=True)


if __name__ == "__main__":
    main()
