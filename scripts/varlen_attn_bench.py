"""Varlen bidirectional attention (``ome_varlen_attention``) vs torch SDPA on the same packed
batches: BERT-large embedding batch, Qwen2-VL ViT images (head dim 80), long single sequences.
Prints per-shape time, TFLOP/s and the max error against SDPA.  Random bf16 operands."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def sdpa(q, k, v, lens, scale):
    outs, s = [], 0
    for n in lens:
        outs.append(F.scaled_dot_product_attention(*(t[s:s + n].transpose(0, 1)[None] for t in (q, k, v)),
                                                   scale=scale)[0].transpose(0, 1))
        s += n
    return torch.cat(outs)


CASES = [("bert-large b32x512", [512] * 32, 16, 64), ("bert mixed lens", [37, 512, 128, 300, 9, 480] * 8, 16, 64),
         ("vit 4 images 1024p D80", [1024] * 4, 16, 80), ("vit 1 image 4096p D80", [4096], 16, 80),
         ("long 8k D128", [8192], 32, 128), ("qwen-image joint 2x4200 D128", [4200, 4200], 24, 128)]
for name, lens, H, D in CASES:
    T = sum(lens)
    torch.manual_seed(0)
    q, k, v = (torch.randn(T, H, D, device="cuda").bfloat16() for _ in range(3))
    sc = D ** -0.5
    ours = ops.varlen_attention(q, k, v, lens, sc)
    err = (ours.float() - sdpa(q, k, v, lens, sc).float()).abs().max().item()
    t_ours = bench(lambda: ops.varlen_attention(q, k, v, lens, sc))
    t_sdpa = bench(lambda: sdpa(q, k, v, lens, sc))
    flop = sum(4 * n * n * D * H for n in lens)
    print(f"{name:26s} ours {t_ours:9.1f} us {flop / t_ours / 1e6:7.1f} TF | sdpa {t_sdpa:9.1f} us "
          f"{flop / t_sdpa / 1e6:7.1f} TF | speedup {t_sdpa / t_ours:5.2f}x | max err {err:.2e}", flush=True)
