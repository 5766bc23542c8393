#!/usr/bin/env python3
"""Decode-GEMM (M <= 256) variants of the stream-K kernel, one variant per process
(OME_SK_VARIANT: 0 = shipped table plan, 1 = 128 x 128 tiles at two workgroups per CU, 2 = nt
weight stream, 3 = both).  Cold weights (> 600 MiB of copies), checked against fp32 first."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.ops._native import call, stream_ptr  # noqa: E402

DEV = torch.device("cuda")
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
VAR = int(os.environ.get("OME_SK_VARIANT", "0"))


def bench(fn, n_w, iters=40):
    for i in range(4):
        fn(i % n_w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def sk(x, w, out, epi, bm, bn, nwg):
    ws, cnt = ops._sk_workspace(x.device)
    M, K = x.shape
    call("ome_gemm_sk", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), None, out.data_ptr(), out.stride(0), M,
         w.shape[0], K, bm, bn, epi, nwg, ws.data_ptr(), cnt.data_ptr(), stream_ptr())
    return out


def main():
    total = {}
    for name, (N, K) in SHAPES.items():
        epi = 2 if name == "gate_up" else 0
        n_w = max(2, -(-(600 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_w)]
        wi = [ops.interleave_gate_up(w) for w in ws] if epi == 2 else ws
        for M in (128, 256):
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            ref = F.linear(x.float(), ws[0].float())
            if epi == 2:
                ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            out = torch.empty(M, N // 2 if epi else N, device=DEV, dtype=torch.bfloat16)
            plan = ops.gemm_sk_plan(M, N, K, epi)
            row = [f"var{VAR} M={M} {name:8s}"]
            if VAR == 0:
                bn, nwg, bm = plan or (128, 192, 128)
                cands = [(bm, bn, nwg)]
            else:
                T = -(-M // 128) * (N // 128)
                cands = sorted({(128, 128, n) for n in (192, 256, 320, 384, 448, 512) if n % 8 == 0} |
                               {(128, 128, min(512, T - T % 8))})
            best = None
            for bm, bn, nwg in cands:
                y = sk(x, wi[0], out, epi, bm, bn, nwg)
                torch.cuda.synchronize()
                err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                if not err < 2e-2:
                    row.append(f"{bm}x{bn}/w{nwg} ERR {err:.3g}")
                    continue
                t = bench(lambda i: sk(x, wi[i], out, epi, bm, bn, nwg), n_w)
                row.append(f"{bm}x{bn}/w{nwg} {t:6.1f}")
                if best is None or t < best:
                    best = t
            row.append(f"BEST {best:6.1f}us {N * K * 2 / best / 1e6:5.2f}TB/s")
            total[M] = total.get(M, 0.0) + best
            print("  ".join(row), flush=True)
        del ws, wi
        torch.cuda.empty_cache()
    print(f"var{VAR} per-layer sum: " + "  ".join(f"M={m}: {t:.1f}us" for m, t in total.items()), flush=True)


if __name__ == "__main__":
    main()
