#!/usr/bin/env python3
"""ome_gemm_xl (csrc/kernels/gemm_xl.hip) vs hipBLASLt (F.linear) and the stream-K kernel's table
plan on the Llama-3-8B projections, plus the skeleton probes.

Cold weights as in scripts/gemm_sk_bench.py (every call uses the next of several weight copies,
> 600 MiB in total); gate_up is timed as the serving path runs it (hipBLASLt + act_and_mul vs the
fused SiLU epilogue).  Every configuration is checked against an fp32 reference before it is timed.
--table PATH writes the measured best per (shape, M) for ``ops.gemm_xl_plan``.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "qkv70": (10240, 8192), "o70": (8192, 8192), "gate_up70": (57344, 8192), "down70": (8192, 28672)}
DEV = torch.device("cuda")


def bench(fn, n_w, iters=30):
    for i in range(4):
        fn(i % n_w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def nwg_cands(M, N, bn):
    T = ops.gemm_sk_tiles(M, N, bn, 256)
    c = {256, 248, 240, 224, 192}
    for k in (1, 2, 3, 4):
        if T % k == 0 and (T // k) % 8 == 0 and T // k <= 256:
            c.add(T // k)
    return sorted((x for x in c if 8 <= x <= 256), reverse=True)


def probes(sizes):
    for S in sizes:
        x = torch.rand(S, S, device=DEV, dtype=torch.bfloat16) * 2 - 1
        w = torch.rand(S, S, device=DEV, dtype=torch.bfloat16) * 2 - 1
        out = torch.empty(S, S, device=DEV, dtype=torch.bfloat16)
        fl = 2 * S ** 3
        t_lib = bench(lambda i: F.linear(x, w), 1, 20)
        row = [f"S={S} hipblaslt {t_lib:7.1f}us {fl / t_lib / 1e6:5.0f}TF"]
        for bn in (256, 128):
            T = ops.gemm_sk_tiles(S, S, bn, 256)
            nwg = 256 if T >= 256 else T
            for pr in ((4, 1, 2) if bn == 256 else (5, 4, 1, 2)):
                t = bench(lambda i: ops.gemm_xl(x, w, out=out, bn=bn, nwg=nwg, probe=pr), 1, 20)
                row.append(f"bn{bn} p{pr} {t:7.1f}us {fl / t / 1e6:5.0f}TF")
        print("  ".join(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="256,512,768,1024,1280,1536,2048,2304")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--probe", default="4096,8192", help="square sizes for the skeleton probes ('' = none)")
    ap.add_argument("--table", default=None)
    ap.add_argument("--stg", default="3,4", help="3 = register staging, 4 = LDS-DMA body")
    a = ap.parse_args()
    a.stg = [int(v) for v in a.stg.split(",")]
    if a.probe:
        probes([int(v) for v in a.probe.split(",")])
    ms = [int(v) for v in a.m.split(",")]
    plan = {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        epi = 2 if name.startswith("gate_up") else 0
        n_w = max(2, -(-(600 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_w)]
        wi = [ops.interleave_gate_up(w) for w in ws] if epi == 2 else ws
        for M in ms:
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            ref = F.linear(x.float(), ws[0].float())
            if epi == 2:
                ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            fl = 2 * M * N * K
            if epi == 2:
                t_lib = bench(lambda i: ops.act_and_mul(F.linear(x, wi[i]), interleaved=True), n_w, a.iters)
            else:
                t_lib = bench(lambda i: F.linear(x, ws[i]), n_w, a.iters)
            row = [f"M={M:5d} {name:8s} lib {t_lib:7.1f}us {fl / t_lib / 1e6:5.0f}TF"]
            sk = ops.gemm_sk_plan(M, N, K, epi)
            out = torch.empty(M, N // 2 if epi else N, device=DEV, dtype=torch.bfloat16)
            if sk:
                bn_s, nwg_s, bm_s = sk
                t_sk = bench(lambda i: ops.gemm_sk(x, wi[i], out=out, epi=epi, bn=bn_s, nwg=nwg_s, bm=bm_s), n_w,
                             a.iters)
                row.append(f"sk {t_sk:6.1f}")
            res = []
            for bn in (256, 128):
                for nwg in nwg_cands(M, N, bn):
                    if not ops.gemm_xl_ok(M, N, K, bn, nwg):
                        continue
                    for stg in a.stg:
                        if stg == 5 and bn != 128:
                            continue
                        out.zero_()
                        y = ops.gemm_xl(x, wi[0], out=out, epi=epi, bn=bn, nwg=nwg, probe=stg)
                        torch.cuda.synchronize()
                        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                        if not err < 2e-2:
                            row.append(f"xl{bn}/w{nwg}/s{stg} ERR {err:.3g}")
                            continue
                        t = bench(lambda i: ops.gemm_xl(x, wi[i], out=out, epi=epi, bn=bn, nwg=nwg, probe=stg), n_w,
                                  a.iters)
                        res.append((t, bn, nwg, stg))
            res.sort()
            row.append(" ".join(f"xl{b}/w{n}/s{g} {t:6.1f}" for t, b, n, g in res[:4]))
            if res:
                t, bn, nwg, _ = res[0]
                row.append(f"BEST {t:6.1f}us {fl / t / 1e6:5.0f}TF x{t_lib / t:.2f}")
                plan.setdefault(f"{N},{K},{epi}", {})[str(M)] = {"bn": bn, "nwg": nwg, "us": round(t, 1),
                                                                 "lib_us": round(t_lib, 1)}
            print("  ".join(row), flush=True)
        del ws, wi
        torch.cuda.empty_cache()
    if a.table:
        with open(a.table, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(), "method": "scripts/gemm_xl_bench.py, cold weights",
                       "shapes": plan}, f, indent=1)


if __name__ == "__main__":
    main()
